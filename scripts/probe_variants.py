#!/usr/bin/env python3
"""Interleaved A/B of checksum-kernel launch variants on cfg2 (round 2).

Each variant is a Device created under its own WGCS_* tuning environment
(read at wgcs_init); rounds interleave the variants so box drift hits all
alike.  Per variant and round: the bench's bracket at K=20 (wall and HIP
events) and K=200 (events).  A "streams2" variant alternates consecutive
launches over two streams (independent batches may overlap).
usage: python scripts/probe_variants.py [rounds]
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ROC_ACTIVE_WAIT_TIMEOUT", "100000")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import Device, MODE_VALIDATE  # noqa: E402

VARIANTS = {
    "base": ({}, 1),
    "xcd": ({"WGCS_XCD": "1"}, 1),
    "bpc8": ({"WGCS_BLOCKS_PER_CU": "8"}, 1),
    "xcd_bpc8": ({"WGCS_XCD": "1", "WGCS_BLOCKS_PER_CU": "8"}, 1),
    "streams2": ({}, 2),
    "xcd_streams2": ({"WGCS_XCD": "1"}, 2),
}


def make_dev(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Device(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    torch.cuda.set_device(0)
    arena_np, pkts_np, _ = synth.make_batch(65536, 1500, kinds="tcp4")
    n = len(pkts_np)
    nbytes = int(pkts_np["len"].astype(np.int64).sum())
    R = 4
    arenas = [torch.from_numpy(arena_np).to("cuda") for _ in range(R)]
    pkts = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
    outs = [torch.empty(n * 2, dtype=torch.uint8, device="cuda") for _ in range(R)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    devs = {k: make_dev(env) for k, (env, _) in VARIANTS.items()}
    res = {k: {"wall20": [], "ev20": [], "ev200": []} for k in VARIANTS}

    def bracket(dev, ns, K, k0):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(streams[0])
        if ns == 2:
            streams[1].wait_event(e0)
        for k in range(K):
            i = (k0 + k) % R
            dev.checksum_batch(MODE_VALIDATE, arenas[i], pkts, n, outs[i], stream=streams[k % ns])
        if ns == 2:
            j = torch.cuda.Event()
            j.record(streams[1])
            streams[0].wait_event(j)
        e1.record(streams[0])
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return wall * 1e6 / K, e0.elapsed_time(e1) * 1e3 / K

    for k, (env, ns) in VARIANTS.items():  # warm
        bracket(devs[k], ns, 10, 0)
        assert bool(outs[0][:n].all().item())
    for r in range(rounds):
        for k, (env, ns) in VARIANTS.items():
            for t in range(3):
                w, e = bracket(devs[k], ns, 20, 5 + t)
                res[k]["wall20"].append(w)
                res[k]["ev20"].append(e)
            _, e = bracket(devs[k], ns, 200, 7)
            res[k]["ev200"].append(e)
    for k, v in res.items():
        out = {"variant": k, "env": VARIANTS[k][0], "streams": VARIANTS[k][1]}
        for m, xs in v.items():
            out[m + "_us_med"] = round(statistics.median(xs), 3)
            out[m + "_us_min"] = round(min(xs), 3)
        out["wall20_GiBps"] = round(nbytes / (out["wall20_us_med"] * 1e-6) / 2**30, 1)
        out["ev200_frac"] = round(nbytes / (out["ev200_us_med"] * 1e-6) / 8e12, 4)
        print(json.dumps(out), flush=True)
    for d in devs.values():
        d.close()


if __name__ == "__main__":
    main()
