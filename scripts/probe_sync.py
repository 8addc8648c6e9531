#!/usr/bin/env python3
"""Where do the ~17-20 us of wall - event span in bench.py's timed region go? (round 3)

Not product code.  The cfg2 region (K launches of the VALIDATE kernel over
rotated copies, one wgcs_checksum_batches call, 2 streams) with host
timestamps around each phase:
  t_enq   the enqueue call returned
  t_e0    e0 (recorded before the first launch) observed complete by a query spin
  t_e1    e1 (after the last launch and the joins) observed complete
  t_sync  torch.cuda.synchronize() returned (after t_e1: nothing left to wait for)
and two empty brackets: sync() alone, and one tiny launch + sync().
Variants: "spin" (query-spin on e0 then e1, then sync), "sync" (the bench's
own: sync right after the enqueue).
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import Device, MODE_VALIDATE  # noqa: E402


def med(x):
    return round(statistics.median(x), 1)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    torch.cuda.set_device(0)
    dev = Device(0)
    arena_np, pkts_np, _ = synth.make_batch(65536, 1500, kinds="tcp4")
    n = len(pkts_np)
    R = 4
    arenas = [torch.from_numpy(arena_np).to("cuda") for _ in range(R)]
    pkts = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
    outs = [torch.empty(n * 2, dtype=torch.uint8, device="cuda") for _ in range(R)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    e1.record(streams[0])
    tiny = dev.batch_list([(arenas[0], pkts, 64, outs[0])])

    def bl(k0):
        return dev.batch_list([(arenas[(k0 + k) % R], pkts, n, outs[(k0 + k) % R]) for k in range(K)])

    def region(var, k0):
        b = bl(k0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.checksum_batches(MODE_VALIDATE, b, streams, e0, e1)
        t_enq = time.perf_counter()
        t_e0 = t_e1 = float("nan")
        if var == "spin":
            while not e0.query():
                pass
            t_e0 = time.perf_counter()
            while not e1.query():
                pass
            t_e1 = time.perf_counter()
        torch.cuda.synchronize()
        t_sync = time.perf_counter()
        span = e0.elapsed_time(e1) * 1e3
        us = lambda t: (t - t0) * 1e6  # noqa: E731
        return {"wall": us(t_sync), "span": span, "enq": us(t_enq), "e0_seen": us(t_e0), "e1_seen": us(t_e1),
                "sync_after_e1": (t_sync - t_e1) * 1e6, "wall_minus_span": us(t_sync) - span}

    def empty_sync():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    def tiny_launch():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.checksum_batches(MODE_VALIDATE, tiny, streams[:1])
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6

    for v in ("sync", "spin"):
        region(v, 0)
        region(v, K)
    res = {"sync": [], "spin": []}
    es, tl = [], []
    for t in range(trials):
        for v in (("sync", "spin") if t % 2 == 0 else ("spin", "sync")):
            res[v].append(region(v, t * K))
        es.append(empty_sync())
        tl.append(tiny_launch())
    for v, rs in res.items():
        out = {"probe": "sync", "variant": v, "K": K, "trials": trials}
        for key in rs[0]:
            vals = [r[key] for r in rs]
            if not any(x != x for x in vals):
                out[key + "_us_med"] = med(vals)
        print(json.dumps(out), flush=True)
    print(json.dumps({"probe": "sync", "variant": "empty_sync", "us_med": med(es), "us_min": round(min(es), 1)}))
    print(json.dumps({"probe": "sync", "variant": "tiny_launch_sync", "us_med": med(tl), "us_min": round(min(tl), 1)}))
    dev.close()


if __name__ == "__main__":
    main()
