"""Interleaved A/B of checksum-kernel launch variants in ONE process
(cdna_hip_programming.md §5.4 rule 24).  GPU only.
usage: python scripts/sweep_checksum.py [--config cfg2] [--rounds 5] [--iters 100]"""
import argparse, os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # first: one HIP runtime per process
from wireguard_amd import synth
from wireguard_amd.tun import Device, MODE_VALIDATE, MODE_L4_FILL

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--variants", default="16:6:4:0,16:6:4:1,16:6:8:1,16:4:8:1,16:8:8:1,64:4:8:1")
ap.add_argument("--mode", default="validate")
a = ap.parse_args()
n, flen, kinds = {"cfg2": (65536, 1500, "tcp4"), "cfg3": (65536, 9000, "tcp4"), "cfg5": (131072, 1500, "mixed")}[a.config]
mode = MODE_VALIDATE if a.mode == "validate" else MODE_L4_FILL
arena_np, pkts_np, _ = synth.make_batch(n, flen, kinds=kinds)
R = 4
arenas = [torch.from_numpy(arena_np).cuda() for _ in range(R)]
pkts = torch.from_numpy(pkts_np.view(np.uint8)).cuda()
out = torch.empty(n * 2, dtype=torch.uint8, device="cuda")
nbytes = int(pkts_np["len"].astype(np.int64).sum())
stream = torch.cuda.Stream()
devs = {}
for v in a.variants.split(","):
    f = v.split(":")
    g, u, b, nt = f[:4]
    os.environ["WGCS_LANES_PER_PKT"], os.environ["WGCS_UNROLL"], os.environ["WGCS_BLOCKS_PER_CU"] = g, u, b
    os.environ["WGCS_NT"] = nt
    os.environ["WGCS_ALIGN"] = f[4] if len(f) > 4 else "16"
    os.environ["WGCS_FLAT"] = f[5] if len(f) > 5 else "0"
    devs[v] = Device(0)
res = {v: [] for v in devs}
for r in range(a.rounds):
    for v, d in devs.items():
        for k in range(10):
            d.checksum_batch(mode, arenas[k % R], pkts, n, out, stream=stream)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for k in range(a.iters):
            d.checksum_batch(mode, arenas[k % R], pkts, n, out, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        res[v].append(us)
        if mode == MODE_VALIDATE:
            assert bool(out[:n].all().item()), v
for v, t in res.items():
    t = np.array(t)
    print(json.dumps({"variant(G:U:BPC:NT[:ALIGN[:FLAT]])": v, "config": a.config, "median_us": round(float(np.median(t)), 2),
                      "min_us": round(float(t.min()), 2), "GBps": round(nbytes / np.median(t) / 1e3, 1),
                      "frac_8TBs": round(nbytes / np.median(t) / 1e3 / 8000, 3)}))
