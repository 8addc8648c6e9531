#!/usr/bin/env python3
"""Interleaved A/B of gro_batch_kernel builds on the gro_device workload
(timing-only -D switches of the experimental revision they were run
against; the committed kernel has neither switch -- the flow-link variant was
slower and reverted, see DESIGN.md, profiles/r2_probe_gro_flow_links.jsonl).
build: python scripts/probe_gro_variants.py build; run: python
scripts/probe_gro_variants.py [rounds].  Prints us per launch (HIP events,
one explicit stream) per variant."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUTDIR = os.path.join(ROOT, "scripts", "probe_so")
VARIANTS = {"fnext_links": [], "scan_all": ["WGCS_P_OLDSCAN"]}

if len(sys.argv) > 1 and sys.argv[1] == "build":
    from wireguard_amd import build as B

    os.makedirs(OUTDIR, exist_ok=True)
    for k, d in VARIANTS.items():
        print(B.build(out=os.path.join(OUTDIR, f"libwgcsum_gro_{k}.so"), extra=[f"-D{x}" for x in d]))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import _lib, gro_bench  # noqa: E402
from wireguard_amd.tun import GRO_BUF_DTYPE, GRO_CALL_DTYPE, GRO_CAN_UDP, Device  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
torch.cuda.set_device(0)
devs = {}
for k in VARIANTS:
    _lib._lib = None
    _lib.LIB_PATH = os.path.join(OUTDIR, f"libwgcsum_gro_{k}.so")
    devs[k] = Device(0)
pkts = gro_bench.make_batch(next(iter(devs.values())))
n, calls, stride, W = len(pkts), 1280, 65552, 1536
N = calls * n
img = np.zeros((n, W), np.uint8)
for i, p in enumerate(pkts):
    img[i, 16: 16 + len(p)] = np.frombuffer(p, np.uint8)
d_img = torch.from_numpy(np.tile(img, (calls, 1))).cuda()
gb = np.zeros(N, GRO_BUF_DTYPE)
gb["off"] = np.arange(N, dtype=np.uint64) * np.uint64(stride)
gb["len"] = np.tile(np.array([16 + len(p) for p in pkts], np.uint32), calls)
gb["cap"] = 65551
gc = np.zeros(calls, GRO_CALL_DTYPE)
gc["first"] = np.arange(calls, dtype=np.uint32) * n
gc["n"] = n
gc["offset"] = 16
gc["flags"] = GRO_CAN_UDP
d_bufs0 = torch.from_numpy(gb.view(np.uint8)).cuda()
d_calls = torch.from_numpy(gc.view(np.uint8)).cuda()
R = 3
arenas = [torch.empty(N * stride, dtype=torch.uint8, device="cuda") for _ in range(R)]
bufs = [d_bufs0.clone() for _ in range(R)]
st = torch.zeros(calls, dtype=torch.int32, device="cuda")
nw = torch.zeros(calls, dtype=torch.int32, device="cuda")
tw = torch.zeros(N, dtype=torch.int32, device="cuda")
res = {k: [] for k in VARIANTS}
qs = torch.cuda.Stream()
for rd in range(rounds + 1):
    for k, dev in devs.items():
        for r in range(R):
            arenas[r].view(N, stride)[:, :W].copy_(d_img)
            bufs[r].copy_(d_bufs0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(qs)
        for r in range(R):
            dev.handle_gro_batch(arenas[r], bufs[r], d_calls, calls, st, nw, tw, stream=qs)
        e1.record(qs)
        torch.cuda.synchronize()
        assert bool((nw == 4).all())
        if rd:
            res[k].append(e0.elapsed_time(e1) * 1e3 / R)
for k, v in res.items():
    print(json.dumps({"variant": k, "defines": VARIANTS[k], "us_med": round(statistics.median(v), 2),
                      "us_min": round(min(v), 2), "packets_per_s_M": round(N / statistics.median(v), 1)}))
