#!/usr/bin/env python3
"""Phase timeline of gro_batch_kernel (timing-only build with -DWGCS_P_STAMPS,
a switch that existed only in the experimental revision this was run against:
thread 0 wrote s_memtime at each phase boundary into to_write[first+100+k],
which the cfg's 128-packet calls never use; output in
profiles/r2_probe_gro_stamps.jsonl).  Prints, over all calls of one
launch, the median cycles per phase.  Build: python scripts/probe_gro_stamps.py build"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "scripts", "probe_so", "libwgcsum_stamps.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    from wireguard_amd import build as B

    os.makedirs(os.path.dirname(SO), exist_ok=True)
    print(B.build(out=SO, extra=["-DWGCS_P_STAMPS"]))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import _lib, gro_bench  # noqa: E402
from wireguard_amd.tun import GRO_BUF_DTYPE, GRO_CALL_DTYPE, GRO_CAN_UDP, Device  # noqa: E402

_lib.LIB_PATH = SO
torch.cuda.set_device(0)
dev = Device(0)
pkts = gro_bench.make_batch(dev)
n = len(pkts)
for calls in (256, 1280):
    N = calls * n
    stride = 65552
    arena = torch.empty(N * stride, dtype=torch.uint8, device="cuda")
    W = 1536
    img = np.zeros((n, W), np.uint8)
    for i, p in enumerate(pkts):
        img[i, 16: 16 + len(p)] = np.frombuffer(p, np.uint8)
    arena.view(N, stride)[:, :W].copy_(torch.from_numpy(np.tile(img, (calls, 1))).cuda())
    gb = np.zeros(N, GRO_BUF_DTYPE)
    gb["off"] = np.arange(N, dtype=np.uint64) * np.uint64(stride)
    gb["len"] = np.tile(np.array([16 + len(p) for p in pkts], np.uint32), calls)
    gb["cap"] = 65551
    gc = np.zeros(calls, GRO_CALL_DTYPE)
    gc["first"] = np.arange(calls, dtype=np.uint32) * n
    gc["n"] = n
    gc["offset"] = 16
    gc["flags"] = GRO_CAN_UDP
    st = torch.zeros(calls, dtype=torch.int32, device="cuda")
    nw = torch.zeros(calls, dtype=torch.int32, device="cuda")
    tw = torch.zeros(N, dtype=torch.int32, device="cuda")
    d_bufs = torch.from_numpy(gb.view(np.uint8)).cuda()
    dev.handle_gro_batch(arena, d_bufs, torch.from_numpy(gc.view(np.uint8)).cuda(), calls, st, nw, tw)
    torch.cuda.synchronize()
    s = tw.cpu().numpy().view(np.uint32).reshape(calls, n)[:, 100:107].astype(np.int64)
    d = np.diff(s, axis=1) % (1 << 32)
    names = ["init", "headers+fields", "flow ids+checksums", "planner", "toWrite+finish", "apply"]
    print(json.dumps({"calls": calls, "cycles_median": {k: int(np.median(d[:, i])) for i, k in enumerate(names)},
                      "total_median": int(np.median(d.sum(1)))}), flush=True)
    del arena
