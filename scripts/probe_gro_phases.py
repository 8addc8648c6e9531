#!/usr/bin/env python3
"""Phase timeline of gro_batch_kernel per call shape (round 4; timing-only
build with -DWGCS_GRO_STAMPS: thread 0 of every call writes s_memrealtime
(100 MHz) at the phase boundaries into to_write[first+100..106), unused by
the bench's 128-buffer shapes).  Prints, per shape, the median µs of each
phase over the calls of one 1,792-call launch.
Build: python scripts/probe_gro_phases.py build"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.environ.get("WGCS_STAMPS_SO") or os.path.join(ROOT, "scripts", "probe_so", "libwgcsum_grostamps.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    from wireguard_amd import build as B

    os.makedirs(os.path.dirname(SO), exist_ok=True)
    print(B.build(out=SO, extra=["-DWGCS_GRO_STAMPS"]))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import _lib, gro_bench  # noqa: E402
from wireguard_amd.tun import GRO_BUF_DTYPE, GRO_CALL_DTYPE, GRO_CAN_UDP, Device  # noqa: E402

_lib.LIB_PATH = SO
torch.cuda.set_device(0)
dev = Device(0)
names = (["headers+checksums", "flow ids", "walk", "toWrite+finish", "apply"] if os.environ.get("R5_PHASES", "1") == "1"
         else ["headers+fields", "flow ids+checksums", "walk", "toWrite+finish", "apply"])  # round 5: step 1 reads each packet once
calls = 1792
for shape in gro_bench.CALL_SHAPES:
    pkts = gro_bench.shape_batch(dev, shape)
    n = len(pkts)
    N = calls * n
    stride = 65552
    arena = torch.empty(N * stride, dtype=torch.uint8, device="cuda")
    W = 1536
    img = np.zeros((n, W), np.uint8)
    for i, p in enumerate(pkts):
        img[i, 16: 16 + len(p)] = np.frombuffer(p, np.uint8)
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
    res = []
    for rep in range(3):
        arena.view(N, stride)[:, :W].copy_(torch.from_numpy(np.tile(img, (calls, 1))).cuda())
        d_bufs = torch.from_numpy(gb.view(np.uint8)).cuda()
        torch.cuda.synchronize()
        dev.handle_gro_batch(arena, d_bufs, torch.from_numpy(gc.view(np.uint8)).cuda(), calls, st, nw, tw)
        torch.cuda.synchronize()
        s = tw.cpu().numpy().view(np.uint32).reshape(calls, n)[:, 100:106].astype(np.int64)
        d = np.diff(s, axis=1) % (1 << 32)
        res.append([float(np.median(d[:, k])) / 100.0 for k in range(5)])  # 100 MHz ticks -> µs
        span = ((s[:, 5].max() - s[:, 0].min()) % (1 << 32)) / 100.0
    med = np.median(np.array(res), axis=0)
    print(json.dumps({"shape": shape, "writes_per_call": int(nw[0].item()), "median_us": dict(zip(names, [round(x, 2) for x in med])),
                      "call_us": round(float(med.sum()), 2), "launch_span_us": round(span, 1)}), flush=True)
    del arena
