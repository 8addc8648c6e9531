#!/usr/bin/env python3
"""DRAM access-pattern probe for the outer-UDP kernels (NOT product code):
1,024 x 128 pieces of 1452 B read (or written) by 16-lane rows, pieces 64 KiB
apart (the Go message buffers udp_coalesce reads / udp_split writes) vs packed
1456 B apart; one stream and two alternating; HIP events over K launches, two
rotated buffer sets.  usage: python scripts/probe_strided.py [K]"""
import ctypes
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
so = "/tmp/probe_strided.so"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(ROOT, "scripts", "probe_strided.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_strided_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_void_p]
K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
npieces, piece = 1024 * 128, 1452
big = [torch.zeros(npieces * 65536, dtype=torch.uint8, device="cuda") for _ in range(2)]  # 2 x 8.6 GB
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
nbytes = npieces * piece


def timed(stride, write, ns):
    def go(k):
        rc = L.probe_strided_launch(big[k % 2].data_ptr() + (k // 2 % 2) * (npieces * 1456 if stride < 65536 else 0),
                                    stride, npieces, piece, write, sink.data_ptr(), streams[k % ns].cuda_stream)
        assert rc == 0
    for k in range(6):
        go(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    streams[1].wait_event(e0)
    for k in range(K):
        go(k)
    j = torch.cuda.Event()
    j.record(streams[1])
    streams[0].wait_event(j)
    e1.record(streams[0])
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


for rd in range(2):
    for write in (0, 1):
        for stride in (65536, 1456):
            for ns in (1, 2):
                us = timed(stride, write, ns)
                print(json.dumps({"round": rd, "op": "write" if write else "read", "stride": stride, "streams": ns,
                                  "us": round(us, 2), "TBps": round(nbytes / us / 1e6, 3),
                                  "frac": round(nbytes / us / 1e6 / 8.0, 3)}), flush=True)
