#!/usr/bin/env python3
"""udp_coalesce timing-only variants (NOT product code): each library in
scripts/probe_so is loaded directly with ctypes (its own wgcs context) and
times wgcs_coalesce_messages_batch on the bench's shape (1,024 Send batches of
128 x 1452 B, 64-KiB buffers), one stream and two alternating, interleaved
over rounds.  Variants other than `ucbase` were built with timing-only -D
switches that existed only while this probe ran (WGCS_P_UC_FULLST: every
chunk one full store, edges overwritten; WGCS_P_UC_NOLOOP: the bench's runs of
45 packets as constants, no coalescing loop, no barrier); the outputs are in
profiles/r3_probe_ucoal.jsonl.
usage: python scripts/probe_ucoal.py ROUNDS lib.so..."""
import ctypes as C
import json
import os
import sys

import torch

ROUNDS = int(sys.argv[1])
libs = sys.argv[2:]
B, NB, MSG, STRIDE, K = 1024, 128, 1452, 65536, 50
bufs = [torch.zeros((B * NB, STRIDE), dtype=torch.uint8, device="cuda") for _ in range(2)]
for b in bufs:
    b[:, :MSG].random_(0, 255)
lens = torch.full((B * NB,), MSG, dtype=torch.int32, device="cuda")
nbs = torch.full((B,), NB, dtype=torch.int32, device="cuda")
outs = [[torch.zeros(B * NB, dtype=torch.int32, device="cuda") for _ in range(4)] for _ in range(2)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
nbytes = 2 * B * (NB - 3) * MSG
ctxs = []
for path in libs:
    L = C.CDLL(path)
    L.wgcs_init.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.wgcs_coalesce_messages_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p,
                                               C.c_void_p, C.c_uint32, C.c_uint32, C.c_int] + [C.c_void_p] * 5
    h = C.c_void_p()
    assert L.wgcs_init(0, C.byref(h)) == 0
    ctxs.append((os.path.basename(path), L, h))


def timed(L, h, ns):
    def go(k):
        q = k % ns
        o = outs[q]
        rc = L.wgcs_coalesce_messages_batch(h, bufs[k % 2].data_ptr(), STRIDE, 65535, None, lens.data_ptr(),
                                            nbs.data_ptr(), NB, B, 0, o[0].data_ptr(), o[1].data_ptr(),
                                            o[2].data_ptr(), o[3].data_ptr(), streams[q].cuda_stream)
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


for rd in range(ROUNDS):
    for name, L, h in ctxs:
        t1 = timed(L, h, 1)
        t2 = timed(L, h, 2)
        print(json.dumps({"round": rd, "lib": name, "us_1stream": round(t1, 2), "us_2streams": round(t2, 2),
                          "frac1": round(nbytes / t1 / 8e6, 3), "frac2": round(nbytes / t2 / 8e6, 3)}), flush=True)
