#!/usr/bin/env python3
"""One-stream GSO launch time over the life of a process (NOT product code):
HIP-event time per launch of cfg4 (gso_bench's layout: 256 x 65,535-B jobs,
128 x 1536-B slots, 8 rotated copies) in consecutive blocks of K launches,
then the same after a two-stream burst and after a CPU-side pause.  Does
the one-stream time depend on how long the GPU has been busy?"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import GSO_JOB_DTYPE, Device  # noqa: E402

torch.cuda.set_device(0)
dev = Device(0)
n_jobs, max_segs, stride, offset, R, K = 256, 128, 1536, 16, 8, 50
pk = [synth.make_super_packet(65535, 1460, seed=synth.SEED + k) for k in range(n_jobs)]
jlen = len(pk[0])
arena = np.frombuffer(b"".join(pk) + bytes(64), np.uint8).copy()
jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(jlen)
jobs["len"] = jlen
d_arena = [torch.from_numpy(arena).cuda() for _ in range(R)]
d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
d_out = [torch.empty(n_jobs * max_segs * stride, dtype=torch.uint8, device="cuda") for _ in range(R)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
sz = [torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda") for _ in range(2)]
ct = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(2)]
st = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(2)]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def block(ns, k0=0):
    torch.cuda.synchronize()
    e0.record(streams[0])
    if ns > 1:
        streams[1].wait_event(e0)
    for k in range(K):
        q = k % ns
        dev.gso_split_batch(d_arena[(k0 + k) % R], d_jobs, n_jobs, d_out[(k0 + k) % R], stride, offset, max_segs,
                            sz[q], ct[q], st[q], stream=streams[q])
    if ns > 1:
        j = torch.cuda.Event()
        j.record(streams[1])
        streams[0].wait_event(j)
    e1.record(streams[0])
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / K, 2)


t0 = time.perf_counter()
seq = [("1s", block(1)) for _ in range(6)]
seq += [("2s", block(2)) for _ in range(4)]
seq += [("1s", block(1)) for _ in range(4)]
time.sleep(0.5)
seq += [("1s after 0.5 s idle", block(1)) for _ in range(3)]
assert (ct[0].cpu().numpy() == 45).all()
print(json.dumps({"probe": "gso_warm", "K": K, "us_per_launch_in_order": seq,
                  "elapsed_s": round(time.perf_counter() - t0, 3)}))
dev.close()
