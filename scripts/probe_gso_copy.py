#!/usr/bin/env python3
"""cfg4's access-pattern ceiling (NOT product code): the
product's gso_lds_kernel and scripts/probe_gso_copy.hip (the same in -> out
byte mapping as 16-byte row copies and nothing else) on the bench's batch --
256 reads of 65,545 B at 128-byte multiples, 45 segments each into 128 slots of
1,536 B with bufs[i][16] on a 128-byte line (the bench's --gso-in-align /
--gso-out-align defaults), 8 rotated copies -- K launches on one stream and on four, HIP events, the
same algorithmic bytes (bytes read + bytes written).  One JSON line per
(kernel, streams); the copy's output is checked once against the product's
segments (the bytes it moves must be the ones the product writes, headers
aside: the probe does not rewrite them)."""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import torch  # first: one HIP runtime per process

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import GSO_JOB_DTYPE, Device  # noqa: E402

so = "/tmp/probe_gso_copy.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(ROOT, "scripts", "probe_gso_copy.hip")], check=True)
P = C.CDLL(so)
P.probe_gso_copy.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                             C.c_uint32, C.c_void_p]
dev = Device(0)
K = int(os.environ.get("K", "200"))
n_jobs, total, gso, max_segs, stride, offset, R = 256, 65535, 1460, 128, 1536, 16, 8
pkts = [synth.make_super_packet(total, gso, seed=synth.SEED + k) for k in range(n_jobs)]
jlen = len(pkts[0])
jpitch = -(-jlen // 128) * 128
oshift = (128 - offset % 128) % 128
arena = np.zeros(n_jobs * jpitch + 64, np.uint8)
for k, p in enumerate(pkts):
    arena[k * jpitch: k * jpitch + jlen] = np.frombuffer(p, np.uint8)
jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(jpitch)
jobs["len"] = jlen
d_arena = [torch.from_numpy(arena).cuda() for _ in range(R)]
d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
d_out = [torch.zeros(n_jobs * max_segs * stride + 256, dtype=torch.uint8, device="cuda")[oshift:] for _ in range(R)]
sts = [torch.cuda.Stream() for _ in range(4)]
d_sizes = [torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda") for _ in range(4)]
d_count = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(4)]
d_status = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(4)]


def product(k, q):
    dev.gso_split_batch(d_arena[k % R], d_jobs, n_jobs, d_out[k % R], stride, offset, max_segs, d_sizes[q],
                        d_count[q], d_status[q], stream=sts[q])


def copy(k, q):
    rc = P.probe_gso_copy(d_arena[k % R].data_ptr(), jpitch, jlen, n_jobs, d_out[k % R].data_ptr(), stride, offset,
                          max_segs, sts[q].cuda_stream)
    assert rc == 0, rc


# bytes: as gso_bench (bytes_in + bytes_out from the product's sizes)
product(0, 0)
torch.cuda.synchronize()
sizes = d_sizes[0].cpu().numpy().reshape(n_jobs, max_segs)
assert (d_count[0].cpu().numpy() == 45).all() and (d_status[0].cpu().numpy() == 0).all()
nbytes = int(sizes.astype(np.int64).sum()) + n_jobs * jlen
# the probe's payload bytes are the product's (segments 0..44 past the 40-byte header)
ref = d_out[0].cpu().numpy().copy()
d_out[0].zero_()
copy(0, 0)
torch.cuda.synchronize()
got = d_out[0].cpu().numpy()
for j in (0, 77, 255):
    for i in (0, 1, 44):
        b = (j * max_segs + i) * stride + offset
        n = int(sizes[j, i])
        assert np.array_equal(got[b + 40: b + n], ref[b + 40: b + n]), (j, i)


def timed(fn, ns):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k in range(10):
        fn(k, k % ns)
    torch.cuda.synchronize()
    e0.record(sts[0])
    for s in sts[1:ns]:
        s.wait_event(e0)
    for k in range(K):
        fn(k, k % ns)
    for s in sts[1:ns]:
        j = torch.cuda.Event()
        j.record(s)
        sts[0].wait_event(j)
    e1.record(sts[0])
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


for rep in range(2):
    for name, fn in (("gso_lds_kernel (product)", product), ("copy probe", copy)):
        for ns in (1, 4):
            us = timed(fn, ns)
            print(json.dumps({"probe": "gso_copy_ceiling", "kernel": name, "streams": ns, "launches": K, "rep": rep,
                              "us_per_launch": round(us, 3), "algorithmic_bytes": nbytes,
                              "frac_of_8TBs": round(nbytes / (us * 1e-6) / 8e12, 4)}), flush=True)
dev.close()
