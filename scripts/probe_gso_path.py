#!/usr/bin/env python3
"""Bisection probe of the cfg4 GSO split (NOT product code): timing of
scripts/probe_gso_path.hip feature variants on the cfg4 layout (256 x 65,535-B
jobs, 45 segments each, 128 x 1536-B output slots per job), next to the product
kernel (wgcs_gso_split_batch) and torch's copy of the same bytes, one stream
and two streams alternating; HIP events over K launches, rotated copies.
usage: python scripts/probe_gso_path.py [K] [rounds]"""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import GSO_JOB_DTYPE, Device  # noqa: E402

so = "/tmp/probe_gso_path.so"
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                f"-I{ROOT}/include", "-o", so, os.path.join(ROOT, "scripts", "probe_gso_path.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_gso_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32] * 4 + [ctypes.c_void_p, ctypes.c_int,
                                                                               ctypes.c_void_p]
K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n_jobs, max_segs, stride, doff = 256, 128, 1536, 16
pk = [synth.make_super_packet(65535, 1460, seed=synth.SEED + k) for k in range(n_jobs)]
arena_np = np.frombuffer(b"".join(pk) + bytes(64), np.uint8).copy()
jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(65535)
jobs["len"] = 65535
R = 8
arenas = [torch.from_numpy(arena_np).cuda() for _ in range(R)]
d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
outs = [torch.empty(n_jobs * max_segs * stride, dtype=torch.uint8, device="cuda") for _ in range(R)]
sums = torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda")
sizes = [torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda") for _ in range(2)]
cnt = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(2)]
stt = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(2)]
dev = Device(0)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
nbytes = 65535 * n_jobs + (44 * 1500 + 1325) * n_jobs


def variant(name):
    def go(k, q):
        i = k % R
        st = streams[q]
        if name == "product":
            dev.gso_split_batch(arenas[i], d_jobs, n_jobs, outs[i], stride, doff, max_segs, sizes[q], cnt[q], stt[q],
                                stream=st)
        elif name == "torch_copy":
            with torch.cuda.stream(st):
                outs[i][: 65535 * n_jobs].copy_(arenas[i][: 65535 * n_jobs])
        else:
            rc = L.probe_gso_launch(arenas[i].data_ptr(), d_jobs.data_ptr(), outs[i].data_ptr(), n_jobs, max_segs,
                                    stride, doff, sums.data_ptr(), int(name), st.cuda_stream)
            assert rc == 0, rc
    return go


def timed(go, ns):
    for k in range(10):
        go(k, k % ns)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    streams[1].wait_event(e0)
    for k in range(K):
        go(k, k % ns)
    j = torch.cuda.Event()
    j.record(streams[1])
    streams[0].wait_event(j)
    e1.record(streams[0])
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


names = ["torch_copy", "0", "1", "3", "7", "15", "product"]
desc = {"torch_copy": "torch copy of the 16.8 MB input", "0": "bare row copy, aligned slots, constants",
        "16": "bare row copy (F_BUF unused)", "1": "+ doff 16 (byte-exact head/tail)", "3": "+ header chunks",
        "7": "+ dependent job/virtio loads", "15": "+ sums (all features)", "product": "wgcs_gso_split_batch"}
for rd in range(ROUNDS):
    for nm in names:
        go = variant(nm)
        t1 = timed(go, 1)
        t2 = timed(go, 2)
        print(json.dumps({"round": rd, "variant": nm, "what": desc[nm], "us_1stream": round(t1, 2),
                          "us_2streams": round(t2, 2), "frac_2streams": round(nbytes / (t2 * 1e-6) / 8e12, 3)}),
              flush=True)
dev.close()
