#!/usr/bin/env python3
"""Phase timeline of gso_rows_kernel on cfg4 (NOT product code).

Timing-only build (-DWGCS_GSO_STAMPS): lane 0 of every wave of the clean path
writes s_memrealtime (100 MHz) at five points into unused sizes[] slots 64..123
of its job (max_segs 128, 45 segments per job):
  T0 wave start, T1 verdict + job sums done (the payload loads issue next),
  T2 payload stream done (loads consumed, stores issued), T3 header stored,
  T4 after s_waitcnt vmcnt(0) (the wave's stores acknowledged).
gso_lds_kernel (NWAVES=<its waves per job>): T0 start, T1 verdict + job sums,
T2 the LDS image landed (after vmcnt(0) + barrier), T3 every row's segments
streamed and stored, T4 stores acknowledged.
With -DWGCS_GSO_STAMPS=2 (run with STAMPS=2) the head of the wave instead:
  T0 start, T1 job descriptor arrived, T2 virtio header + header chunks
  arrived, T3 verdict + job sums done, T4 payload stream done.
Prints, per launch, the spread of each stamp over the launch's waves (us from
the launch's first wave start) beside the HIP-event time per launch, for the
last launch of a one-stream run and the last two launches of a two-stream run.
usage: probe_gso_stamps.py build | run
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.environ.get("STAMPS_SO") or os.path.join(ROOT, "scripts", "probe_so", "libwgcsum_gso_stamps.so")

if len(sys.argv) > 1 and sys.argv[1] == "build":
    from wireguard_amd import build as B

    os.makedirs(os.path.dirname(SO), exist_ok=True)
    print(B.build(out=SO, extra=["-DWGCS_GSO_STAMPS"] + sys.argv[2:]))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import _lib, synth  # noqa: E402
from wireguard_amd.tun import GSO_JOB_DTYPE, Device  # noqa: E402

_lib.LIB_PATH = os.environ.get("WGCS_LIB", SO)
torch.cuda.set_device(0)
dev = Device(0)
n_jobs, total, gso, max_segs, stride, offset = 256, 65535, 1460, 128, 1536, 16
pkts = [synth.make_super_packet(total, gso, seed=synth.SEED + k) for k in range(n_jobs)]
jlen = len(pkts[0])
# ALIGN=128 (default): bench.py cfg4's layout -- each read at a 128-B multiple
# of the arena, bufs[i][offset] on a 128-B line; ALIGN=0: packed, as allocated
ALIGN = int(os.environ.get("ALIGN", "128"))
jpitch = -(-jlen // ALIGN) * ALIGN if ALIGN else jlen
arena = np.zeros(n_jobs * jpitch + 64, np.uint8)
for k, p in enumerate(pkts):
    arena[k * jpitch: k * jpitch + jlen] = np.frombuffer(p, np.uint8)
jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(jpitch)
jobs["len"] = jlen
oshift = (ALIGN - offset % ALIGN) % ALIGN if ALIGN else 0
R = int(os.environ.get("PROBE_R", "8"))  # rotated arena / output copies
d_arena = [torch.from_numpy(arena).cuda() for _ in range(R)]
d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
d_out = [torch.empty(n_jobs * max_segs * stride + 256, dtype=torch.uint8, device="cuda")[oshift:] for _ in range(R)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
d_sizes = [torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda") for _ in range(2)]
d_count = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(2)]
d_status = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(2)]
e0 = torch.cuda.Event(enable_timing=True)
e1 = torch.cuda.Event(enable_timing=True)


def launch(k, q):
    dev.gso_split_batch(d_arena[k % R], d_jobs, n_jobs, d_out[k % R], stride, offset, max_segs, d_sizes[q],
                        d_count[q], d_status[q], stream=streams[q])


def run(K, ns, k0):
    torch.cuda.synchronize()
    e0.record(streams[0])
    if ns > 1:
        streams[1].wait_event(e0)
    for k in range(K):
        launch(k0 + k, k % ns)
    if ns > 1:
        j = torch.cuda.Event()
        j.record(streams[1])
        streams[0].wait_event(j)
    e1.record(streams[0])
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


NWAVES = int(os.environ.get("NWAVES", "12"))  # stamp-writing waves per job: 12 (rows kernel), NW (gso_lds_kernel)


def stamps(q):
    s = d_sizes[q].cpu().numpy().reshape(n_jobs, max_segs)[:, 64:64 + 5 * NWAVES].reshape(n_jobs, NWAVES, 5)
    s = s.astype(np.int64)
    return s.reshape(-1, 5) & 0xFFFFFFFF


def summary(st, base):
    us = (st - base) * 0.01  # 100 MHz ticks -> us
    out = {}
    names = (["T0_start", "T1_desc", "T2_hdr_loads", "T3_sums", "T4_stream_done"] if os.environ.get("STAMPS") == "2"
             else ["T0_start", "T1_verdict", "T2_image_landed", "T3_rows_done", "T4_stores_acked"]
             if os.environ.get("NWAVES") else ["T0_start", "T1_verdict", "T2_stream_done", "T3_hdr_done", "T4_stores_acked"])
    for k, name in enumerate(names):
        v = us[:, k]
        out[name] = [round(float(np.percentile(v, p)), 2) for p in (0, 10, 50, 90, 100)]
    for a in range(4):
        out[f"T{a + 1}-T{a}_med"] = round(float(np.median(us[:, a + 1] - us[:, a])), 2)
    return out


for k in range(12):
    launch(k, 0)
ev1 = run(20, 1, 100)
st = stamps(0)
print(json.dumps({"probe": "gso_stamps", "streams": 1, "event_us_per_launch": round(ev1, 2),
                  "percentiles": [0, 10, 50, 90, 100], **summary(st, st[:, 0].min())}), flush=True)
run(20, 2, 150)  # the first two-stream region of a process pays a one-off cross-stream cost
ev2 = run(20, 2, 200)
sa, sb = stamps(0), stamps(1)  # last launch on each stream: launches 18 (A) and 19 (B)
base = min(sa[:, 0].min(), sb[:, 0].min())
print(json.dumps({"probe": "gso_stamps", "streams": 2, "event_us_per_launch": round(ev2, 2), "launch": "18 (stream A)",
                  **summary(sa, base)}), flush=True)
print(json.dumps({"probe": "gso_stamps", "streams": 2, "launch": "19 (stream B)", **summary(sb, base)}), flush=True)
dev.close()
