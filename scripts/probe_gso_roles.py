#!/usr/bin/env python3
"""Per-role phase stamps of the staged gso_lds_kernel (NOT product code).
Build with -DWGCS_GSO_STAMPS=3 (STAMPS_SO); lane 0 of every wave writes 5
s_memrealtime stamps into sizes[] slots 64.. of its job (wave slot part*4+wv):
  loader (wave 0):   T0 start, T1 init barrier, T2 header DMA landed, T3 all landed, T4 end
  head (wave 1):     T0 start, T1 init barrier, T2 header seen, T3 head published, T4 end
  rows (waves 2, 3): T0 start, T1 init barrier, T2 head seen, T3 first rows start, T4 end
Prints per role the percentiles (us from the launch's first wave start) of a
one-stream launch."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from wireguard_amd import _lib, synth
from wireguard_amd.tun import GSO_JOB_DTYPE, Device
_lib.LIB_PATH = os.environ["STAMPS_SO"]
torch.cuda.set_device(0)
dev = Device(0)
n_jobs, total, gso, max_segs, stride, offset = int(os.environ.get("N_JOBS", "256")), 65535, 1460, 128, 1536, 16
pkts = [synth.make_super_packet(total, gso, seed=synth.SEED + k) for k in range(n_jobs)]
jlen = len(pkts[0]); jpitch = -(-jlen // 128) * 128
arena = np.zeros(n_jobs * jpitch + 64, np.uint8)
for k, p in enumerate(pkts):
    arena[k * jpitch: k * jpitch + jlen] = np.frombuffer(p, np.uint8)
jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(jpitch); jobs["len"] = jlen
R = 8
d_arena = [torch.from_numpy(arena).cuda() for _ in range(R)]
d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
oshift = (128 - offset % 128) % 128
d_out = [torch.empty(n_jobs * max_segs * stride + 256, dtype=torch.uint8, device="cuda")[oshift:] for _ in range(R)]
d_sizes = torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda")
d_count = torch.zeros(n_jobs, dtype=torch.int32, device="cuda"); d_status = torch.zeros(n_jobs, dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
for k in range(30):
    dev.gso_split_batch(d_arena[k % R], d_jobs, n_jobs, d_out[k % R], stride, offset, max_segs, d_sizes, d_count, d_status, stream=s)
torch.cuda.synchronize()
st = d_sizes.cpu().numpy().reshape(n_jobs, max_segs)[:, 64:64 + 60].reshape(n_jobs, 3, 4, 5).astype(np.int64) & 0xFFFFFFFF
base = st[..., 0].min()
us = (st - base) * 0.01
names = {"loader": ["T0", "T1_init", "T2_hdr_landed", "T3_all_landed", "T4_end"],
         "head": ["T0", "T1_init", "T2_hdr_seen", "T3_head_published", "T4_end"],
         "rows": ["T0", "T1_init", "T2_head_seen", "T3_rows_start", "T4_end"]}
for role, w in (("loader", [0]), ("head", [1]), ("rows", [2, 3])):
    v = us[:, :, w, :].reshape(-1, 5)
    print(json.dumps({"role": role, **{n: [round(float(np.percentile(v[:, k], p)), 2) for p in (0, 10, 50, 90, 100)]
                                       for k, n in enumerate(names[role])}}))
dev.close()
