"""Per-wave phase timeline of gso_rows_kernel from a WGCS_GSO_EXP=64 build
(s_memtime stamps, diagnostic only).  usage: WGCS_LIB=exp/gso64.so python scripts/exp_stamps.py"""
import ctypes, json, os, sys
import numpy as np
import torch  # first: one HIP runtime per process
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wireguard_amd import synth, _lib
from wireguard_amd.tun import Device, GSO_JOB_DTYPE

dev = Device(0)
n_jobs, max_segs, stride, offset = 256, 64, 1536, 16
pkts = [synth.make_super_packet(65535, 1460, seed=synth.SEED + k) for k in range(n_jobs)]
jlen = len(pkts[0])
arena = np.frombuffer(b"".join(pkts), dtype=np.uint8).copy()
jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(jlen)
jobs["len"] = jlen
R = 8
st = torch.cuda.Stream()
d_arena = [torch.from_numpy(arena).cuda() for _ in range(R)]
d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
d_out = [torch.empty(n_jobs * max_segs * stride, dtype=torch.uint8, device="cuda") for _ in range(R)]
d_sizes = torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda")
d_count = torch.zeros(n_jobs, dtype=torch.int32, device="cuda")
d_status = torch.zeros(n_jobs, dtype=torch.int32, device="cuda")
L = _lib.load()
L.wgcs_exp_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
for k in range(40):
    dev.gso_split_batch(d_arena[k % R], d_jobs, n_jobs, d_out[k % R], stride, offset, max_segs, d_sizes, d_count,
                        d_status, stream=st)
torch.cuda.synchronize()
buf = np.zeros(1 << 16, dtype=np.uint64)
L.wgcs_exp_stamps(buf.ctypes.data, buf.nbytes)
nw = n_jobs * 2 * 16  # (job, segment group) blocks x 16 waves
S = buf[: nw * 8].reshape(nw, 8).astype(np.int64)
t0 = S[:, 0][S[:, 0] > 0].min()
out = {}
alive = S[:, 0] > 0
for k in range(8):
    v = S[:, k]
    m = v > 0
    out[f"t{k}_from_start"] = {q: int(np.percentile(v[m] - t0, q)) for q in (0, 10, 50, 90, 100)} if m.any() else None
for a, b in ((0, 1), (1, 3), (3, 4), (0, 4), (0, 3), (0, 5), (5, 2), (2, 6), (5, 6), (6, 7), (7, 1)):
    m = (S[:, a] > 0) & (S[:, b] > 0)
    d = S[m, b] - S[m, a]
    out[f"d{a}{b}"] = {q: int(np.percentile(d, q)) for q in (10, 50, 90)} if m.any() else None
out["waves_started"] = int(alive.sum())
out["waves_full"] = int((S[:, 4] > 0).sum())
print(json.dumps(out, indent=1))
