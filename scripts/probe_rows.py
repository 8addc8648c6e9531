"""Row access patterns of the checksum kernel vs the flat stream (NOT product
code): G-lane rows with and without the dependent descriptor load, next to
the flat register stream, interleaved on one box at the cfg2 byte count."""
import ctypes, os, subprocess, json
import numpy as np
import torch  # first: one HIP runtime per process
here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_stream.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_stream.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
L.probe_rowsg_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
npk, flen = 65536, 1500
nbytes = npk * flen
R = 4
bufs = [torch.randint(0, 255, (nbytes + 4096,), dtype=torch.uint8, device="cuda") for _ in range(R)]
d = np.zeros((npk, 4), np.uint32)
d[:, 0] = (np.arange(npk, dtype=np.uint64) * flen).astype(np.uint32)
d[:, 2] = flen
desc = torch.from_numpy(d.view(np.uint8).reshape(-1)).cuda()
out = torch.empty(16384 * 256, dtype=torch.int32, device="cuda")
st = torch.cuda.Stream()
V = [("flat", 2048, 4, 0), ("flat+16", 2048, 4, 0), ("flat+48", 2048, 4, 0), ("flat+64", 2048, 4, 0), ("rows", 4096, 16, 0), ("rows", 4096, 16, 1), ("rows32u4", 4096, 32, 0),
     ("rows32u4", 4096, 32, 1), ("rows32u3", 4096, 32, 0), ("rows32u3", 4096, 32, 1), ("rows64", 4096, 64, 0)]
res = {v: [] for v in V}


def launch(v, buf):
    kind, grid, g, dd = v
    if kind.startswith("flat"):  # flat+N: the whole stream shifted by N bytes off 128-B line alignment
        sh = int(kind[5:]) if "+" in kind else 0
        L.probe_launch(buf.data_ptr() + sh, nbytes, out.data_ptr(), grid, g, 1, st.cuda_stream)
    else:
        u = 3 if kind == "rows32u3" else 4
        L.probe_rowsg_launch(buf.data_ptr(), desc.data_ptr(), npk, flen, out.data_ptr(), grid, g, u, dd, st.cuda_stream)


for rnd in range(3):
    for v in V:
        for k in range(5):
            launch(v, bufs[k % R])
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(100):
            launch(v, bufs[k % R])
        e1.record(st)
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) * 1e3 / 100)
for v in V:
    us = sorted(res[v])[1]
    print(json.dumps({"pattern": v[0], "grid": v[1], "G": v[2], "desc": v[3], "us": round(us, 2),
                      "GBps": round(nbytes / us / 1e3, 1)}))
