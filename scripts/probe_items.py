"""Per-item prologue/epilogue cost on the flat stream (NOT product code):
items of 6 / 12 / 24 KiB per wave, each with a dependent descriptor load and
4 / 8 / 16 wave reductions + stores (one per 1500-B packet it would hold),
interleaved with the plain flat stream at the cfg2 byte count."""
import ctypes, os, subprocess, json
import numpy as np
import torch  # first: one HIP runtime per process
here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_stream.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_stream.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
L.probe_items_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p]
nbytes = 98304000
R = 4
bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(R)]
descs = {}
for kb in (6, 12, 24):
    n_items = nbytes // (1024 * kb)
    d = np.zeros((n_items, 4), np.uint32)
    d[:, 0] = np.arange(n_items, dtype=np.uint32) * (64 * kb)
    descs[kb] = torch.from_numpy(d.view(np.uint8).reshape(-1)).cuda()
out = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
st = torch.cuda.Stream()
V = [("flat", 2048), ("items6", 4096), ("items6", 2048), ("items12", 2048), ("items12", 1024), ("items24", 1024), ("items24", 512)]
res = {v: [] for v in V}


def launch(v, buf):
    if v[0] == "flat":
        L.probe_launch(buf.data_ptr(), nbytes, out.data_ptr(), v[1], 4, 1, st.cuda_stream)
    else:
        kb = int(v[0][5:])
        L.probe_items_launch(buf.data_ptr(), nbytes, descs[kb].data_ptr(), out.data_ptr(), v[1], kb, st.cuda_stream)


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
    print(json.dumps({"pattern": v[0], "grid": v[1], "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}))
