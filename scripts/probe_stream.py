"""Practical HBM streaming-read ceiling on this GPU (NOT product code).
Builds scripts/probe_stream.hip with hipcc, reads the same byte count as the
cfg2 checksum batch (98.3 MB x 4 rotated copies) and reports GB/s."""
import ctypes, os, subprocess, sys, json
import torch  # first: one HIP runtime per process
import numpy as np
here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_stream.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_stream.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
nbytes = 98304000
R = 4
bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(R)]
out = torch.empty(256 * 256 * 64, dtype=torch.int32, device="cuda")
st = torch.cuda.Stream()
res = []
for grid in (1024, 2048, 4096):
    for u in (2, 4, 8):
        for nt in (0, 1):
            for k in range(5):
                L.probe_launch(bufs[k % R].data_ptr(), nbytes, out.data_ptr(), grid, u, nt, st.cuda_stream)
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            it = 100
            for k in range(it):
                L.probe_launch(bufs[k % R].data_ptr(), nbytes, out.data_ptr(), grid, u, nt, st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / it
            res.append((nbytes / us / 1e3, grid, u, nt, us))
            print(json.dumps({"grid": grid, "U": u, "nt": nt, "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}))
L.probe_rows_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
for grid in (1024, 2048):
    for nt in (0, 1):
        for k in range(5):
            L.probe_rows_launch(bufs[k % R].data_ptr(), 65536, 1500, out.data_ptr(), grid, nt, st.cuda_stream)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(100):
            L.probe_rows_launch(bufs[k % R].data_ptr(), 65536, 1500, out.data_ptr(), grid, nt, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 100
        print(json.dumps({"pattern": "rows16x4 (checksum kernel access pattern)", "grid": grid, "nt": nt, "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}))
L.probe_wavef_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
for grid in (1024, 2048, 4096):
    for f in (1, 2, 4):
        for k in range(5):
            L.probe_wavef_launch(bufs[k % R].data_ptr(), 65536, 1500, out.data_ptr(), grid, f, st.cuda_stream)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(100):
            L.probe_wavef_launch(bufs[k % R].data_ptr(), 65536, 1500, out.data_ptr(), grid, f, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 100
        print(json.dumps({"pattern": f"wave-per-packet, {f} packets in flight (1 KiB per load instruction)", "grid": grid, "nt": 1, "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}))
best = max(res)
print(json.dumps({"best_GBps": round(best[0], 1), "frac_8TBs": round(best[0] / 8000, 3), "grid": best[1], "U": best[2], "nt": best[3]}))
