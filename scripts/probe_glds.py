"""LDS-DMA vs register streaming read (NOT product code).  Builds
scripts/probe_stream.hip, times interleaved variants on the cfg2 byte count
(98.3 MB x 4 rotated copies) and on one 393-MB launch (ramp cost)."""
import ctypes, os, subprocess, json
import torch  # first: one HIP runtime per process
here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_stream.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_stream.hip")], check=True)
L = ctypes.CDLL(so)
sig = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
L.probe_launch.argtypes = sig
L.probe_glds_launch.argtypes = sig
nbytes = 98304000
R = 4
big = torch.randint(0, 255, (nbytes * R,), dtype=torch.uint8, device="cuda")
bufs = [big[k * nbytes:(k + 1) * nbytes] for k in range(R)]
out = torch.empty(8192 * 256, dtype=torch.int32, device="cuda")
st = torch.cuda.Stream()
variants = [("reg", 2048, 4, 1), ("reg", 4096, 8, 1)]
for g in (1024, 2048, 4096):
    for u in (2, 4, 8):
        for nt in (0, 1):
            variants.append(("glds", g, u, nt))
res = {v: [] for v in variants}
resbig = {v: [] for v in variants}
for rnd in range(3):
    for v in variants:
        f = L.probe_launch if v[0] == "reg" else L.probe_glds_launch
        for k in range(5):
            f(bufs[k % R].data_ptr(), nbytes, out.data_ptr(), v[1], v[2], v[3], st.cuda_stream)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True); e2 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(100):
            f(bufs[k % R].data_ptr(), nbytes, out.data_ptr(), v[1], v[2], v[3], st.cuda_stream)
        e1.record(st)
        for k in range(25):
            f(big.data_ptr(), nbytes * R, out.data_ptr(), v[1], v[2], v[3], st.cuda_stream)
        e2.record(st)
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) * 1e3 / 100)
        resbig[v].append(e1.elapsed_time(e2) * 1e3 / 25)
    print("round", rnd, flush=True)
for v in variants:
    us = sorted(res[v])[1]
    ub = sorted(resbig[v])[1]
    print(json.dumps({"kind": v[0], "grid": v[1], "U": v[2], "nt": v[3], "us_98MB": round(us, 2),
                      "GBps_98MB": round(nbytes / us / 1e3, 1), "us_393MB": round(ub, 2),
                      "GBps_393MB": round(nbytes * R / ub / 1e3, 1)}))
