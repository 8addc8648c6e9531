"""Segment-copy probe (NOT product code): 11,520 x 1460-B segments (the cfg4
GSO payload volume) copied into 1536-B slots, unaligned-load vs funnel mode,
at several source misalignments.  Prints one JSON line per variant."""
import ctypes, json, os, subprocess
import torch  # first: one HIP runtime per process
here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_copy.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_copy.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_copy_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
nseg, seg, stride, R = 11520, 1460, 1536, 8
src = [torch.randint(0, 255, (nseg * seg + 4096,), dtype=torch.uint8, device="cuda") for _ in range(R)]
dst = [torch.empty(nseg * stride, dtype=torch.uint8, device="cuda") for _ in range(R)]
sink = torch.zeros(16, dtype=torch.int32, device="cuda")
st = torch.cuda.Stream()
for mode in (0, 1, 2, 3):
    for mis in (0, 1, 6):
        def go(k):
            L.probe_copy_launch(src[k % R].data_ptr() + mis, dst[k % R].data_ptr(), nseg, seg, stride, mode,
                                sink.data_ptr(), st.cuda_stream)
        for k in range(10):
            go(k)
        if mis in (1, 6):
            torch.cuda.synchronize()
            a = src[0][mis:mis + seg].cpu(); b = dst[0][:seg].cpu()
            ok = bool(torch.equal(a, b))
        else:
            ok = None
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(200):
            go(k)
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 200
        nb = 2 * nseg * seg
        print(json.dumps({"mode": ["unaligned", "funnel", "dword-aligned+alignbyte", "aligned+LDS byte-phase read"][mode], "misalign": mis, "us": round(us, 2),
                          "GBps_rw": round(nb / us / 1e3, 1), "check": ok}), flush=True)
