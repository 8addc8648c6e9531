"""Flat streaming-read ceiling with consecutive launches on two streams, next
to the same on one stream (NOT product code): how far the cfg2 checksum
launch (14.7 us on two streams, 17.0 on one) is from a flat read of the same
98.3 MB.  Builds scripts/probe_stream.hip."""
import ctypes
import json
import os
import subprocess

import torch  # first: one HIP runtime per process

here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_stream2.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_stream.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p]
nbytes, R = 98304000, 4
bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(R)]
outs = [torch.empty(256 * 256 * 64, dtype=torch.int32, device="cuda") for _ in range(2)]
sts = [torch.cuda.Stream(), torch.cuda.Stream()]
for ns in (1, 2, 1, 2):
    for grid, u, nt in ((2048, 4, 1), (4096, 4, 1), (4096, 8, 1)):
        def run(K):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(sts[0])
            if ns > 1:
                sts[1].wait_event(e0)
            for k in range(K):
                q = k % ns
                L.probe_launch(bufs[k % R].data_ptr(), nbytes, outs[q].data_ptr(), grid, u, nt, sts[q].cuda_stream)
            if ns > 1:
                j = torch.cuda.Event()
                j.record(sts[1])
                sts[0].wait_event(j)
            e1.record(sts[0])
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / K
        run(10)
        us = run(200)
        print(json.dumps({"streams": ns, "grid": grid, "U": u, "nt": nt, "us_per_launch": round(us, 2),
                          "frac_of_8TBps": round(nbytes / us / 1e3 / 8000, 4)}), flush=True)
