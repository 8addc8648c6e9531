"""Flat streaming-read ceiling at cfg5's size (NOT product code): the fastest
plain 16-B-per-lane read of 1.57 GB (configs[4]'s 1 M x 1500 B, far past the
256 MiB Infinity Cache) next to the same read of cfg2's 98.3 MB, one and two
streams, several grids.  The cfg5_strong line (one 0.26-ms launch per step) is
compared against this, not against the 8 TB/s spec.  Builds
scripts/probe_stream.hip."""
import ctypes
import json
import os
import subprocess
import sys

import torch  # first: one HIP runtime per process

here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_stream3.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_stream.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p]
L.probe_glds_launch.argtypes = L.probe_launch.argtypes
outs = [torch.empty(65536 * 256, dtype=torch.int32, device="cuda") for _ in range(2)]
sts = [torch.cuda.Stream(), torch.cuda.Stream()]
SIZES = ((98304000, 4, 200), (1572864000, 2, 20))
if os.environ.get("BIG_ONLY"):
    SIZES = SIZES[1:]
for nbytes, R, K in SIZES:
    bufs = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(R)]
    for ns in (1, 2):
        for kind, grid, u in (("reg", 2048, 4), ("reg", 4096, 4), ("reg", 8192, 4), ("reg", 4096, 8),
                              ("reg", 16384, 4), ("glds", 2048, 4), ("glds", 4096, 4))[:int(os.environ.get("NSHAPES", "7"))]:
            fn = L.probe_launch if kind == "reg" else L.probe_glds_launch

            def run(K):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(sts[0])
                if ns > 1:
                    sts[1].wait_event(e0)
                for k in range(K):
                    q = k % ns
                    fn(bufs[k % R].data_ptr(), nbytes, outs[q].data_ptr(), grid, u, 1, sts[q].cuda_stream)
                if ns > 1:
                    j = torch.cuda.Event()
                    j.record(sts[1])
                    sts[0].wait_event(j)
                e1.record(sts[0])
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) * 1e3 / K

            run(4)
            warm_ms = float(os.environ.get("WARM_MS", "0"))  # sustained launches before timing (r5_cfg5_regions)
            if warm_ms > 0:
                import time
                t_end = time.perf_counter() + warm_ms / 1e3
                while time.perf_counter() < t_end:
                    run(8)
            us = min(run(K) for _ in range(3))
            print(json.dumps({"bytes": nbytes, "kind": kind, "streams": ns, "grid": grid, "U": u, "nt": 1,
                              "warm_ms": float(os.environ.get("WARM_MS", "0")), "us_per_launch": round(us, 2), "frac_of_8TBps": round(nbytes / us / 1e3 / 8000, 4)}),
                  flush=True)
    del bufs
    torch.cuda.empty_cache()
sys.exit(0)
