"""FETCH_SIZE calibration for gro_batch_kernel's read pattern (NOT product
code; MI355X_MICROARCH.md: 'other access widths are uncalibrated: calibrate
on a known byte count in your own access pattern').  Run under
`rocprofv3 --pmc FETCH_SIZE --kernel-trace`; prints the requested byte counts
per launch, which scripts/pmc_traffic.py-style parsing divides into."""
import ctypes
import json
import os
import subprocess

import torch  # first: one HIP runtime per process

here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_fetch_cal.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_fetch_cal.hip")], check=True)
L = ctypes.CDLL(so)
L.cal_wide_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
L.cal_rows_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.c_void_p, ctypes.c_void_p]
s = torch.cuda.current_stream().cuda_stream
out = torch.zeros(16, dtype=torch.int32, device="cuda")
wide_bytes = 384 << 20  # past the 256 MiB Infinity Cache
wide = torch.ones(wide_bytes, dtype=torch.uint8, device="cuda")
npk = 229376  # gro_device's 1,792 calls x 128 buffers
arena = torch.ones(npk * 65552 + 4096, dtype=torch.uint8, device="cuda")
rec = {"wide_bytes": wide_bytes, "rows": {}}
for k in range(5):
    L.cal_wide_launch(wide.data_ptr(), wide_bytes, out.data_ptr(), s)
# (stride, offset, length): gro_device's packets (1,488 B), their payload
# pieces (1,448), a 1,500-B frame, a 60-B header read, and udp_coalesce's
# 1,452-B pieces 64 KiB apart
for stride, off, ln in ((65552, 16, 1488), (65552, 16, 1448), (65552, 16, 1500), (65552, 16, 60), (65536, 0, 1452)):
    a0 = [(arena.data_ptr() + p * stride + off) & ~15 for p in range(0, npk)]
    span = sum(((arena.data_ptr() + p * stride + off + ln + 15) & ~15) - a for p, a in zip(range(npk), a0))
    # the bytes of the 128-B (and 64-B) lines the rows touch: a read's floor
    # at line granularity (round 5: the sized-request counters, scripts/pmc_sized.py)
    base = arena.data_ptr()
    lines128 = sum((((base + p * stride + off + ln + 127) >> 7) - ((base + p * stride + off) >> 7)) for p in range(npk))
    lines64 = sum((((base + p * stride + off + ln + 63) >> 6) - ((base + p * stride + off) >> 6)) for p in range(npk))
    rec["rows"][f"{ln}@{stride}+{off}"] = {"len_bytes": npk * ln, "span_bytes": span, "line128_bytes": 128 * lines128,
                                         "line64_bytes": 64 * lines64}
    for k in range(5):
        L.cal_rows_launch(arena.data_ptr(), npk, stride, off, ln, out.data_ptr(), s)
torch.cuda.synchronize()
print(json.dumps(rec))
