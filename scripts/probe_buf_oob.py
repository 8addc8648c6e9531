"""Buffer-load range-check probe (NOT product code): which dwords of a
straddling raw buffer_load_dwordx4 return zero, for num_records 37, 38, 40."""
import ctypes, json, os, subprocess
import torch  # first: one HIP runtime per process
here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/probe_buf_oob.so"
subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", so,
                os.path.join(here, "probe_buf_oob.hip")], check=True)
L = ctypes.CDLL(so)
L.probe_buf_oob_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
src = (torch.arange(256, dtype=torch.int32) % 255 + 1).to(torch.uint8).cuda()
for n in (37, 38, 40):
    out = torch.zeros(16 * 4, dtype=torch.int32, device="cuda")
    assert L.probe_buf_oob_launch(src.data_ptr(), n, out.data_ptr(), 0) == 0
    torch.cuda.synchronize()
    o = out.cpu().view(torch.uint8).view(16, 16)
    rows = {}
    for l in range(6, 11):  # offsets 24..40
        rows[4 * l] = o[l].tolist()
    print(json.dumps({"num_records": n, "bytes_by_offset": rows}), flush=True)
