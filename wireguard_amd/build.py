"""Build the in-tree gfx950 library (wireguard_amd/libwgcsum.so) with hipcc.

`python -m wireguard_amd.build` or `__graft_entry__.build()`.
Cross-compiles for gfx950 without a GPU.  Only `wgcs_*` symbols are exported
(linker version script), so the .so's dynamic symbol table is exactly the
C ABI of include/wgcsum.h.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libwgcsum.so")
ARCH = os.environ.get("WGCS_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def build(verbose: bool = False, out: str = OUT, extra: list[str] | None = None) -> str:
    srcs = sources()
    with tempfile.TemporaryDirectory() as td:
        vs = os.path.join(td, "exports.map")
        with open(vs, "w") as f:
            f.write("{ global: wgcs_*; local: *; };\n")
        tmp_out = out + ".tmp"
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wno-unused-result", "-Wno-unused-value", f"-I{os.path.join(ROOT, 'include')}",
               f"-Wl,--version-script={vs}", "-o", tmp_out, *srcs, *(extra or [])]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-8000:]}")
        os.replace(tmp_out, out)  # atomic: never leave a half-written .so
    return out


if __name__ == "__main__":
    print(build(verbose=True))
