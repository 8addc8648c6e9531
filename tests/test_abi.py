"""CPU tests of the C ABI boundary (no GPU compute): the in-tree library
loads, exports exactly the symbols include/wgcsum.h declares, the header is
valid C with the documented struct layouts, and the Python mirror agrees with
the header's constants.  Without a device, every compute entry fails loudly
(there is no CPU fallback)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import wireguard_amd
from wireguard_amd import _lib, tun

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "wgcsum.h")


def _defines():
    out = {}
    for m in re.finditer(r"#define\s+(WGCS_\w+)\s+\(?(-?(?:0x)?[0-9a-fA-F]+)u?\)?", open(HDR).read()):
        out[m.group(1)] = int(m.group(2), 0)
    return out


def test_library_exports_every_declared_symbol():
    L = wireguard_amd.load()
    declared = _lib.declared_symbols()
    assert len(declared) >= 17
    for name in declared:
        assert hasattr(L, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = sorted({l.split()[-1] for l in nm.stdout.splitlines() if l.split()[-1].startswith("wgcs_")})
    assert exported == declared
    other = [l for l in nm.stdout.splitlines() if " T " in l and "wgcs_" not in l]
    assert not other, f"unexpected exports: {other[:5]}"


def test_header_is_c_and_layouts(tmp_path):
    src = tmp_path / "t.c"
    src.write_text(
        '#include "wgcsum.h"\n#include <stddef.h>\n'
        "_Static_assert(sizeof(wgcs_pkt) == 16, \"pkt\");\n"
        "_Static_assert(offsetof(wgcs_pkt, off_hi) == 4, \"off_hi\");\n"
        "_Static_assert(offsetof(wgcs_pkt, proto) == 6, \"proto\");\n"
        "_Static_assert(offsetof(wgcs_pkt, flags) == 7, \"flags\");\n"
        "_Static_assert(offsetof(wgcs_pkt, len) == 8, \"len\");\n"
        "_Static_assert(offsetof(wgcs_pkt, csum_start) == 12, \"cs\");\n"
        "_Static_assert(offsetof(wgcs_pkt, csum_offset) == 14, \"co\");\n"
        "_Static_assert(sizeof(wgcs_gso_job) == 16, \"job\");\n"
        "_Static_assert(sizeof(wgcs_virtio_hdr) == 10, \"virtio_net_hdr is 10 bytes (gro.go:69-71)\");\n"
        "int main(void) { return 0; }\n")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HDR), str(src), "-o",
                    str(tmp_path / "t")], check=True)


def test_python_constants_match_header():
    d = _defines()
    for name, val in d.items():
        short = name[len("WGCS_"):]
        if hasattr(_lib, short):
            assert getattr(_lib, short) == val, name
    assert tun.PKT_DTYPE.itemsize == 16 and tun.GSO_JOB_DTYPE.itemsize == 16
    for f in ("off_lo", "off_hi", "proto", "flags", "len", "csum_start", "csum_offset"):
        assert tun.PKT_DTYPE.fields[f][1] == oracle_dtype().fields[f][1], f
    assert C.sizeof(_lib.VirtioHdr) == 10
    assert d["WGCS_MODE_VALIDATE"] == _lib.MODE_VALIDATE


def oracle_dtype():
    import oracle
    return oracle.PKT_DTYPE


def test_pkt_set_matches_python_layout(tmp_path):
    """wgcs_pkt_set (header-only helper) packs what tun.set_pkt_off + fields do."""
    src = tmp_path / "p.c"
    src.write_text('#include "wgcsum.h"\n#include <stdio.h>\n#include <string.h>\n'
                   "int main(void) { wgcs_pkt p; unsigned char b[16]; "
                   "wgcs_pkt_set(&p, 0x123456789ABCull, 1500, 20, 40000, 17, WGCS_PKT_V6); "
                   "memcpy(b, &p, 16); for (int i = 0; i < 16; i++) printf(\"%02x\", b[i]); return 0; }\n")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HDR), str(src), "-o",
                    str(tmp_path / "p")], check=True)
    out = subprocess.run([str(tmp_path / "p")], capture_output=True, text=True, check=True).stdout
    p = np.zeros(1, tun.PKT_DTYPE)
    tun.set_pkt_off(p, [0x123456789ABC])
    p["len"], p["csum_start"], p["csum_offset"], p["proto"], p["flags"] = 1500, 20, 40000, 17, tun.PKT_V6
    assert out == p.tobytes().hex()
    assert int(tun.pkt_off(p)[0]) == 0x123456789ABC


def test_version_and_errors():
    L = wireguard_amd.load()
    assert L.wgcs_abi_version() == _defines()["WGCS_ABI_VERSION"]
    for code in [0, -1, -2, -3, -4, -5, -6, -7, -8, -9, -10, -11, -12, -13, -14, -15, -16, -17, -100, -101, -102]:
        assert L.wgcs_strerror(code) and L.wgcs_strerror(code) != b"unknown status"
    assert L.wgcs_strerror(-9999) == b"unknown status"


def test_gso_kernel_shape_reports_compiled_grid():
    """gso_bench names the kernel (and its traffic record) from the library's
    compiled shape, not from constants of its own."""
    L = wireguard_amd.load()
    nw, parts, u, rows = (C.c_int(-1) for _ in range(4))
    assert L.wgcs_gso_kernel_shape(C.byref(nw), C.byref(parts), C.byref(u), C.byref(rows)) == 0
    assert nw.value in (1, 2, 4, 8, 16) and 1 <= parts.value <= 8 and u.value > 0 and rows.value in (0, 1)
    assert L.wgcs_gso_kernel_shape(None, None, None, None) == 0


def test_no_device_fails_loudly():
    """In this container there is no GPU: the product must refuse, not fall back."""
    L = wireguard_amd.load()
    n = C.c_int(-1)
    rc = L.wgcs_device_count(C.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a device is present")
    with pytest.raises(_lib.WgcsError) as ei:
        tun.Device(0)
    assert ei.value.code == _lib.ERR_NO_DEVICE
    # NULL-context calls are rejected without touching any device
    assert L.wgcs_checksum_batch(None, 0, 0, None, None, None, 1, None, None) == _lib.ERR_INVALID_ARG
    assert L.wgcs_gso_split_batch(None, None, None, 1, None, 0, 0, 1, None, None, None, None) == _lib.ERR_INVALID_ARG
    assert L.wgcs_destroy(None) == _lib.ERR_INVALID_ARG


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(ImportError):
        _lib.load()


def test_synth_descriptors_layout():
    from wireguard_amd import synth
    arena, pkts, k = synth.make_batch(64, 1500, kinds="mixed")
    assert pkts.dtype == tun.PKT_DTYPE
    assert (tun.pkt_off(pkts) == np.arange(64) * 1500).all()
    assert set(np.unique(pkts["csum_offset"])) <= {6, 16}
    assert ((pkts["proto"] == 17) == (pkts["csum_offset"] == 6)).all()
