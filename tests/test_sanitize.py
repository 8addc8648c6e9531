"""Host-side C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer (CPU
only; SURVEY.md §5's "test under ASan/TSan on host").

tests/sanitize/sanitize_driver.cpp links the GRO planner
(wireguard_amd/csrc/wgcs_gro_plan.h, the host half of wgcs_handle_gro and of
the write stager), the GSO layout bounds (wgcs_host.h) and the C oracle
(oracle/wg_oracle.c, as the checker), all built with -fsanitize=address,undefined
and -fno-sanitize-recover: any report aborts the run.  The corpora are the GPU
tests' own: the GRO header-field fuzz and long-run calls (tests/gro_cases.py),
the handleVirtioRead / gsoSplit header fuzz and the short-packet cases
(tests/gso_cases.py)."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

import gro_cases
import gso_cases

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "sanitize", "sanitize_driver.cpp")


def _gro_records(calls):
    out = bytearray()
    off = gro_cases.OFFSET
    for pkts, cap, can_udp, lens in calls:
        out += struct.pack("<IIiI", 1, len(pkts), off, int(can_udp))
        for k, p in enumerate(pkts):
            c = cap(len(p)) if callable(cap) else cap
            ln = off + len(p) if lens is None else lens[k]
            buf = bytearray(ln)
            buf[off:off + len(p)] = p[: max(0, ln - off)]
            out += struct.pack("<II", ln, max(c, ln) if ln else c) + bytes(buf)
    return out


def _gso_records():
    out = bytearray()
    for raw in (False, True):
        for k, (vp, nbufs, bufsize, fill, offset, hdr, is_v6) in enumerate(gso_cases.fuzz_cases(raw)):
            if k % 2:  # every other case keeps the run short under the sanitizers
                continue
            out += struct.pack("<III", 3 if raw else 2, len(vp), len(vp)) + bytes(vp)
            out += struct.pack("<IIIi", nbufs, bufsize, fill, offset)
            if raw:
                out += bytes([hdr[0], hdr[1]]) + struct.pack("<HHHH", *hdr[2:]) + struct.pack("<I", int(is_v6))
    return out


def _short_records():
    """Short packets with spare capacity after the read (gso_cases.short_cases)."""
    out = bytearray()
    for raw in (False, True):
        for rb, n_read, nbufs, bufsize, fill, offset, hdr, is_v6 in gso_cases.short_cases(raw, count=120):
            out += struct.pack("<III", 3 if raw else 2, n_read, len(rb)) + bytes(rb)
            out += struct.pack("<IIIi", nbufs, bufsize, fill, offset)
            if raw:
                out += bytes([hdr[0], hdr[1]]) + struct.pack("<HHHH", *hdr[2:]) + struct.pack("<I", int(is_v6))
    return out


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    d = tmp_path_factory.mktemp("sanitize")
    exe = d / "sanitize_driver"
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]
    inc = ["-I", os.path.join(ROOT, "wireguard_amd", "csrc"), "-I", os.path.join(ROOT, "oracle"),
           "-I", os.path.join(ROOT, "include")]
    obj = d / "wg_oracle.o"
    subprocess.run(["gcc", "-std=gnu11", "-c", *flags, *inc, "-o", str(obj), os.path.join(ROOT, "oracle", "wg_oracle.c")],
                   check=True, timeout=300)
    subprocess.run([cxx, "-std=c++17", *flags, *inc, "-o", str(exe), SRC, str(obj)], check=True, timeout=300)
    return str(exe)


def _run(driver, tmp_path, data: bytes, name: str):
    corpus = tmp_path / f"{name}.bin"
    corpus.write_bytes(data)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([driver, str(corpus)], capture_output=True, text=True, timeout=600, env=env)
    if p.returncode != 0 and "LeakSanitizer does not work under ptrace" in p.stderr:
        env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1"
        p = subprocess.run([driver, str(corpus)], capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stdout + p.stderr[-4000:]
    assert "sanitize_driver: ok" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    return p.stdout


def test_gro_planner_sanitized(driver, tmp_path):
    calls = gro_cases.field_fuzz_calls(count=150) + gro_cases.long_run_calls()
    out = _run(driver, tmp_path, bytes(_gro_records(calls)), "gro")
    assert f"{len(calls)} handleGRO calls" in out


def test_gro_planner_edge_calls_sanitized(driver, tmp_path):
    """Invalid offsets (the loop stops mid-call), zero-capacity buffers, an
    empty call, non-candidates and bad checksums through the planner."""
    rng = np.random.default_rng(5)
    p = gro_cases.packet(False, False, b"\x0a\x00\x00\x01", b"\x0a\x00\x00\x02", 1, 2, 1000,
                         rng.integers(0, 256, 100, dtype=np.uint8).tobytes())
    q = gro_cases.packet(False, False, b"\x0a\x00\x00\x01", b"\x0a\x00\x00\x02", 1, 2, 1100,
                         rng.integers(0, 256, 100, dtype=np.uint8).tobytes())
    bad = q[:-1] + bytes([q[-1] ^ 1])
    off = gro_cases.OFFSET
    calls = [
        ([p, q], 4096, True, None),
        # a third buffer of capacity 0 (the cgo shim passes NULL, len = cap = 0): invalid offset
        ([p, q, b""], lambda n: 4096 if n else 0, True, [off + len(p), off + len(q), 0]),
        ([p, bad], 4096, True, None),
        ([], 4096, True, None),
        ([b"\x45" + bytes(30)], 4096, True, None),
        ([p, q], lambda n: off + n, True, None),  # no room to append
    ]
    _run(driver, tmp_path, bytes(_gro_records(calls)), "gro_edge")


def test_gso_host_bounds_sanitized(driver, tmp_path):
    out = _run(driver, tmp_path, bytes(_gso_records()), "gso")
    assert "handleVirtioRead" in out


def test_gso_short_packets_sanitized(driver, tmp_path):
    _run(driver, tmp_path, bytes(_short_records()), "gso_short")


def test_sanitizers_are_live(tmp_path):
    """Negative controls: the same compilers and flags report a one-byte heap
    overflow (ASan) and a signed shift overflow (UBSan), so a clean run above
    means no report, not a sanitizer that never ran."""
    cases = {"address": ("char* p = (char*)malloc(8); p[8 + c - 1] = 1; int r = p[0]; free(p); return r;",
                         "heap-buffer-overflow"),
             "undefined": ("int x = 1 << (31 + c); return x & 1;", "runtime error")}
    for san, (body, want) in cases.items():
        src = tmp_path / f"{san}.cpp"
        src.write_text("#include <stdlib.h>\nint main(int c, char** v) { " + body + " }\n")
        exe = tmp_path / san
        subprocess.run(["g++", "-O0", "-g", f"-fsanitize={san}", "-fno-sanitize-recover=all", "-o", str(exe), str(src)],
                       check=True, timeout=120)
        p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60,
                           env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
        assert p.returncode != 0 and want in p.stderr, (san, p.stderr[-2000:])
