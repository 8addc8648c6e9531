"""The C ABI driven from plain C (tests/c_harness/abi_harness.c): a process
with no Python or torch around the library, calling the entry points the way
INTEGRATION.md's cgo shims do (handleVirtioRead with cap(readBuf),
checksumValid, handleGRO with Go-slice len/cap), checked against the oracle
linked into the same binary.  Built on the CPU by __graft_entry__.build()."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c_harness", "abi_harness")


def test_harness_is_built():
    """build() compiles it; on a tree where it has not run yet, make does (it
    needs only gcc and the in-tree libwgcsum.so)."""
    import wireguard_amd

    wireguard_amd.load()  # the library the harness links against
    subprocess.run(["make", "-s", "-C", os.path.dirname(BIN)], check=True, timeout=120)
    assert os.access(BIN, os.X_OK)


@pytest.mark.gpu
def test_c_harness_runs_bit_exact():
    p = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "abi_harness: ok" in p.stdout
