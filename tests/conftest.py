import os
import sys

import pytest

try:
    # torch bundles its own HIP runtime (libamdhip64.so.7); importing it before
    # libwgcsum.so is loaded makes the process use ONE HIP runtime (our .so
    # then binds to the already-loaded soname) -- two runtimes in one process
    # break torch's device init.
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size BASELINE configs")


@pytest.fixture(scope="session")
def dev():
    from wireguard_amd.tun import Device

    d = Device(0)
    yield d
    d.close()
