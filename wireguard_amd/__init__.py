"""wireguard_amd -- MI355X-native (gfx950) Internet-checksum hot path of
muhtutorials/wireguard's `tun` package (checksum / GSO split / GRO validate),
behind a C ABI (include/wgcsum.h) implemented by hand-written HIP kernels.
"""
from ._lib import LIB_PATH, WgcsError, declared_symbols, load  # noqa: F401

__all__ = ["LIB_PATH", "WgcsError", "declared_symbols", "load"]
