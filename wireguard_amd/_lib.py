"""ctypes binding of the in-tree C ABI library (wireguard_amd/libwgcsum.so).

The library is the product: every checksum / GSO / GRO byte is processed by
its gfx950 HIP kernels.  There is no Python or CPU fallback -- if the library
is missing or no device is present, loading or context creation raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WGCS_LIB") or os.path.join(_HERE, "libwgcsum.so")  # WGCS_LIB: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "wgcsum.h")

# status codes (include/wgcsum.h)
OK = 0
ERR_INVALID_ARG = -1
ERR_SHORT_BUFFER = -2
ERR_TOO_MANY_SEGMENTS = -3
ERR_INVALID_OFFSET = -4
ERR_UNSUPPORTED_GSO = -5
ERR_IP_GSO_MISMATCH = -6
ERR_BAD_IP_VERSION = -7
ERR_PACKET_TOO_SHORT = -8
ERR_TCP_HDR_LEN = -9
ERR_HDR_LEN = -10
ERR_CSUM_OFFSET = -11
ERR_READ_OVERFLOW = -12
ERR_OUT_OF_RANGE = -13
ERR_BATCH_FULL = -14
ERR_NOT_READY = -15
ERR_CMSG = -16
ERR_SPLIT_OVERFLOW = -17
ERR_HIP = -100
ERR_NOMEM = -101
ERR_NO_DEVICE = -102

MODE_FOLD, MODE_L4_FILL, MODE_VALIDATE, MODE_PARTIAL, MODE_IP4HDR = 0, 1, 2, 3, 4
F_INPLACE = 0x1
PKT_V6 = 0x01


class WgcsError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"wgcs error {code}: {msg}")
        self.code = code


class VirtioHdr(C.Structure):
    _fields_ = [
        ("flags", C.c_uint8), ("gso_type", C.c_uint8), ("hdr_len", C.c_uint16),
        ("gso_size", C.c_uint16), ("csum_start", C.c_uint16), ("csum_offset", C.c_uint16),
    ]


_lib = None


def declared_symbols() -> list[str]:
    """Function names declared in include/wgcsum.h."""
    with open(HEADER_PATH) as f:
        src = f.read()
    inline = set(re.findall(r"static inline [^(]*\b(wgcs_[a-z0-9_]+)\s*\(", src))  # header-only helpers
    return sorted(set(re.findall(r"\b(wgcs_[a-z0-9_]+)\s*\(", src)) - inline)


def load() -> C.CDLL:
    """Load libwgcsum.so.  If the process also uses torch, import torch FIRST:
    torch ships its own libamdhip64.so.7 and the dynamic linker then binds our
    library to that already-loaded runtime (one HIP runtime per process)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, sz, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t, C.c_int
    u8pp = C.POINTER(C.POINTER(C.c_uint8))
    sig = {
        "wgcs_abi_version": ([], i32),
        "wgcs_device_count": ([C.POINTER(i32)], i32),
        "wgcs_init": ([i32, C.POINTER(vp)], i32),
        "wgcs_destroy": ([vp], i32),
        "wgcs_strerror": ([i32], C.c_char_p),
        "wgcs_last_error": ([vp], C.c_char_p),
        "wgcs_sync": ([vp], i32),
        "wgcs_num_cu": ([vp], i32),
        "wgcs_checksum_batch": ([vp, i32, C.c_uint, vp, vp, vp, u32, vp, vp], i32),
        "wgcs_checksum_batches": ([vp, i32, C.c_uint, vp, u32, vp, u32, vp, vp], i32),
        "wgcs_gso_split_batch": ([vp, vp, vp, u32, vp, u32, u32, u32, vp, vp, vp, vp], i32),
        "wgcs_gso_kernel_shape": ([vp, vp, vp, vp], i32),
        "wgcs_handle_gro_batch": ([vp, vp, vp, vp, u32, vp, vp, vp, vp], i32),
        "wgcs_checksum": ([vp, vp, sz, u64, C.POINTER(C.c_uint16)], i32),
        "wgcs_checksum_valid": ([vp, vp, sz, C.c_uint8, C.c_uint8, i32, C.POINTER(i32)], i32),
        "wgcs_checksum_valid_cap": ([vp, vp, sz, sz, C.c_uint8, C.c_uint8, i32, C.POINTER(i32)], i32),
        "wgcs_gso_none_checksum": ([vp, vp, sz, C.c_uint16, C.c_uint16], i32),
        "wgcs_checksum_batch_host": ([vp, i32, C.c_uint, vp, sz, vp, vp, u32, vp], i32),
        "wgcs_gso_split": ([vp, vp, sz, C.POINTER(VirtioHdr), u8pp, C.POINTER(sz), i32, C.POINTER(i32), i32, i32,
                            C.POINTER(i32)], i32),
        "wgcs_handle_virtio_read": ([vp, vp, sz, u8pp, C.POINTER(sz), i32, C.POINTER(i32), i32, C.POINTER(i32)], i32),
        "wgcs_handle_virtio_read_cap": ([vp, vp, sz, sz, u8pp, C.POINTER(sz), i32, C.POINTER(i32), i32,
                                         C.POINTER(i32)], i32),
        "wgcs_gso_split_cap": ([vp, vp, sz, sz, C.POINTER(VirtioHdr), u8pp, C.POINTER(sz), i32, C.POINTER(i32), i32,
                                i32, C.POINTER(i32)], i32),
        "wgcs_handle_gro": ([vp, u8pp, C.POINTER(sz), C.POINTER(sz), i32, i32, i32, C.POINTER(i32), C.POINTER(i32)],
                            i32),
        "wgcs_stager_create": ([vp, u32, u32, sz, u32, u32, C.POINTER(vp)], i32),
        "wgcs_stager_destroy": ([vp], i32),
        "wgcs_stager_push": ([vp, vp, sz, C.POINTER(i32)], i32),
        "wgcs_stager_push_many": ([vp, C.POINTER(vp), C.POINTER(sz), i32, C.POINTER(i32), C.POINTER(i32)], i32),
        "wgcs_stager_reserve": ([vp, sz, C.POINTER(vp), C.POINTER(i32)], i32),
        "wgcs_stager_commit": ([vp, i32, sz], i32),
        "wgcs_stager_submit": ([vp, C.POINTER(u64)], i32),
        "wgcs_stager_wait": ([vp, u64], i32),
        "wgcs_stager_result": ([vp, u64, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(vp), C.POINTER(vp)], i32),
        "wgcs_get_gso_size": ([vp, sz, C.POINTER(i32)], i32),
        "wgcs_set_gso_size": ([vp, C.POINTER(sz), sz, C.c_uint16], i32),
        "wgcs_split_messages_batch": ([vp, vp, u64, u32, vp, vp, u32, u32, u32, vp, u64, vp, vp, vp, vp, vp], i32),
        "wgcs_coalesce_messages_batch": ([vp, vp, u64, u32, vp, vp, vp, u32, u32, i32, vp, vp, vp, vp, vp], i32),
        "wgcs_split_messages": ([vp, u8pp, sz, C.POINTER(i32), u8pp, C.POINTER(sz), i32, i32, C.POINTER(i32),
                                 C.POINTER(i32)], i32),
        "wgcs_coalesce_messages": ([vp, u8pp, C.POINTER(sz), C.POINTER(sz), i32, i32, vp, sz, u8pp, C.POINTER(sz),
                                    C.POINTER(sz), C.POINTER(i32), C.POINTER(sz), C.POINTER(i32)], i32),
        "wgcs_stager_copy_out": ([vp, u64, i32, u8pp, C.POINTER(sz), i32, C.POINTER(i32), i32, C.POINTER(i32)], i32),
        "wgcs_wstager_create": ([vp, u32, u32, u32, sz, C.POINTER(vp)], i32),
        "wgcs_wstager_destroy": ([vp], i32),
        "wgcs_wstager_push": ([vp, C.POINTER(vp), C.POINTER(sz), C.POINTER(sz), i32, i32, i32, C.POINTER(i32)], i32),
        "wgcs_wstager_push_pinned": ([vp, C.POINTER(vp), C.POINTER(sz), C.POINTER(sz), i32, i32, i32,
                                      C.POINTER(i32)], i32),
        "wgcs_wstager_submit": ([vp, C.POINTER(u64)], i32),
        "wgcs_ring_create": ([vp, u32, C.POINTER(vp)], i32),
        "wgcs_ring_destroy": ([vp], i32),
        "wgcs_ring_info": ([vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(i32)], i32),
        "wgcs_ring_checksum_valid": ([vp, vp, sz, C.c_uint8, C.c_uint8, i32, C.POINTER(i32)], i32),
        "wgcs_ring_checksum_valid_cap": ([vp, vp, sz, sz, C.c_uint8, C.c_uint8, i32, C.POINTER(i32)], i32),
        "wgcs_ring_handle_virtio_read": ([vp, vp, sz, u8pp, C.POINTER(sz), i32, C.POINTER(i32), i32,
                                          C.POINTER(i32)], i32),
        "wgcs_ring_handle_virtio_read_cap": ([vp, vp, sz, sz, u8pp, C.POINTER(sz), i32, C.POINTER(i32), i32,
                                              C.POINTER(i32)], i32),
        "wgcs_host_alloc": ([vp, sz, C.POINTER(vp)], i32),
        "wgcs_host_free": ([vp, vp], i32),
        "wgcs_stream_wait_flag": ([vp, vp, vp, u32], i32),
        "wgcs_wstager_wait": ([vp, u64], i32),
        "wgcs_wstager_result": ([vp, u64, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(vp),
                                 C.POINTER(sz)], i32),
    }
    missing = [name for name in sig if not hasattr(L, name)]
    if missing:
        # only an explicit A/B build of an older revision may lack entry points
        # (scripts/probe_lib_bench.sh sets WGCS_LIB_PARTIAL=1); anything else
        # fails here, at load, not later at the first call
        if os.environ.get("WGCS_LIB_PARTIAL") != "1":
            raise RuntimeError(f"{LIB_PATH}: missing wgcsum entry points {missing} (a stale or mismatched library; "
                               "rebuild with `python -m wireguard_amd.build`)")
        import warnings

        warnings.warn(f"{LIB_PATH}: partial A/B library without {missing}", RuntimeWarning, stacklevel=2)
    for name, (args, res) in sig.items():
        if name in missing:
            continue
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L
