"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper around oracle/_build/libwgoracle.so.

The oracle is the CPU restatement of the reference's hot path
(/root/reference/tun/checksum.go, tun/gro.go, tun/tun.go:514-632), see
wg_oracle.c.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module; the product (wireguard_amd/) never does.

Parity pinning: the reference ships no tests or fixtures and cannot be built
here (no Go toolchain), so the restatement is pinned by independent KATs and a
closed-form cross-check only ("parity unpinned" against reference outputs; see
DESIGN.md).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libwgoracle.so")

PKT_DTYPE = np.dtype(  # or_pkt == wgcs_pkt layout (ABI 2)
    [("off_lo", "<u4"), ("off_hi", "<u2"), ("proto", "u1"), ("flags", "u1"), ("len", "<u4"),
     ("csum_start", "<u2"), ("csum_offset", "<u2")]
)
assert PKT_DTYPE.itemsize == 16


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        u8p = C.POINTER(C.c_uint8)
        L.or_checksum_nofold.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.or_checksum_nofold.restype = C.c_uint64
        L.or_checksum.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.or_checksum.restype = C.c_uint16
        L.or_pseudo_header_nofold.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint8, C.c_uint16]
        L.or_pseudo_header_nofold.restype = C.c_uint64
        L.or_checksum_valid.argtypes = [C.c_void_p, C.c_size_t, C.c_uint8, C.c_uint8, C.c_int]
        L.or_checksum_valid.restype = C.c_int
        L.or_gso_none_checksum.argtypes = [C.c_void_p, C.c_size_t, C.c_uint16, C.c_uint16]
        L.or_gso_none_checksum.restype = C.c_int
        L.or_handle_virtio_read.argtypes = [
            C.c_void_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t), C.c_int,
            C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int),
        ]
        L.or_handle_virtio_read.restype = C.c_int
        L.or_handle_virtio_read_cap.argtypes = [
            C.c_void_p, C.c_size_t, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t), C.c_int,
            C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int),
        ]
        L.or_handle_virtio_read_cap.restype = C.c_int
        L.or_handle_gro.argtypes = [
            C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.c_int, C.c_int, C.c_int,
            C.POINTER(C.c_int), C.POINTER(C.c_int),
        ]
        L.or_handle_gro.restype = C.c_int
        L.or_checksum_batch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int]
        L.or_checksum_batch.restype = None
        L.or_checksum_batch_mt.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int]
        L.or_checksum_batch_mt.restype = None
        L.or_gso_bench_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_double, C.POINTER(C.c_uint64)]
        L.or_gso_bench_mt.restype = C.c_double
        L.or_gro_bench_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_double, C.POINTER(C.c_uint64)]
        L.or_gro_bench_mt.restype = C.c_double
        L.or_checksum_bench_mt.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32, C.c_int, C.c_double,
                                           C.POINTER(C.c_uint64)]
        L.or_checksum_bench_mt.restype = C.c_double
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def checksum_nofold(b: bytes, initial: int = 0) -> int:
    a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)
    return lib().or_checksum_nofold(_ptr(a), len(b), initial & (2**64 - 1))


def checksum(b: bytes, initial: int = 0) -> int:
    a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)
    return lib().or_checksum(_ptr(a), len(b), initial & (2**64 - 1))


def pseudo_header_nofold(src: bytes, dst: bytes, proto: int, total_len: int) -> int:
    s = np.frombuffer(bytes(src), dtype=np.uint8)
    d = np.frombuffer(bytes(dst), dtype=np.uint8)
    return lib().or_pseudo_header_nofold(_ptr(s), _ptr(d), len(src), proto, total_len & 0xFFFF)


def checksum_valid(pkt: bytes, iph_len: int, proto: int, is_v6: bool, n: int | None = None):
    """checksumValid(pkt[:n], ...) with cap len(pkt) (n: the whole of pkt).
    True / False, or the OUT_OF_RANGE code where Go panics."""
    L = lib()
    if not getattr(L, "_valid_cap_ready", False):
        L.or_checksum_valid_cap.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_uint8, C.c_uint8, C.c_int]
        L.or_checksum_valid_cap.restype = C.c_int
        L._valid_cap_ready = True
    a = np.frombuffer(bytes(pkt) + b"\0", dtype=np.uint8)
    ln = len(pkt) if n is None else n
    rc = L.or_checksum_valid_cap(_ptr(a), ln, len(pkt), iph_len, proto, int(is_v6))
    return rc if rc < 0 else bool(rc)


def checksum_batch(mode: int, arena: np.ndarray, pkts: np.ndarray, initial=None, inplace=False):
    """Run the oracle's batch restatement; returns the per-packet outputs."""
    assert arena.dtype == np.uint8 and pkts.dtype == PKT_DTYPE
    n = len(pkts)
    out = np.zeros(n, dtype=np.uint8 if mode == 2 else np.uint16)
    ini = 0
    if initial is not None:
        initial = np.ascontiguousarray(initial, dtype=np.uint64)
        ini = _ptr(initial)
    lib().or_checksum_batch(mode, _ptr(arena), _ptr(pkts), ini or None, n, _ptr(out), int(inplace))
    return out


def checksum_batch_mt(mode: int, arena: np.ndarray, pkts: np.ndarray, threads: int):
    n = len(pkts)
    out = np.zeros(n, dtype=np.uint8 if mode == 2 else np.uint16)
    lib().or_checksum_batch_mt(mode, _ptr(arena), _ptr(pkts), n, _ptr(out), threads)
    return out


def host_threads() -> int:
    """Host threads for all-cores baselines: OMP_NUM_THREADS (16 on the GPU
    box, its CPU share) capped by the process's CPU affinity."""
    t = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    return max(1, min(t, len(os.sched_getaffinity(0))))


def gso_bench_mt(reads: list, nbufs: int, buf_len: int, offset: int, threads: int, seconds: float):
    """handleVirtioRead calls/s over `threads` pthreads (wg_oracle_bench.c)."""
    arena = np.frombuffer(b"".join(reads), np.uint8)
    lens = np.array([len(r) for r in reads], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    calls = C.c_uint64(0)
    rate = lib().or_gso_bench_mt(_ptr(arena), _ptr(offs), _ptr(lens), len(reads), nbufs, buf_len, offset, threads,
                                 seconds, C.byref(calls))
    return rate, calls.value


def checksum_bench_mt(mode: int, arena: np.ndarray, pkts: np.ndarray, threads: int, seconds: float):
    """Whole-batch passes/s summed over `threads` pthreads, each on its own
    copy of the arena (wg_oracle_bench.c)."""
    passes = C.c_uint64(0)
    rate = lib().or_checksum_bench_mt(mode, _ptr(arena), arena.nbytes, _ptr(pkts), len(pkts), threads, seconds,
                                      C.byref(passes))
    return rate, passes.value


def gro_bench_mt(pkts: list, offset: int, can_udp: bool, threads: int, seconds: float):
    """handleGRO calls/s (one call = the whole batch) over `threads` pthreads."""
    stride = max(len(p) for p in pkts)
    a = np.zeros((len(pkts), stride), np.uint8)
    for i, p in enumerate(pkts):
        a[i, : len(p)] = np.frombuffer(p, np.uint8)
    lens = np.array([len(p) for p in pkts], np.uint64)
    calls = C.c_uint64(0)
    rate = lib().or_gro_bench_mt(_ptr(a), _ptr(lens), stride, len(pkts), offset, int(can_udp), threads, seconds,
                                 C.byref(calls))
    return rate, calls.value


def _bufs_ctypes(bufs):
    u8p = C.POINTER(C.c_uint8)
    arr = (u8p * len(bufs))()
    for i, b in enumerate(bufs):
        arr[i] = C.cast(b.ctypes.data, u8p)
    return arr


def handle_virtio_read(read_buf: bytearray, bufs: list, offset: int, n_read: int | None = None):
    """Oracle handleVirtioRead.  Mutates read_buf (like the reference) and the
    numpy bufs.  With n_read, the read is read_buf[:n_read] and the rest of
    read_buf its spare capacity (Tun.Read's tun.readBuf[:n]).  Returns
    (rc, n, sizes)."""
    rb = np.frombuffer(read_buf, dtype=np.uint8) if not isinstance(read_buf, np.ndarray) else read_buf
    lens = (C.c_size_t * len(bufs))(*[len(b) for b in bufs])
    sizes = (C.c_int * len(bufs))()
    n = C.c_int(0)
    nr = len(rb) if n_read is None else n_read
    assert 0 <= nr <= len(rb)
    rc = lib().or_handle_virtio_read_cap(_ptr(rb) if len(rb) else None, nr, len(rb), _bufs_ctypes(bufs), lens,
                                         len(bufs), sizes, offset, C.byref(n))
    return rc, n.value, list(sizes)


class VirtioHdr(C.Structure):  # or_virtio_hdr (gro.go:42-67)
    _fields_ = [("flags", C.c_uint8), ("gso_type", C.c_uint8), ("hdr_len", C.c_uint16), ("gso_size", C.c_uint16),
                ("csum_start", C.c_uint16), ("csum_offset", C.c_uint16)]


def gso_split(read_buf, hdr: tuple, bufs: list, offset: int, is_v6: bool, n_read: int | None = None):
    """Oracle gsoSplit(readBuf, hdr, bufs, sizes, offset, isV6).  hdr =
    (flags, gso_type, hdr_len, gso_size, csum_start, csum_offset).  Mutates
    read_buf and bufs.  With n_read, readBuf is read_buf[:n_read] with the
    rest as its spare capacity.  Returns (rc, n, sizes)."""
    L = lib()
    if not getattr(L, "_split_ready", False):
        u8p = C.POINTER(C.c_uint8)
        L.or_gso_split_cap.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, VirtioHdr, C.POINTER(u8p),
                                       C.POINTER(C.c_size_t), C.c_int, C.POINTER(C.c_int), C.c_int, C.c_int,
                                       C.POINTER(C.c_int)]
        L.or_gso_split_cap.restype = C.c_int
        L._split_ready = True
    rb = np.frombuffer(read_buf, dtype=np.uint8) if not isinstance(read_buf, np.ndarray) else read_buf
    lens = (C.c_size_t * len(bufs))(*[len(b) for b in bufs])
    sizes = (C.c_int * len(bufs))()
    n = C.c_int(0)
    nr = len(rb) if n_read is None else n_read
    assert 0 <= nr <= len(rb)
    rc = L.or_gso_split_cap(_ptr(rb) if len(rb) else None, nr, len(rb), VirtioHdr(*hdr), _bufs_ctypes(bufs), lens,
                            len(bufs), sizes, offset, int(is_v6), C.byref(n))
    return rc, n.value, list(sizes)


def handle_gro(bufs: list, lens: list, offset: int, can_udp_gro: bool):
    """Oracle handleGRO.  bufs: list of numpy uint8 arrays (capacity = len(array)),
    lens: slice lengths.  Returns (rc, to_write, order, lens) where `order[i]` is
    the index of the original numpy buffer now at position i (prepends swap)."""
    n = len(bufs)
    u8p = C.POINTER(C.c_uint8)
    arr = _bufs_ctypes(bufs)
    orig = {b.ctypes.data: i for i, b in enumerate(bufs)}
    clens = (C.c_size_t * n)(*lens)
    ccaps = (C.c_size_t * n)(*[len(b) for b in bufs])
    tw = (C.c_int * n)()
    ntw = C.c_int(0)
    rc = lib().or_handle_gro(arr, clens, ccaps, n, offset, int(can_udp_gro), tw, C.byref(ntw))
    addrs = C.cast(arr, C.POINTER(C.c_void_p))
    order = [orig[addrs[i]] for i in range(n)]
    return rc, list(tw)[: ntw.value], order, list(clens)


# ---------------------------------------------------------------------------
# Independent closed form: checksum(b, init) ==
#   S == 0 ? 0 : 1 + (S - 1) mod 0xFFFF,  S = sum of big-endian u16 words
#   (odd tail zero-padded) + init, as a plain integer.
# ---------------------------------------------------------------------------
def closed_form_checksum(b: bytes, initial: int = 0) -> int:
    b = bytes(b)
    if len(b) % 2:
        b += b"\0"
    s = int(np.frombuffer(b, dtype=">u2").astype(np.uint64).sum()) + initial
    return 0 if s == 0 else 1 + (s - 1) % 0xFFFF


# ---------------------------------------------------------------------------
# Outer-UDP message batching (conn/bind.go:542-662, conn/gso.go:35-100),
# wg_oracle_conn.c.  Messages are duck-typed: .buf (numpy uint8, cap = len),
# .buf_len, .n, .oob (numpy uint8, cap = len), .oob_len, .nn, .addr.
# ---------------------------------------------------------------------------
class _OrMsg(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("buf_len", C.c_size_t), ("buf_cap", C.c_size_t), ("n", C.c_int),
                ("oob", C.c_void_p), ("oob_len", C.c_size_t), ("oob_cap", C.c_size_t), ("nn", C.c_int),
                ("addr", C.c_int)]


def _conn_lib():
    L = lib()
    if not getattr(L, "_conn_ready", False):
        L.or_get_gso_size.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_int)]
        L.or_get_gso_size.restype = C.c_int
        L.or_set_gso_size.argtypes = [C.c_void_p, C.POINTER(C.c_size_t), C.c_size_t, C.c_uint16]
        L.or_set_gso_size.restype = None
        L.or_split_messages.argtypes = [C.POINTER(_OrMsg), C.c_int, C.c_int, C.POINTER(C.c_int)]
        L.or_split_messages.restype = C.c_int
        L.or_coalesce_messages.argtypes = [C.POINTER(_OrMsg), C.c_int, C.POINTER(C.c_void_p),
                                           C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.c_int, C.c_int,
                                           C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_int)]
        L.or_coalesce_messages.restype = C.c_int
        L._conn_ready = True
    return L


def get_gso_size(control: bytes):
    """getGSOSize -> (gso, rc)."""
    a = np.frombuffer(bytes(control) + b"\0", dtype=np.uint8)
    g = C.c_int(0)
    rc = _conn_lib().or_get_gso_size(_ptr(a), len(control), C.byref(g))
    return g.value, rc


def set_gso_size(oob: np.ndarray, oob_len: int, gso: int) -> int:
    """setGSOSize on oob[:oob_len] (cap len(oob)); returns the new length."""
    ln = C.c_size_t(oob_len)
    _conn_lib().or_set_gso_size(_ptr(oob), C.byref(ln), len(oob), gso & 0xFFFF)
    return ln.value


def split_messages(msgs: list, first_msg_at: int):
    """splitMessages(msgs, firstMsgAt) -> (n_packets, rc); mutates msgs (addr
    becomes the Addr of the source message, as an index into the original addrs)."""
    n = len(msgs)
    arr = (_OrMsg * n)()
    for i, m in enumerate(msgs):
        arr[i] = _OrMsg(m.buf.ctypes.data, len(m.buf), len(m.buf), m.n, m.oob.ctypes.data, m.oob_len,
                        len(m.oob), m.nn, i)
    npk = C.c_int(0)
    rc = _conn_lib().or_split_messages(arr, n, first_msg_at, C.byref(npk))
    addrs = [m.addr for m in msgs]
    for i, m in enumerate(msgs):
        m.n = arr[i].n
        m.addr = addrs[arr[i].addr]
    return npk.value, rc


def coalesce_messages(msgs: list, bufs: list, lens: list, src_control: bytes, addr, dst_is_v6: bool):
    """coalesceMessages -> n_msgs; msgs[m].buf aliases the run's first buffer,
    msgs[m].buf_len its new length, msgs[m].oob/oob_len set as the reference does."""
    nb = len(bufs)
    arr = (_OrMsg * len(msgs))()
    for i, m in enumerate(msgs):
        arr[i] = _OrMsg(None, 0, 0, m.n, m.oob.ctypes.data, m.oob_len, len(m.oob), m.nn, -1)
    cb = (C.c_void_p * max(nb, 1))(*[b.ctypes.data for b in bufs])
    cl = (C.c_size_t * max(nb, 1))(*lens)
    cc = (C.c_size_t * max(nb, 1))(*[len(b) for b in bufs])
    sc = np.frombuffer(bytes(src_control) + b"\0", dtype=np.uint8)
    nm = C.c_int(0)
    rc = _conn_lib().or_coalesce_messages(arr, len(msgs), cb, cl, cc, nb, int(dst_is_v6), _ptr(sc),
                                          len(src_control), 0, C.byref(nm))
    assert rc == 0, rc
    index = {b.ctypes.data: j for j, b in enumerate(bufs)}
    for m in range(nm.value):
        msgs[m].buf = bufs[index[arr[m].buf]]
        msgs[m].buf_len = arr[m].buf_len
        msgs[m].oob_len = arr[m].oob_len
        msgs[m].addr = addr
    return nm.value
