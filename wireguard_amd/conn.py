"""Host-side mirror of the reference's outer-UDP message batching (package
`conn`) over the C ABI -- SURVEY.md §8f row 3.

Names, argument meaning and error behaviour follow /root/reference/conn:
  get_gso_size(control)                     conn/gso.go:35-67
  set_gso_size(msg, gso_size)               conn/gso.go:71-100
  split_messages(dev, msgs, first_msg_at)   conn/bind.go:542-597
  coalesce_messages(dev, msgs, bufs, lens, src_control, addr, dst_is_v6)
                                            conn/bind.go:599-662
A `Message` stands for golang.org/x/net/ipv6.Message with one buffer:
`buf` (numpy uint8, len == cap, like device/receive.go:119's bufs[i]),
`buf_len` (len(Buffers[0]) where it differs from cap: coalesce),
`n`, `oob` (numpy uint8 of the OOB capacity) + `oob_len`, `nn`, `addr`.
Every payload byte moves in the gfx950 kernels of libwgcsum.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import WgcsError

BATCH_SIZE = 128  # conn/conn.go:14
MAX_UDP_SEGMENTS = 64  # conn/bind.go:36
MAX_IPV4_PAYLOAD_LEN = (1 << 16) - 1 - 20 - 8  # conn/bind.go:25
MAX_IPV6_PAYLOAD_LEN = (1 << 16) - 1 - 8  # conn/bind.go:28
STICKY_CONTROL_SIZE = 16 + 24  # CmsgSpace(SizeofInet6Pktinfo = 20), conn/sticky.go:42
GSO_CONTROL_SIZE = 16 + 8  # CmsgSpace(2), conn/gso.go:22

__all__ = ["Message", "get_gso_size", "set_gso_size", "split_messages", "coalesce_messages", "udp_gro_cmsg",
           "BATCH_SIZE", "MAX_UDP_SEGMENTS", "MAX_IPV4_PAYLOAD_LEN", "MAX_IPV6_PAYLOAD_LEN"]


class Message:
    """ipv6.Message with a single buffer (conn/bind.go:91-99 pool layout)."""

    def __init__(self, buf: np.ndarray | None = None, oob_cap: int = STICKY_CONTROL_SIZE + GSO_CONTROL_SIZE):
        self.buf = buf
        self.buf_len = 0 if buf is None else len(buf)
        self.n = 0
        self.oob = np.zeros(oob_cap, dtype=np.uint8)
        self.oob_len = 0
        self.nn = 0
        self.addr = None


def udp_gro_cmsg(gso_size: int) -> bytes:
    """The SOL_UDP/UDP_GRO control message the kernel attaches to a GRO datagram
    (what getGSOSize looks for): Cmsghdr{Len=18, Level=17, Type=104} + u16 + pad."""
    return (18).to_bytes(8, "little") + (17).to_bytes(4, "little") + (104).to_bytes(4, "little") + \
        int(gso_size).to_bytes(2, "little") + b"\0" * 6


def _u8(a) -> np.ndarray:
    if isinstance(a, np.ndarray):
        return a
    return np.frombuffer(bytes(a) + b"\0", dtype=np.uint8)


def get_gso_size(control) -> tuple[int, WgcsError | None]:
    """getGSOSize(control []byte) (int, error)."""
    lib = _lib.load()
    a = _u8(control)
    n = len(control)
    g = C.c_int(0)
    rc = lib.wgcs_get_gso_size(a.ctypes.data if n else None, n, C.byref(g))
    return g.value, (WgcsError(rc, lib.wgcs_strerror(rc).decode()) if rc else None)


def set_gso_size(msg: Message, gso_size: int) -> None:
    """setGSOSize(&msg.OOB, gsoSize): appends UDP_SEGMENT if it fits."""
    lib = _lib.load()
    ln = C.c_size_t(msg.oob_len)
    rc = lib.wgcs_set_gso_size(msg.oob.ctypes.data, C.byref(ln), len(msg.oob), gso_size & 0xFFFF)
    if rc:
        raise WgcsError(rc, lib.wgcs_strerror(rc).decode())
    msg.oob_len = ln.value


def _ptrs(arrs):
    u8p = C.POINTER(C.c_uint8)
    out = (u8p * len(arrs))()
    for i, a in enumerate(arrs):
        out[i] = C.cast(a.ctypes.data, u8p) if a is not None else None
    return out


def split_messages(dev, msgs: list[Message], first_msg_at: int) -> tuple[int, WgcsError | None]:
    """splitMessages(msgs, firstMsgAt) (nPackets int, err error).  Mutates
    msgs[i].buf / .n / .addr as the reference does."""
    n = len(msgs)
    buf_len = len(msgs[0].buf)
    if any(len(m.buf) != buf_len for m in msgs):
        raise ValueError("split_messages: all message buffers must have the same length")
    bufs = _ptrs([m.buf for m in msgs])
    ns = (C.c_int * n)(*[m.n for m in msgs])
    oobs = _ptrs([m.oob for m in msgs])
    nns = (C.c_size_t * n)(*[m.nn for m in msgs])
    src = (C.c_int * n)()
    npk = C.c_int(0)
    rc = dev.lib.wgcs_split_messages(dev.h, bufs, buf_len, ns, oobs, nns, n, first_msg_at, src, C.byref(npk))
    addrs = [m.addr for m in msgs]
    for k, m in enumerate(msgs):
        m.n = ns[k]
        m.addr = addrs[src[k]]
    return npk.value, dev._err(rc)


def coalesce_messages(dev, msgs: list[Message], bufs: list[np.ndarray], lens: list[int], src_control: bytes,
                      addr, dst_is_v6: bool) -> int:
    """coalesceMessages(msgs, bufs, endpoint, addr) int.  bufs[j] is a numpy
    array of cap(bufs[j]) bytes holding len = lens[j]; appends land in the
    first buffer of each run.  msgs[m].buf aliases that buffer afterwards, with
    msgs[m].buf_len its new length; msgs[m].oob gets setSrcControl + setGSOSize."""
    nb = len(bufs)
    if nb == 0:
        return 0
    if len(msgs) < nb:
        raise ValueError("coalesce_messages: need len(msgs) >= len(bufs)")
    cb = _ptrs(bufs)
    clens = (C.c_size_t * nb)(*lens)
    ccaps = (C.c_size_t * nb)(*[len(b) for b in bufs])
    oobs = _ptrs([msgs[m].oob for m in range(nb)])
    olens = (C.c_size_t * nb)(*[msgs[m].oob_len for m in range(nb)])
    ocaps = (C.c_size_t * nb)(*[len(msgs[m].oob) for m in range(nb)])
    first = (C.c_int * nb)()
    mlen = (C.c_size_t * nb)()
    nm = C.c_int(0)
    sc = _u8(src_control)
    rc = dev.lib.wgcs_coalesce_messages(dev.h, cb, clens, ccaps, nb, int(dst_is_v6),
                                        sc.ctypes.data if len(src_control) else None, len(src_control), oobs, olens,
                                        ocaps, first, mlen, C.byref(nm))
    dev._check(rc)
    for m in range(nm.value):
        msgs[m].buf = bufs[first[m]]
        msgs[m].buf_len = mlen[m]
        msgs[m].oob_len = olens[m]
        msgs[m].addr = addr
    return nm.value
