"""TEST INFRASTRUCTURE ONLY -- a second, independent CPU restatement of the
reference's GSO / GRO path, in pure Python, written straight from the Go text
(it is NOT a translation of wg_oracle.c, and it shares no code with it):

  checksumNoFold / checksum / pseudoHeaderChecksumNoFold  tun/checksum.go:8-167
  checksumValid                                           tun/gro.go:554-612
  gsoSplit / gsoNoneChecksum                              tun/gro.go:1373-1517
  handleVirtioRead                                        tun/tun.go:514-632
  handleGRO, tcpGRO, udpGRO, coalesce*, apply*            tun/gro.go:95-376, 388-544, 614-1367

Purpose: the reference cannot run here (no Go toolchain,
no vectors in the reference), so oracle/wg_oracle.c -- which every GPU test
compares against -- is cross-checked by this second formulation on the GSO
header-fuzz corpus and the GRO call corpus (tests/test_py_restatement.py).  A
misreading of gro.go shared by the C oracle and the kernels would show up as a
disagreement here.  Only tests/ import this module.

Go semantics modelled explicitly:
  - `Slice` is a Go []byte: a backing array, a start, len and cap.  Slicing
    may reach up to cap (not len), indexing only below len, and anything else
    raises GoPanic -- the reference's runtime panic (the C ABI maps it to
    WGCS_ERR_OUT_OF_RANGE).  append() within cap writes into the same backing
    array, as Go does; the paths restated here never append past cap.
  - uint8 / uint16 / uint32 arithmetic wraps where the Go expression's type
    does (masks are written at each such expression, with the line).
  - Go maps keyed by structs become dicts keyed by tuples.  Their iteration
    order only matters in apply*, where every item writes its own buffer.
"""
from __future__ import annotations

import numpy as np

M16, M32, M64 = 0xFFFF, 0xFFFFFFFF, (1 << 64) - 1

# status codes, as include/wgcsum.h maps the reference's errors
OK = 0
ERR_SHORT_BUFFER = -2          # io.ErrShortBuffer                   gro.go:75, :86
ERR_TOO_MANY_SEGMENTS = -3     # ErrTooManySegments                  gro.go:1410
ERR_INVALID_OFFSET = -4        # errors.New("invalid offset")        gro.go:1336
ERR_UNSUPPORTED_GSO = -5       # tun.go:567
ERR_IP_GSO_MISMATCH = -6       # tun.go:575, :584
ERR_BAD_IP_VERSION = -7        # tun.go:591
ERR_PACKET_TOO_SHORT = -8      # tun.go:603
ERR_TCP_HDR_LEN = -9           # tun.go:611
ERR_HDR_LEN = -10              # tun.go:616
ERR_CSUM_OFFSET = -11          # tun.go:625
ERR_READ_OVERFLOW = -12        # tun.go:546
ERR_OUT_OF_RANGE = -13         # a Go runtime panic (slice / index out of range)

# golang.org/x/sys/unix constants (Linux UAPI values)
IPPROTO_TCP, IPPROTO_UDP = 6, 17
VIRTIO_NET_HDR_F_NEEDS_CSUM = 1
GSO_NONE, GSO_TCPV4, GSO_TCPV6, GSO_UDP_L4 = 0, 1, 4, 5
VIRTIO_NET_HDR_LEN = 10  # gro.go:71
TCP_FLAGS_OFFSET = 13    # gro.go:25
TCP_FIN, TCP_PSH, TCP_ACK = 0x01, 0x08, 0x10  # gro.go:35-39
UDPH_LEN = 8             # gro.go:249
IPV4_SRC, IPV6_SRC = 12, 8  # gro.go:547-548
MAX_UINT16 = (1 << 16) - 1  # gro.go:550
IPV4_FLAG_MF = 0x20      # gro.go:785


class GoPanic(Exception):
    """The Go runtime would panic here (index or slice bounds out of range)."""


class Slice:
    """A Go []byte over a numpy uint8 backing array."""
    __slots__ = ("a", "off", "n", "cap")

    def __init__(self, a: np.ndarray, off: int = 0, n: int | None = None, cap: int | None = None):
        self.a = a
        self.off = off
        self.cap = len(a) - off if cap is None else cap
        self.n = self.cap if n is None else n

    def __len__(self):
        return self.n

    def s(self, lo: int = 0, hi: int | None = None) -> "Slice":
        """s[lo:hi] (hi defaults to len): 0 <= lo <= hi <= cap, else a panic."""
        if hi is None:
            hi = self.n
        if not (0 <= lo <= hi <= self.cap):
            raise GoPanic(f"slice bounds out of range [{lo}:{hi}] with capacity {self.cap}")
        return Slice(self.a, self.off + lo, hi - lo, self.cap - lo)

    def __getitem__(self, i: int) -> int:
        if not 0 <= i < self.n:
            raise GoPanic(f"index out of range [{i}] with length {self.n}")
        return int(self.a[self.off + i])

    def __setitem__(self, i: int, v: int) -> None:
        if not 0 <= i < self.n:
            raise GoPanic(f"index out of range [{i}] with length {self.n}")
        self.a[self.off + i] = v & 0xFF

    def view(self) -> np.ndarray:
        return self.a[self.off: self.off + self.n]

    def same_array(self, other: "Slice") -> bool:
        return self.a is other.a


def gcopy(dst: Slice, src) -> int:
    """copy(dst, src): min(len) bytes, overlapping ranges allowed."""
    sv = src.view() if isinstance(src, Slice) else np.asarray(src, np.uint8)
    k = min(len(dst), len(sv))
    if k:
        dst.a[dst.off: dst.off + k] = sv[:k].copy()
    return k


def gappend_zeros(b: Slice, k: int) -> Slice:
    """append(b, make([]byte, k)...) for k bytes that fit cap(b) (every
    append of the restated paths does: their capacity checks come first)."""
    if b.n + k > b.cap:
        raise AssertionError("append past cap would reallocate; not a path of the reference restated here")
    b.a[b.off + b.n: b.off + b.n + k] = 0
    return Slice(b.a, b.off, b.n + k, b.cap)


def be16(b: Slice, i: int) -> int:
    """binary.BigEndian.Uint16(b[i:])."""
    t = b.s(i)
    return (t[0] << 8) | t[1]


def be32(b: Slice, i: int) -> int:
    t = b.s(i)
    return (t[0] << 24) | (t[1] << 16) | (t[2] << 8) | t[3]


def put_be16(b: Slice, i: int, v: int) -> None:
    """binary.BigEndian.PutUint16(b[i:], v): `_ = b[1]` first, as Go's does."""
    t = b.s(i)
    _ = t[1]
    t[0] = (v >> 8) & 0xFF
    t[1] = v & 0xFF


def put_be32(b: Slice, i: int, v: int) -> None:
    t = b.s(i)
    _ = t[3]
    for k in range(4):
        t[k] = (v >> (24 - 8 * k)) & 0xFF


def le16(b: Slice, i: int) -> int:
    """binary.NativeEndian.Uint16 on little-endian (amd64 / arm64)."""
    t = b.s(i)
    return t[0] | (t[1] << 8)


def _bswap64(v: int) -> int:
    return int.from_bytes((v & M64).to_bytes(8, "little"), "big")


# --------------------------------------------------------------- checksum.go
def checksum_no_fold(b, initial: int) -> int:
    """checksumNoFold(b, initial), tun/checksum.go:8-120.

    :39-41 and :118-119 swap the accumulator between native (little) and big
    endian.  :44-104 add b's native-endian u64 words (the 128/64/32/16/8-byte
    blocks cover len(b) & ~7 bytes in order), then its u32 and u16 tail, and
    :105-117 the last odd byte zero-padded ({b0, 0} read as native u16 = b0).
    Each block is a bits.Add64 carry chain closed by `ac += carry`: the carry
    out of a step is the carry in of the next, and the last is added back, so
    the block returns R = S - (2^64-1) * C for S = ac + the block's words and
    C carries.  A carry out implies the sum left ac <= 2^64-2 (induction from
    the first step, whose carry-in is 0), so `ac += carry` never wraps and
    0 <= R <= 2^64-1; R == 0 only if S == 0.  So every block maps S to
    0 if S == 0 else 1 + (S-1) mod (2^64-1), and that map composes over blocks
    (it keeps S mod 2^64-1 and whether S is 0): one sum over all words gives
    the same accumulator.  (`checksum_no_fold_adc` below restates the chain
    step by step; tests check the two against each other.)"""
    v = b.view() if isinstance(b, Slice) else np.frombuffer(bytes(b), np.uint8)
    n = len(v)
    n8 = n & ~7
    s = _bswap64(initial)
    if n8:
        w = v[:n8].view("<u4").astype(np.uint64)  # u64 words as lo + hi << 32, exact in Python ints
        s += int(w[0::2].sum()) + (int(w[1::2].sum()) << 32)
    r = v[n8:]
    if len(r) >= 4:
        s += int(r[0]) | int(r[1]) << 8 | int(r[2]) << 16 | int(r[3]) << 24
        r = r[4:]
    if len(r) >= 2:
        s += int(r[0]) | int(r[1]) << 8
        r = r[2:]
    if len(r) == 1:
        s += int(r[0])
    ac = 0 if s == 0 else 1 + (s - 1) % M64
    return _bswap64(ac)


def checksum_no_fold_adc(b: bytes, initial: int) -> int:
    """checksum.go:8-120 step by step (bits.Add64 chains, block by block)."""
    b = bytes(b)
    ac = _bswap64(initial)

    def add64(x, y, c):
        t = x + y + c
        return t & M64, t >> 64

    def block(ac, words):
        carry = 0
        for k, w in enumerate(words):
            ac, carry = add64(ac, w, 0 if k == 0 else carry)
        return (ac + carry) & M64  # `ac += carry` (plain uint64 add)

    def u64s(x):
        return [int.from_bytes(x[k:k + 8], "little") for k in range(0, len(x), 8)]

    while len(b) >= 128:
        ac = block(ac, u64s(b[:128]))
        b = b[128:]
    for size in (64, 32, 16, 8):
        if len(b) >= size:
            ac = block(ac, u64s(b[:size]))
            b = b[size:]
    if len(b) >= 4:
        ac = block(ac, [int.from_bytes(b[:4], "little")])
        b = b[4:]
    if len(b) >= 2:
        ac = block(ac, [int.from_bytes(b[:2], "little")])
        b = b[2:]
    if len(b) == 1:
        ac = block(ac, [b[0]])
    return _bswap64(ac)


def checksum(b, initial: int) -> int:
    """checksum(b, initial) uint16, tun/checksum.go:152-167: four folds, no complement."""
    ac = checksum_no_fold(b, initial)
    for _ in range(4):
        ac = (ac >> 16) + (ac & 0xFFFF)
    return ac & M16


def pseudo_header_checksum_no_fold(src, dst, protocol: int, total_len: int) -> int:
    """tun/checksum.go:127-150."""
    s = checksum_no_fold(src, 0)
    s = checksum_no_fold(dst, s)
    s = checksum_no_fold(bytes([0, protocol & 0xFF]), s)
    return checksum_no_fold((total_len & M16).to_bytes(2, "big"), s)


def checksum_valid(pkt: Slice, iph_len: int, protocol: int, is_v6: bool) -> bool:
    """checksumValid, tun/gro.go:554-612.  The address slices may reach into
    pkt's spare capacity (a slice up to cap is legal Go)."""
    at, size = (IPV6_SRC, 16) if is_v6 else (IPV4_SRC, 4)
    src = pkt.s(at, at + size)
    dst = pkt.s(at + size, at + 2 * size)
    total_len = (len(pkt) - iph_len) & M16  # uint16(len(pkt) - int(iphLen)), :564
    hc = pseudo_header_checksum_no_fold(src, dst, protocol, total_len)
    return (~checksum(pkt.s(iph_len), hc)) & M16 == 0


# ------------------------------------------------------------ virtioNetHdr
class VirtioHdr:
    """gro.go:42-67; encode/decode (:73-93) copy its 10 bytes in native
    (little-endian) order: u8 flags, u8 gsoType, u16 hdrLen, gsoSize,
    csumStart, csumOffset."""
    __slots__ = ("flags", "gso_type", "hdr_len", "gso_size", "csum_start", "csum_offset")

    def __init__(self, flags=0, gso_type=0, hdr_len=0, gso_size=0, csum_start=0, csum_offset=0):
        self.flags, self.gso_type = flags & 0xFF, gso_type & 0xFF
        self.hdr_len, self.gso_size = hdr_len & M16, gso_size & M16
        self.csum_start, self.csum_offset = csum_start & M16, csum_offset & M16

    def encode(self, b: Slice) -> int:
        if len(b) < VIRTIO_NET_HDR_LEN:
            return ERR_SHORT_BUFFER
        raw = bytes([self.flags, self.gso_type]) + b"".join(
            v.to_bytes(2, "little") for v in (self.hdr_len, self.gso_size, self.csum_start, self.csum_offset))
        gcopy(b.s(0, VIRTIO_NET_HDR_LEN), np.frombuffer(raw, np.uint8))
        return OK

    @classmethod
    def decode(cls, b: Slice):
        if len(b) < VIRTIO_NET_HDR_LEN:
            return None, ERR_SHORT_BUFFER
        return cls(b[0], b[1], le16(b, 2), le16(b, 4), le16(b, 6), le16(b, 8)), OK


# ------------------------------------------------------------------ GSO side
def gso_split(read_buf: Slice, hdr: VirtioHdr, bufs: list, sizes: list, offset: int, is_v6: bool):
    """gsoSplit, tun/gro.go:1373-1493 -> (n, status)."""
    iph_len = hdr.csum_start                                       # :1381
    src_off, addr_len = IPV6_SRC, 16                               # :1382-1383
    if not is_v6:
        src_off, addr_len = IPV4_SRC, 4
        read_buf[10] = 0                                           # :1388
        read_buf[11] = 0
    checksum_at = (hdr.csum_start + hdr.csum_offset) & M16         # :1391 (uint16 sum)
    read_buf[checksum_at] = 0                                      # :1393
    read_buf[checksum_at + 1] = 0
    first_seq = 0
    if hdr.gso_type in (GSO_TCPV4, GSO_TCPV6):                     # :1398-1405
        protocol = IPPROTO_TCP
        first_seq = be32(read_buf, (hdr.csum_start + 4) & M16)
    else:
        protocol = IPPROTO_UDP
    nxt = hdr.hdr_len                                              # :1406
    i = 0
    while nxt < len(read_buf):                                     # :1408
        if i == len(bufs):
            return i - 1, ERR_TOO_MANY_SEGMENTS                    # :1409-1410
        seg_end = min(nxt + hdr.gso_size, len(read_buf))           # :1412-1413
        seg_len = seg_end - nxt
        pkt_len = hdr.hdr_len + seg_len                            # :1415
        sizes[i] = pkt_len
        pkt = bufs[i].s(offset)                                    # :1417
        gcopy(pkt, read_buf.s(0, iph_len))                         # :1419
        if not is_v6:
            if i > 0:                                              # :1426-1431 (id0 + 1 for every i >= 1)
                put_be16(pkt, 4, (be16(pkt, 4) + 1) & M16)
            put_be16(pkt, 2, pkt_len & M16)                        # :1433
            put_be16(pkt, 10, ~checksum(pkt.s(0, iph_len), 0) & M16)  # :1434-1436
        else:
            put_be16(pkt, 4, (pkt_len - iph_len) & M16)            # :1439
        gcopy(pkt.s(hdr.csum_start, hdr.hdr_len), read_buf.s(hdr.csum_start, hdr.hdr_len))  # :1442
        if protocol == IPPROTO_TCP:
            seq = (first_seq + ((hdr.gso_size * i) & M16)) & M32   # :1445 uint32(hdr.gsoSize*uint16(i))
            put_be32(pkt, (hdr.csum_start + 4) & M16, seq)
            if seg_end != len(read_buf):                           # :1447-1459
                fa = (hdr.csum_start + TCP_FLAGS_OFFSET) & M16
                pkt[fa] = pkt[fa] & ~(TCP_FIN | TCP_PSH)
        else:
            put_be16(pkt, (hdr.csum_start + 4) & M16,              # :1462-1465
                     ((seg_len & M16) + ((hdr.hdr_len - hdr.csum_start) & M16)) & M16)
        gcopy(pkt.s(hdr.hdr_len), read_buf.s(nxt, seg_end))        # :1468
        th_len = (hdr.hdr_len - hdr.csum_start) & M16              # :1469 int(hdr.hdrLen - hdr.csumStart)
        t_len = (th_len + seg_len) & M16                           # :1471
        ph = pseudo_header_checksum_no_fold(read_buf.s(src_off, src_off + addr_len),
                                            read_buf.s(src_off + addr_len, src_off + 2 * addr_len),
                                            protocol, t_len)       # :1472-1478
        tc = ~checksum(pkt.s(hdr.csum_start, pkt_len), ph) & M16   # :1480-1483
        put_be16(pkt, (hdr.csum_start + hdr.csum_offset) & M16, tc)  # :1485-1488
        nxt += hdr.gso_size                                        # :1489
        i += 1
    return i, OK


def gso_none_checksum(read_buf: Slice, checksum_start: int, checksum_offset: int) -> int:
    """gsoNoneChecksum, tun/gro.go:1497-1517."""
    at = (checksum_start + checksum_offset) & M16                  # :1503 (uint16)
    initial = be16(read_buf, at)                                   # :1508
    read_buf[at] = 0                                               # :1510
    read_buf[at + 1] = 0
    put_be16(read_buf, at, ~checksum(read_buf.s(checksum_start), initial) & M16)  # :1512-1515
    return OK


def handle_virtio_read(read_buf: Slice, bufs: list, sizes: list, offset: int):
    """handleVirtioRead, tun/tun.go:514-632 -> (n, status)."""
    hdr, rc = VirtioHdr.decode(read_buf)                           # :522-525
    if rc:
        return 0, rc
    read_buf = read_buf.s(VIRTIO_NET_HDR_LEN)                      # :527
    if hdr.gso_type == GSO_NONE:                                   # :532-556
        if hdr.flags & VIRTIO_NET_HDR_F_NEEDS_CSUM:
            rc = gso_none_checksum(read_buf, hdr.csum_start, hdr.csum_offset)
            if rc:
                return 0, rc
        if len(read_buf) > len(bufs[0].s(offset)):
            return 0, ERR_READ_OVERFLOW
        sizes[0] = gcopy(bufs[0].s(offset), read_buf)
        return 1, OK
    if hdr.gso_type not in (GSO_TCPV4, GSO_TCPV6, GSO_UDP_L4):     # :564-568
        return 0, ERR_UNSUPPORTED_GSO
    ip_version = read_buf[0] >> 4                                  # :570
    if ip_version == 4:
        if hdr.gso_type not in (GSO_TCPV4, GSO_UDP_L4):
            return 0, ERR_IP_GSO_MISMATCH
    elif ip_version == 6:
        if hdr.gso_type not in (GSO_TCPV6, GSO_UDP_L4):
            return 0, ERR_IP_GSO_MISMATCH
    else:
        return 0, ERR_BAD_IP_VERSION
    if hdr.gso_type == GSO_UDP_L4:                                 # :597-614
        hdr.hdr_len = (hdr.csum_start + 8) & M16
    else:
        at = (hdr.csum_start + 12) & M16
        if len(read_buf) <= at:
            return 0, ERR_PACKET_TOO_SHORT
        tcp_hlen = ((read_buf[at] >> 4) * 4) & 0xFF                # :608 (uint8 >> 4 * 4)
        if tcp_hlen < 20 or tcp_hlen > 60:
            return 0, ERR_TCP_HDR_LEN
        hdr.hdr_len = (hdr.csum_start + tcp_hlen) & M16
    if len(read_buf) < hdr.hdr_len:                                # :615-621
        return 0, ERR_HDR_LEN
    checksum_at = (hdr.csum_start + hdr.csum_offset) & M16         # :622
    if checksum_at + 1 >= len(read_buf):                           # :624-630
        return 0, ERR_CSUM_OFFSET
    return gso_split(read_buf, hdr, bufs, sizes, offset, ip_version == 6)


def _np_slices(bufs):
    return [Slice(b) for b in bufs]


def run_handle_virtio_read(read_buf: np.ndarray, bufs: list, offset: int, n_read: int | None = None):
    """oracle.handle_virtio_read's interface: mutates read_buf and the numpy
    bufs in place; returns (rc, n, sizes).  A Go panic is (OUT_OF_RANGE, 0, sizes).
    With n_read, readBuf is read_buf[:n_read] with capacity len(read_buf)."""
    sizes = [0] * len(bufs)
    try:
        n, rc = handle_virtio_read(Slice(read_buf, 0, n_read), _np_slices(bufs), sizes, offset)
    except GoPanic:
        return ERR_OUT_OF_RANGE, 0, sizes
    return rc, n, sizes


def run_gso_split(read_buf: np.ndarray, hdr: tuple, bufs: list, offset: int, is_v6: bool,
                  n_read: int | None = None):
    """oracle.gso_split's interface (hdr = the six virtio header fields)."""
    sizes = [0] * len(bufs)
    try:
        n, rc = gso_split(Slice(read_buf, 0, n_read), VirtioHdr(*hdr), _np_slices(bufs), sizes, offset, is_v6)
    except GoPanic:
        return ERR_OUT_OF_RANGE, 0, sizes
    return rc, n, sizes


# ------------------------------------------------------------------ GRO side
class TcpItem:
    """tcpGROItem, gro.go:131-149."""
    __slots__ = ("key", "seq_num", "bufs_index", "num_merged", "gso_size", "iph_len", "tcph_len", "psh_set")

    def copy(self) -> "TcpItem":
        c = TcpItem()
        for k in self.__slots__:
            setattr(c, k, getattr(self, k))
        return c


class UdpItem:
    """udpGROItem, gro.go:279-293."""
    __slots__ = ("key", "bufs_index", "num_merged", "gso_size", "iph_len", "csum_known_invalid")

    def copy(self) -> "UdpItem":
        c = UdpItem()
        for k in self.__slots__:
            setattr(c, k, getattr(self, k))
        return c


def _addr16(pkt: Slice, a: int, b: int) -> bytes:
    """copy(key.srcAddr[:], pkt[a:b]) into a zeroed [16]byte."""
    return bytes(pkt.s(a, b).view()).ljust(16, b"\0")[:16]


def new_tcp_flow_key(pkt: Slice, src_off: int, dst_off: int, tcph_off: int):
    """newTCPFlowKey, gro.go:111-127."""
    addr_size = dst_off - src_off
    return (_addr16(pkt, src_off, dst_off), _addr16(pkt, dst_off, dst_off + addr_size), be16(pkt, tcph_off),
            be16(pkt, tcph_off + 2), be32(pkt, tcph_off + 8), addr_size == 16)


def new_udp_flow_key(pkt: Slice, src_off: int, dst_off: int, udph_off: int):
    """newUDPFlowKey, gro.go:261-275."""
    addr_size = dst_off - src_off
    return (_addr16(pkt, src_off, dst_off), _addr16(pkt, dst_off, dst_off + addr_size), be16(pkt, udph_off),
            be16(pkt, udph_off + 2), addr_size == 16)


class TcpTable:
    """tcpGROTable, gro.go:151-247 (itemsByFlow; the pool is an allocation detail)."""

    def __init__(self):
        self.items_by_flow: dict = {}

    def get_or_insert(self, pkt, src_off, dst_off, tcph_off, tcph_len, bufs_index):  # :189-204
        key = new_tcp_flow_key(pkt, src_off, dst_off, tcph_off)
        items = self.items_by_flow.get(key)
        if items is not None:
            return items, True
        self.insert(pkt, src_off, dst_off, tcph_off, tcph_len, bufs_index)
        return None, False

    def insert(self, pkt, src_off, dst_off, tcph_off, tcph_len, bufs_index):  # :207-232
        it = TcpItem()
        it.key = new_tcp_flow_key(pkt, src_off, dst_off, tcph_off)
        it.bufs_index = bufs_index & M16
        it.num_merged = 0
        it.gso_size = len(pkt.s(tcph_off + tcph_len)) & M16
        it.iph_len = tcph_off & 0xFF
        it.tcph_len = tcph_len & 0xFF
        it.seq_num = be32(pkt, tcph_off + 4)
        it.psh_set = pkt[tcph_off + TCP_FLAGS_OFFSET] & TCP_PSH != 0
        self.items_by_flow.setdefault(it.key, []).append(it)

    def update_at(self, item, i):  # :234-239
        self.items_by_flow[item.key][i] = item

    def delete_at(self, key, i):  # :241-247
        del self.items_by_flow[key][i]


class UdpTable:
    """udpGROTable, gro.go:295-376."""

    def __init__(self):
        self.items_by_flow: dict = {}

    def get_or_insert(self, pkt, src_off, dst_off, udph_off, bufs_index):  # :332-346
        key = new_udp_flow_key(pkt, src_off, dst_off, udph_off)
        items = self.items_by_flow.get(key)
        if items is not None:
            return items, True
        self.insert(pkt, src_off, dst_off, udph_off, bufs_index, False)
        return None, False

    def insert(self, pkt, src_off, dst_off, udph_off, bufs_index, csum_known_invalid):  # :349-371
        it = UdpItem()
        it.key = new_udp_flow_key(pkt, src_off, dst_off, udph_off)
        it.bufs_index = bufs_index & M16
        it.num_merged = 0
        it.gso_size = len(pkt.s(udph_off + UDPH_LEN)) & M16
        it.iph_len = udph_off & 0xFF
        it.csum_known_invalid = csum_known_invalid
        self.items_by_flow.setdefault(it.key, []).append(it)

    def update_at(self, item, i):  # :373-376
        self.items_by_flow[item.key][i] = item


COALESCE_PREPEND, COALESCE_UNAVAILABLE, COALESCE_APPEND = -1, 0, 1  # gro.go:382-386
(INSUFFICIENT_CAP, PSH_ENDING, ITEM_INVALID_CSUM, PKT_INVALID_CSUM, COALESCE_SUCCESS) = range(5)  # :618-624
GRO_NOOP, GRO_TABLE_INSERT, GRO_COALESCED = range(3)  # :789-793


def ip_headers_can_coalesce(a: Slice, b: Slice) -> bool:
    """gro.go:392-427."""
    if len(a) < 9 or len(b) < 9:
        return False
    if a[0] >> 4 == 6:
        if a[0] != b[0] or a[1] >> 4 != b[1] >> 4:
            return False
        if a[7] != b[7]:
            return False
    else:
        if a[1] != b[1]:
            return False
        if a[6] >> 5 != b[6] >> 5:
            return False
        if a[8] != b[8]:
            return False
    return True


def tcp_packets_can_coalesce(pkt, iph_len, tcph_len, seq_num, psh_set, gso_size, item: TcpItem, bufs, offset):
    """gro.go:433-512."""
    target = bufs[item.bufs_index].s(offset)
    if tcph_len != item.tcph_len:
        return COALESCE_UNAVAILABLE
    if tcph_len > 20:
        if not np.array_equal(pkt.s(iph_len + 20, iph_len + tcph_len).view(),
                              target.s(item.iph_len + 20, iph_len + tcph_len).view()):
            return COALESCE_UNAVAILABLE
    if not ip_headers_can_coalesce(pkt, target):
        return COALESCE_UNAVAILABLE
    lhs_len = (item.gso_size + item.gso_size * item.num_merged) & M16  # :468 (uint16)
    if seq_num == (item.seq_num + lhs_len) & M32:
        if item.psh_set:
            return COALESCE_UNAVAILABLE
        if len(target.s(iph_len + tcph_len)) % item.gso_size != 0:
            return COALESCE_UNAVAILABLE
        if gso_size > item.gso_size:
            return COALESCE_UNAVAILABLE
        return COALESCE_APPEND
    elif (seq_num + gso_size) & M32 == item.seq_num:
        if psh_set:
            return COALESCE_UNAVAILABLE
        if gso_size < item.gso_size:
            return COALESCE_UNAVAILABLE
        if gso_size > item.gso_size and item.num_merged > 0:
            return COALESCE_UNAVAILABLE
        return COALESCE_PREPEND
    return COALESCE_UNAVAILABLE


def udp_packets_can_coalesce(pkt, iph_len, gso_size, item: UdpItem, bufs, offset):
    """gro.go:519-544."""
    target = bufs[item.bufs_index].s(offset)
    if not ip_headers_can_coalesce(pkt, target):
        return COALESCE_UNAVAILABLE
    if len(target.s(iph_len + UDPH_LEN)) % item.gso_size != 0:
        return COALESCE_UNAVAILABLE
    if gso_size > item.gso_size:
        return COALESCE_UNAVAILABLE
    return COALESCE_APPEND


def coalesce_tcp_packets(mode, pkt: Slice, pkt_bi, gso_size, seq_num, psh_set, item: TcpItem, bufs, offset, is_v6):
    """coalesceTCPPackets, gro.go:630-741.  May swap bufs entries (prepend)."""
    headers_len = (item.iph_len + item.tcph_len) & 0xFF           # :643 (uint8 sum)
    pkt_payload_len = len(pkt) - headers_len
    new_len = len(bufs[item.bufs_index].s(offset)) + pkt_payload_len
    if mode == COALESCE_PREPEND:
        pkt_head = pkt
        if pkt.cap < new_len:                                      # :652
            return INSUFFICIENT_CAP
        if psh_set:
            return PSH_ENDING
        if item.num_merged == 0:
            if not checksum_valid(bufs[item.bufs_index].s(offset), item.iph_len, IPPROTO_TCP, is_v6):
                return ITEM_INVALID_CSUM
        if not checksum_valid(pkt, item.iph_len, IPPROTO_TCP, is_v6):
            return PKT_INVALID_CSUM
        item.seq_num = seq_num                                     # :682
        item_payload_len = new_len - len(pkt_head)
        bufs[pkt_bi] = gappend_zeros(bufs[pkt_bi], item_payload_len)  # :685-688
        gcopy(bufs[pkt_bi].s(offset + len(pkt)), bufs[item.bufs_index].s(offset + headers_len))  # :690-693
        bufs[item.bufs_index], bufs[pkt_bi] = bufs[pkt_bi], bufs[item.bufs_index]  # :696-697
    else:
        pkt_head = bufs[item.bufs_index].s(offset)
        if pkt_head.cap < new_len:                                 # :701
            return INSUFFICIENT_CAP
        if item.num_merged == 0:
            if not checksum_valid(bufs[item.bufs_index].s(offset), item.iph_len, IPPROTO_TCP, is_v6):
                return ITEM_INVALID_CSUM
        if not checksum_valid(pkt, item.iph_len, IPPROTO_TCP, is_v6):
            return PKT_INVALID_CSUM
        if psh_set:                                                # :724-729
            item.psh_set = psh_set
            fa = item.iph_len + TCP_FLAGS_OFFSET
            pkt_head[fa] = pkt_head[fa] | TCP_PSH
        bufs[item.bufs_index] = gappend_zeros(bufs[item.bufs_index], pkt_payload_len)  # :730-733
        gcopy(bufs[item.bufs_index].s(offset + len(pkt_head)), pkt.s(headers_len))    # :734
    item.gso_size = max(item.gso_size, gso_size)                   # :738
    item.num_merged = (item.num_merged + 1) & M16
    return COALESCE_SUCCESS


def coalesce_udp_packets(pkt: Slice, item: UdpItem, bufs, offset, is_v6):
    """coalesceUDPPackets, gro.go:745-783."""
    pkt_head = bufs[item.bufs_index].s(offset)
    headers_len = (item.iph_len + UDPH_LEN) & 0xFF
    pkt_payload_len = len(pkt) - headers_len
    new_len = len(pkt_head) + pkt_payload_len
    if pkt_head.cap < new_len:                                     # :758
        return INSUFFICIENT_CAP
    if item.num_merged == 0:
        if item.csum_known_invalid or not checksum_valid(pkt_head, item.iph_len, IPPROTO_UDP, is_v6):
            return ITEM_INVALID_CSUM
    if not checksum_valid(pkt, item.iph_len, IPPROTO_UDP, is_v6):
        return PKT_INVALID_CSUM
    bufs[item.bufs_index] = gappend_zeros(bufs[item.bufs_index], pkt_payload_len)  # :776-779
    gcopy(bufs[item.bufs_index].s(offset + len(pkt_head)), pkt.s(headers_len))
    item.num_merged = (item.num_merged + 1) & M16
    return COALESCE_SUCCESS


def tcp_gro(bufs, offset, bufs_index, table: TcpTable, is_v6):
    """tcpGRO, gro.go:801-963."""
    pkt = bufs[bufs_index].s(offset)
    if len(pkt) > MAX_UINT16:
        return GRO_NOOP
    iph_len = (pkt[0] & 0x0F) * 4
    if is_v6:
        iph_len = 40
        if be16(pkt, 4) != len(pkt) - iph_len:
            return GRO_NOOP
    else:
        if be16(pkt, 2) != len(pkt):
            return GRO_NOOP
    if len(pkt) < iph_len:
        return GRO_NOOP
    tcph_len = (pkt[iph_len + 12] >> 4) * 4                        # :847
    if tcph_len < 20 or tcph_len > 60:
        return GRO_NOOP
    if len(pkt) < iph_len + tcph_len:
        return GRO_NOOP
    if not is_v6:
        if pkt[6] & IPV4_FLAG_MF != 0 or (pkt[6] << 3) & 0xFF != 0 or pkt[7] != 0:  # :858 (uint8 shift)
            return GRO_NOOP
    tcp_flags = pkt[iph_len + TCP_FLAGS_OFFSET]
    psh_set = False
    if tcp_flags != TCP_ACK:
        if tcp_flags != TCP_ACK | TCP_PSH:
            return GRO_NOOP
        psh_set = True
    gso_size = (len(pkt) - iph_len - tcph_len) & M16               # :880
    if gso_size < 1:
        return GRO_NOOP
    seq_num = be32(pkt, iph_len + 4)
    src_off, addr_len = (IPV6_SRC, 16) if is_v6 else (IPV4_SRC, 4)
    items, existing = table.get_or_insert(pkt, src_off, src_off + addr_len, iph_len, tcph_len, bufs_index)
    if not existing:
        return GRO_TABLE_INSERT
    for i in range(len(items) - 1, -1, -1):                        # :903 (deleteAt shifts only indices >= i)
        item = items[i].copy()                                     # :913 (a copy of the struct)
        can = tcp_packets_can_coalesce(pkt, iph_len, tcph_len, seq_num, psh_set, gso_size, item, bufs, offset)
        if can != COALESCE_UNAVAILABLE:
            result = coalesce_tcp_packets(can, pkt, bufs_index, gso_size, seq_num, psh_set, item, bufs, offset, is_v6)
            if result == COALESCE_SUCCESS:
                table.update_at(item, i)
                return GRO_COALESCED
            elif result == ITEM_INVALID_CSUM:
                table.delete_at(item.key, i)
            elif result == PKT_INVALID_CSUM:
                return GRO_NOOP
    table.insert(pkt, src_off, src_off + addr_len, iph_len, tcph_len, bufs_index)  # :954-961
    return GRO_TABLE_INSERT


def udp_gro(bufs, offset, bufs_index, table: UdpTable, is_v6):
    """udpGRO, gro.go:971-1095."""
    pkt = bufs[bufs_index].s(offset)
    if len(pkt) > MAX_UINT16:
        return GRO_NOOP
    iph_len = (pkt[0] & 0x0F) * 4
    if is_v6:
        iph_len = 40
        if be16(pkt, 4) != len(pkt) - iph_len:
            return GRO_NOOP
    else:
        if be16(pkt, 2) != len(pkt):
            return GRO_NOOP
    if len(pkt) < iph_len + UDPH_LEN:
        return GRO_NOOP
    if not is_v6:
        if pkt[6] & IPV4_FLAG_MF != 0 or (pkt[6] << 3) & 0xFF != 0 or pkt[7] != 0:
            return GRO_NOOP
    gso_size = (len(pkt) - iph_len - UDPH_LEN) & M16
    if gso_size < 1:
        return GRO_NOOP
    src_off, addr_len = (IPV6_SRC, 16) if is_v6 else (IPV4_SRC, 4)
    items, existing = table.get_or_insert(pkt, src_off, src_off + addr_len, iph_len, bufs_index)
    if not existing:
        return GRO_TABLE_INSERT
    item = items[-1].copy()                                        # :1046
    can = udp_packets_can_coalesce(pkt, iph_len, gso_size, item, bufs, offset)
    pkt_known_invalid = False
    if can == COALESCE_APPEND:
        result = coalesce_udp_packets(pkt, item, bufs, offset, is_v6)
        if result == COALESCE_SUCCESS:
            table.update_at(item, len(items) - 1)
            return GRO_COALESCED
        elif result == PKT_INVALID_CSUM:
            pkt_known_invalid = True
    table.insert(pkt, src_off, src_off + addr_len, iph_len, bufs_index, pkt_known_invalid)
    return GRO_TABLE_INSERT


def _pseudo_field(bufs, item, offset, is_v6, proto, pkt: Slice):
    addr_len, addr_off = (16, IPV6_SRC) if is_v6 else (4, IPV4_SRC)
    at = offset + addr_off
    src = bufs[item.bufs_index].s(at, at + addr_len)
    dst = bufs[item.bufs_index].s(at + addr_len, at + 2 * addr_len)
    ph = pseudo_header_checksum_no_fold(src, dst, proto, (len(pkt) - item.iph_len) & M16)
    return checksum(b"", ph)


def apply_tcp_coalesce(bufs, offset, table: TcpTable) -> int:
    """applyTCPCoalesce, gro.go:1099-1179."""
    for items in table.items_by_flow.values():
        for item in items:
            if item.num_merged > 0:
                hdr = VirtioHdr(VIRTIO_NET_HDR_F_NEEDS_CSUM, 0, (item.iph_len + item.tcph_len) & 0xFF, item.gso_size,
                                item.iph_len, 16)
                pkt = bufs[item.bufs_index].s(offset)
                is_v6 = item.key[5]
                if is_v6:
                    hdr.gso_type = GSO_TCPV6
                    put_be16(pkt, 4, ((len(pkt) & M16) - item.iph_len) & M16)
                else:
                    hdr.gso_type = GSO_TCPV4
                    put_be16(pkt, 2, len(pkt) & M16)
                    pkt[10] = 0
                    pkt[11] = 0
                    put_be16(pkt, 10, ~checksum(pkt.s(0, item.iph_len), 0) & M16)
                rc = hdr.encode(bufs[item.bufs_index].s(offset - VIRTIO_NET_HDR_LEN))
                if rc:
                    return rc
                put_be16(pkt, (hdr.csum_start + hdr.csum_offset) & M16,
                         _pseudo_field(bufs, item, offset, is_v6, IPPROTO_TCP, pkt))
            else:
                rc = VirtioHdr().encode(bufs[item.bufs_index].s(offset - VIRTIO_NET_HDR_LEN))
                if rc:
                    return rc
    return OK


def apply_udp_coalesce(bufs, offset, table: UdpTable) -> int:
    """applyUDPCoalesce, gro.go:1183-1268."""
    for items in table.items_by_flow.values():
        for item in items:
            if item.num_merged > 0:
                hdr = VirtioHdr(VIRTIO_NET_HDR_F_NEEDS_CSUM, GSO_UDP_L4, (item.iph_len + UDPH_LEN) & 0xFF,
                                item.gso_size, item.iph_len, 6)
                pkt = bufs[item.bufs_index].s(offset)
                is_v6 = item.key[4]
                if is_v6:
                    put_be16(pkt, 4, ((len(pkt) & M16) - item.iph_len) & M16)
                else:
                    put_be16(pkt, 2, len(pkt) & M16)
                    pkt[10] = 0
                    pkt[11] = 0
                    put_be16(pkt, 10, ~checksum(pkt.s(0, item.iph_len), 0) & M16)
                rc = hdr.encode(bufs[item.bufs_index].s(offset - VIRTIO_NET_HDR_LEN))
                if rc:
                    return rc
                put_be16(pkt, (item.iph_len + 4) & 0xFF, len(pkt.s(item.iph_len)) & M16)  # :1229-1232 (uint8 sum)
                put_be16(pkt, (hdr.csum_start + hdr.csum_offset) & M16,
                         _pseudo_field(bufs, item, offset, is_v6, IPPROTO_UDP, pkt))
            else:
                rc = VirtioHdr().encode(bufs[item.bufs_index].s(offset - VIRTIO_NET_HDR_LEN))
                if rc:
                    return rc
    return OK


NOT_CANDIDATE, TCP4, TCP6, UDP4, UDP6 = range(5)  # gro.go:1272-1278


def gro_candidate(pkt: Slice, can_udp_gro: bool) -> int:
    """groCandidate, gro.go:1280-1317."""
    if len(pkt) < 28:
        return NOT_CANDIDATE
    v = pkt[0] >> 4
    if v == 4:
        if pkt[0] & 0x0F != 5:
            return NOT_CANDIDATE
        if pkt[9] == IPPROTO_TCP and len(pkt) >= 40:
            return TCP4
        if pkt[9] == IPPROTO_UDP and can_udp_gro:
            return UDP4
    elif v == 6:
        if pkt[6] == IPPROTO_TCP and len(pkt) >= 60:
            return TCP6
        if pkt[6] == IPPROTO_UDP and len(pkt) >= 48 and can_udp_gro:
            return UDP6
    return NOT_CANDIDATE


def handle_gro(bufs: list, offset: int, tcp_table: TcpTable, udp_table: UdpTable, can_udp_gro: bool,
               to_write: list) -> int:
    """handleGRO, gro.go:1326-1367."""
    for i in range(len(bufs)):
        if offset < VIRTIO_NET_HDR_LEN or offset > len(bufs[i]) - 1:
            return ERR_INVALID_OFFSET
        result = GRO_NOOP
        c = gro_candidate(bufs[i].s(offset), can_udp_gro)
        if c == TCP4:
            result = tcp_gro(bufs, offset, i, tcp_table, False)
        elif c == TCP6:
            result = tcp_gro(bufs, offset, i, tcp_table, True)
        elif c == UDP4:
            result = udp_gro(bufs, offset, i, udp_table, False)
        elif c == UDP6:
            result = udp_gro(bufs, offset, i, udp_table, True)
        if result == GRO_NOOP:
            rc = VirtioHdr().encode(bufs[i].s(offset - VIRTIO_NET_HDR_LEN))
            if rc:
                return rc
            to_write.append(i)  # fallthrough
        elif result == GRO_TABLE_INSERT:
            to_write.append(i)
    err_tcp = apply_tcp_coalesce(bufs, offset, tcp_table)
    err_udp = apply_udp_coalesce(bufs, offset, udp_table)
    return err_tcp or err_udp  # errors.Join: non-nil if either is


def run_handle_gro(bufs: list, lens: list, offset: int, can_udp_gro: bool):
    """oracle.handle_gro's interface: bufs are numpy arrays (cap = their
    length), lens the slice lengths; the arrays are mutated in place.
    Returns (rc, to_write, order, new_lens), order[i] = the index of the
    original array now at position i (prepend swaps)."""
    sl = [Slice(b, 0, ln, len(b)) for b, ln in zip(bufs, lens)]
    tw: list = []
    try:
        rc = handle_gro(sl, offset, TcpTable(), UdpTable(), can_udp_gro, tw)
    except GoPanic:
        return ERR_OUT_OF_RANGE, [], list(range(len(bufs))), list(lens)
    ident = {id(b): k for k, b in enumerate(bufs)}
    return rc, tw, [ident[id(s.a)] for s in sl], [len(s) for s in sl]
