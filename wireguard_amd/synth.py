"""Seeded synthetic packet batches for the BASELINE.json configs.

Vectorised numpy construction of IPv4/IPv6 TCP/UDP frames with valid IPv4
header checksums and valid L4 checksums.  The checksums are set with the
order-free big-endian word-sum formulation, which is
independent of both the HIP kernels and the oracle restatement, so synthetic
batches are a third, independent witness in parity tests.

Layout in memory ("arena"): frames are packed back-to-back at
`off[i] = i * stride`; `pkts` is an array of the 16-byte wgcs_pkt descriptor
(include/wgcsum.h).  Header layouts follow /root/reference/packets.txt.
"""
from __future__ import annotations

import numpy as np

SEED = 20261015

from .tun import PKT_DTYPE, pkt_off, set_pkt_off  # noqa: E402,F401  (wgcs_pkt, include/wgcsum.h)

FLAG_V6 = 0x01
KIND_TCP4, KIND_UDP4, KIND_TCP6, KIND_UDP6 = 0, 1, 2, 3


def _fold(s: np.ndarray) -> np.ndarray:
    """checksum() closed form on uint64 integer sums: 0 -> 0, else 1+(S-1)%0xFFFF."""
    s = s.astype(np.uint64)
    out = np.where(s == 0, np.uint64(0), np.uint64(1) + (s - np.uint64(1)) % np.uint64(0xFFFF))
    return out.astype(np.uint16)


def word_sum(rows: np.ndarray) -> np.ndarray:
    """Sum of big-endian u16 words along axis 1 (rows must have even width)."""
    assert rows.shape[1] % 2 == 0
    w = np.ascontiguousarray(rows).view(">u2")
    return w.sum(axis=1, dtype=np.uint64)


def _put16(a: np.ndarray, col: int, v) -> None:
    v = np.asarray(v, dtype=np.uint32)
    a[:, col] = (v >> 8) & 0xFF
    a[:, col + 1] = v & 0xFF


def build_frames(kinds: np.ndarray, frame_len: int, rng: np.random.Generator,
                 valid: bool = True) -> np.ndarray:
    """Return an (n, frame_len) uint8 array of frames of the given kinds."""
    n = len(kinds)
    f = rng.integers(0, 256, size=(n, frame_len), dtype=np.uint8)
    v6 = (kinds == KIND_TCP6) | (kinds == KIND_UDP6)
    udp = (kinds == KIND_UDP4) | (kinds == KIND_UDP6)
    v4 = ~v6
    # ---- IPv4 header (20 B, IHL 5) ----
    if v4.any():
        h = f[v4]
        h[:, 0] = 0x45
        h[:, 1] = 0
        _put16(h, 2, frame_len)
        h[:, 6] = 0x40  # DF
        h[:, 7] = 0
        h[:, 8] = 64
        h[:, 9] = np.where(udp[v4], 17, 6)
        h[:, 10] = 0
        h[:, 11] = 0
        c = (~_fold(word_sum(h[:, :20]))).astype(np.uint16)
        _put16(h, 10, c)
        f[v4] = h
    # ---- IPv6 header (40 B) ----
    if v6.any():
        h = f[v6]
        h[:, 0] = 0x60
        h[:, 1] &= 0x0F
        _put16(h, 4, frame_len - 40)
        h[:, 6] = np.where(udp[v6], 17, 6)
        h[:, 7] = 64
        f[v6] = h
    iph = np.where(v6, 40, 20)
    # ---- L4 headers ----
    for kind in (KIND_TCP4, KIND_UDP4, KIND_TCP6, KIND_UDP6):
        m = kinds == kind
        if not m.any():
            continue
        is6 = kind in (KIND_TCP6, KIND_UDP6)
        isudp = kind in (KIND_UDP4, KIND_UDP6)
        ih = 40 if is6 else 20
        p = f[m]
        if isudp:
            _put16(p, ih + 4, frame_len - ih)
            co = 6
        else:
            p[:, ih + 12] = 0x50  # data offset 5
            p[:, ih + 13] = 0x10  # ACK
            p[:, ih + 18] = 0
            p[:, ih + 19] = 0
            co = 16
        p[:, ih + co] = 0
        p[:, ih + co + 1] = 0
        # pseudo header: addresses + proto + L4 length
        a0, a1 = (8, 40) if is6 else (12, 20)
        ph = word_sum(p[:, a0:a1]) + np.uint64(17 if isudp else 6) + np.uint64(frame_len - ih)
        l4 = p[:, ih:]
        if l4.shape[1] % 2:
            l4 = np.concatenate([l4, np.zeros((l4.shape[0], 1), np.uint8)], axis=1)
        c = (~_fold(word_sum(l4) + ph)).astype(np.uint16)
        if not valid:
            c = c ^ np.uint16(0x0101)
        _put16(p, ih + co, c)
        f[m] = p
    del iph
    return f


def make_batch(n: int, frame_len: int = 1500, kinds="tcp4", seed: int = SEED,
               stride: int | None = None, valid: bool = True, pad: int = 64):
    """Build a contiguous arena of n frames and their wgcs_pkt descriptors.

    kinds: "tcp4" | "udp4" | "tcp6" | "udp6" | "mixed" (25 % each, seeded
    shuffle, SURVEY.md §8(d) cfg 5) | an explicit integer array.
    """
    rng = np.random.default_rng(seed)
    if isinstance(kinds, str):
        if kinds == "mixed":
            k = np.repeat(np.arange(4, dtype=np.int64), (n + 3) // 4)[:n]
            rng.shuffle(k)
        else:
            k = np.full(n, {"tcp4": 0, "udp4": 1, "tcp6": 2, "udp6": 3}[kinds], dtype=np.int64)
    else:
        k = np.asarray(kinds, dtype=np.int64)
    stride = stride or frame_len
    arena = np.zeros(n * stride + pad, dtype=np.uint8)
    view = arena[: n * stride].reshape(n, stride)
    chunk = max(1, (64 << 20) // max(frame_len, 1))  # ~64 MB of frames per step
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        view[lo:hi, :frame_len] = build_frames(k[lo:hi], frame_len, rng, valid=valid)
    pkts = describe(k, frame_len, np.arange(n, dtype=np.uint64) * np.uint64(stride))
    return arena, pkts, k


def describe(kinds: np.ndarray, frame_len, offsets) -> np.ndarray:
    """wgcs_pkt descriptors of frames of the given kinds at the given arena offsets."""
    k = np.asarray(kinds)
    pkts = np.zeros(len(k), dtype=PKT_DTYPE)
    set_pkt_off(pkts, offsets)
    pkts["len"] = frame_len
    v6 = (k == KIND_TCP6) | (k == KIND_UDP6)
    udp = (k == KIND_UDP4) | (k == KIND_UDP6)
    pkts["csum_start"] = np.where(v6, 40, 20)
    pkts["csum_offset"] = np.where(udp, 6, 16)
    pkts["proto"] = np.where(udp, 17, 6)
    pkts["flags"] = v6 * FLAG_V6
    return pkts


def make_super_packet(total_len: int = 65535, gso_size: int = 1460, seed: int = SEED,
                      v6: bool = False, udp: bool = False, tcp_flags: int = 0x18) -> bytes:
    """A virtio-prefixed TSO/USO super-packet as the kernel hands it to Tun.Read
    (tun/tun.go:490): 10-byte virtio_net_hdr + IP + L4 + payload.  The L4
    checksum field holds the kernel's partial pseudo-header sum (arbitrary here:
    gsoSplit zeroes it, gro.go:1393)."""
    rng = np.random.default_rng(seed)
    ih = 40 if v6 else 20
    lh = 8 if udp else 20
    pkt = rng.integers(0, 256, size=total_len, dtype=np.uint8)
    if v6:
        pkt[0] = 0x60
        pkt[4:6] = [(total_len - 40) >> 8, (total_len - 40) & 0xFF]
        pkt[6] = 17 if udp else 6
        pkt[7] = 64
    else:
        pkt[0] = 0x45
        pkt[2:4] = [total_len >> 8, total_len & 0xFF]
        pkt[6] = 0x40
        pkt[7] = 0
        pkt[8] = 64
        pkt[9] = 17 if udp else 6
    if udp:
        pkt[ih + 4: ih + 6] = [(total_len - ih) >> 8 & 0xFF, (total_len - ih) & 0xFF]
    else:
        pkt[ih + 12] = 0x50
        pkt[ih + 13] = tcp_flags
    gso_type = (5 if udp else (4 if v6 else 1))
    co = 6 if udp else 16
    hdr = np.zeros(10, dtype=np.uint8)
    hdr[0] = 1  # NEEDS_CSUM
    hdr[1] = gso_type
    hdr[2:4] = np.frombuffer(np.uint16(ih + lh).tobytes(), np.uint8)
    hdr[4:6] = np.frombuffer(np.uint16(gso_size).tobytes(), np.uint8)
    hdr[6:8] = np.frombuffer(np.uint16(ih).tobytes(), np.uint8)
    hdr[8:10] = np.frombuffer(np.uint16(co).tobytes(), np.uint8)
    return hdr.tobytes() + pkt.tobytes()
