"""Seeded scenario generators for the outer-UDP message batching tests
(splitMessages / coalesceMessages, conn/bind.go:542-662), shared by the CPU
oracle tests and the GPU parity tests."""
from __future__ import annotations

import numpy as np

PKTINFO4 = (28).to_bytes(8, "little") + (0).to_bytes(4, "little") + (8).to_bytes(4, "little") + bytes(12) + bytes(4)


class Msg:
    """Duck-typed ipv6.Message (see wireguard_amd.conn.Message)."""

    def __init__(self, buf, oob_cap=64):
        self.buf = buf
        self.buf_len = len(buf)
        self.n = 0
        self.oob = np.zeros(oob_cap, dtype=np.uint8)
        self.oob_len = 0
        self.nn = 0
        self.addr = None


def gro_cmsg(g: int) -> bytes:
    return (18).to_bytes(8, "little") + (17).to_bytes(4, "little") + (104).to_bytes(4, "little") + \
        int(g).to_bytes(2, "little") + bytes(6)


def split_case(rng: np.random.Generator, n_msgs: int = 128, first: int | None = None, buf_len: int = 65535,
               kinds=("gro", "gro", "gro", "plain", "short_tail", "lt_gso", "zero", "bad_cmsg", "pktinfo")):
    """One recvmmsg batch: returns (msgs, first).  Source messages s >= first
    get random contents, N and control messages; the others are pool buffers
    with stale bytes (N = 0, as putMessages leaves them)."""
    if first is None:
        first = n_msgs - max(1, n_msgs // 64)  # readAt = len(msgs) - BatchSize/maxUDPSegments
    msgs = []
    for s in range(n_msgs):
        buf = rng.integers(0, 256, buf_len, dtype=np.uint8)
        m = Msg(buf)
        m.addr = f"addr{s}"
        msgs.append(m)
    for s in range(first, n_msgs):
        m = msgs[s]
        kind = kinds[int(rng.integers(len(kinds)))]
        ctl = b""
        if kind in ("gro", "short_tail", "pktinfo"):
            g = int(rng.choice([1452, 1280, 1200, 900, 64, 1]))
            segs = int(rng.integers(1, 64))
            n = min(g * segs, buf_len)
            if kind == "short_tail" and min(g, n) > 1:
                n -= int(rng.integers(1, min(g, n)))
            ctl = (PKTINFO4 if kind == "pktinfo" else b"") + gro_cmsg(g)
        elif kind == "plain":
            n = int(rng.integers(1, buf_len + 1))
        elif kind == "lt_gso":  # N < gsoSize: packet 0 is Buffers[0][0:gsoSize] (stale bytes past N)
            g = int(rng.integers(2, 4000))
            n = min(int(rng.integers(1, g)), buf_len)  # recvmmsg never returns more than the buffer
            ctl = gro_cmsg(g)
        elif kind == "zero":
            n = 0
        else:  # bad_cmsg: Len beyond the buffer
            n = min(int(rng.integers(1, 3000)), buf_len)
            ctl = (4096).to_bytes(8, "little") + (17).to_bytes(4, "little") + (104).to_bytes(4, "little") + bytes(8)
        m.n = n
        m.oob[: len(ctl)] = np.frombuffer(ctl, dtype=np.uint8)
        m.nn = len(ctl)
    return msgs, first


def clone_msgs(msgs):
    out = []
    for m in msgs:
        c = Msg(m.buf.copy(), len(m.oob))
        c.buf_len, c.n, c.nn, c.addr = m.buf_len, m.n, m.nn, m.addr
        c.oob[:] = m.oob
        c.oob_len = m.oob_len
        out.append(c)
    return out


def coalesce_case(rng: np.random.Generator, nbufs: int | None = None, size: int | None = None):
    """One Send batch: returns (bufs, lens, src_control, dst_is_v6, oob_cap)."""
    if nbufs is None:
        nbufs = int(rng.integers(1, 129))
    if size is None:
        size = int(rng.choice([1452, 1280, 148, 32, 4000, 9000, 65535]))
    pattern = rng.choice(["uniform", "uniform_tail", "random", "mixed", "zeros"])
    lens = []
    for j in range(nbufs):
        if pattern == "uniform":
            ln = size
        elif pattern == "uniform_tail":
            ln = size if rng.random() > 0.08 else int(rng.integers(0, size + 1))
        elif pattern == "random":
            ln = int(rng.integers(0, min(size, 65535) + 1))
        elif pattern == "zeros":
            ln = 0 if rng.random() < 0.3 else size
        else:
            ln = size if rng.random() > 0.3 else int(rng.choice([size // 2, size + 16, 16, 0]))
        lens.append(min(ln, 65535))
    bufs = []
    for j in range(nbufs):
        cap = 65535 if rng.random() > 0.15 else int(rng.integers(lens[j], 65536))
        b = rng.integers(0, 256, cap, dtype=np.uint8)
        bufs.append(b)
    src = [b"", PKTINFO4 + bytes(4), bytes(rng.integers(0, 256, 40, dtype=np.uint8))][int(rng.integers(3))]
    v6 = bool(rng.integers(2))
    oob_cap = int(rng.choice([64, 64, 64, 40, 30, 0]))
    return bufs, lens, src, v6, oob_cap
