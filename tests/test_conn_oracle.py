"""CPU: the conn/ message-batching oracle (oracle/wg_oracle_conn.c) against
known answers and against an independent pure-Python transcription of
splitMessages / coalesceMessages / getGSOSize / setGSOSize
(conn/bind.go:542-662, conn/gso.go:35-100).

Parity pinning: the reference ships no tests or fixtures for conn/ and its Go
toolchain is absent, so these are hand-derived known answers from the source
text plus a second, independent restatement ("parity unpinned" against
reference outputs)."""
import numpy as np
import pytest

import oracle
from conn_cases import PKTINFO4, clone_msgs, coalesce_case, gro_cmsg, split_case

ERR_OUT_OF_RANGE, ERR_CMSG, ERR_SPLIT_OVERFLOW = -13, -16, -17


# ---------------------------------------------------------------- restatement 2
def py_get_gso(ctl: bytes):
    rem = bytes(ctl)
    while len(rem) > 16:  # conn/gso.go:42
        hl = int.from_bytes(rem[0:8], "little")
        level = int.from_bytes(rem[8:12], "little", signed=True)
        typ = int.from_bytes(rem[12:16], "little", signed=True)
        if hl < 16 or hl > len(rem):
            return 0, ERR_CMSG
        data = rem[16:hl]
        if level == 17 and typ == 104 and len(data) >= 2:
            return int.from_bytes(data[:2], "little"), 0
        adv = (hl + 7) & ~7
        rem = rem[adv:] if adv < len(rem) else b""
    return 0, 0


def py_split(msgs, first):
    """conn/bind.go:542-597 on plain Python lists (buf as bytearray)."""
    bufs = [bytearray(m.buf.tobytes()) for m in msgs]
    ns = [m.n for m in msgs]
    addrs = [m.addr for m in msgs]
    npk = 0
    for i in range(first, len(msgs)):
        if ns[i] == 0:
            return npk, 0, bufs, ns, addrs
        g, err = py_get_gso(msgs[i].oob[: msgs[i].nn].tobytes())
        if err:
            return npk, err, bufs, ns, addrs
        num, start, end = 1, 0, ns[i]
        if g > 0:
            num, end = (ns[i] + g - 1) // g, g
        for _ in range(num):
            if npk > i:
                return npk, ERR_SPLIT_OVERFLOW, bufs, ns, addrs
            if end > len(bufs[i]):
                return npk, ERR_OUT_OF_RANGE, bufs, ns, addrs
            seg = bytes(bufs[i][start:end])
            nb = min(len(bufs[npk]), len(seg))
            bufs[npk][:nb] = seg[:nb]
            ns[npk] = nb
            addrs[npk] = addrs[i]
            start = end
            end = min(end + g, ns[i])
            npk += 1
        if i != npk - 1:
            ns[i] = 0
    return npk, 0, bufs, ns, addrs


def py_coalesce(bufs, lens, src, v6, oob_cap):
    """conn/bind.go:599-662: returns [(first, len, oob bytes)], new buffers."""
    data = [bytearray(b.tobytes()) for b in bufs]
    maxp = 65527 if v6 else 65507
    msgs = []  # [first, len, cap, oob(bytearray of oob_cap), oob_len]
    npk = gso = 0
    end_batch = False

    def set_gso(m, g):
        if 24 > oob_cap - m[4]:
            return
        o = m[3]
        at = m[4]
        o[at: at + 18] = (18).to_bytes(8, "little") + (17).to_bytes(4, "little") + (103).to_bytes(4, "little") + \
            int(g & 0xFFFF).to_bytes(2, "little")
        m[4] += 24

    for j in range(len(bufs)):
        if j > 0:
            m = msgs[-1]
            bl = lens[j]
            if bl + m[1] <= maxp and bl <= gso and bl <= m[2] - m[1] and npk < 64 and not end_batch:
                data[m[0]][m[1]: m[1] + bl] = data[j][:bl]
                m[1] += bl
                if j == len(bufs) - 1:
                    set_gso(m, gso)
                npk += 1
                if bl < gso:
                    end_batch = True
                continue
        if npk > 1:
            set_gso(msgs[-1], gso)
        npk, gso, end_batch = 1, lens[j], False
        oob = bytearray(oob_cap)
        m = [j, lens[j], len(bufs[j]), oob, 0]
        if oob_cap >= len(src):
            oob[: len(src)] = src
            m[4] = len(src)
        msgs.append(m)
    return [(m[0], m[1], bytes(m[3]), m[4]) for m in msgs], data


# ---------------------------------------------------------------- KATs
def test_get_gso_size_kats():
    assert oracle.get_gso_size(b"") == (0, 0)
    assert oracle.get_gso_size(gro_cmsg(1452)) == (1452, 0)
    assert oracle.get_gso_size(PKTINFO4 + gro_cmsg(1200)) == (1200, 0)  # skips IP_PKTINFO (28 -> 32 aligned)
    assert oracle.get_gso_size(PKTINFO4) == (0, 0)
    assert oracle.get_gso_size(gro_cmsg(1452)[:16]) == (0, 0)  # exactly SizeofCmsghdr left: not parsed (:42)
    bad = (8).to_bytes(8, "little") + bytes(16)  # Len < SizeofCmsghdr
    assert oracle.get_gso_size(bad)[1] == ERR_CMSG
    long = (100).to_bytes(8, "little") + bytes(24)  # Len beyond the buffer
    assert oracle.get_gso_size(long)[1] == ERR_CMSG
    short_data = (17).to_bytes(8, "little") + (17).to_bytes(4, "little") + (104).to_bytes(4, "little") + bytes(8)
    assert oracle.get_gso_size(short_data) == (0, 0)  # UDP_GRO with 1 data byte: skipped
    # a UDP_SEGMENT (103) cmsg is not UDP_GRO
    seg = (18).to_bytes(8, "little") + (17).to_bytes(4, "little") + (103).to_bytes(4, "little") + bytes(8)
    assert oracle.get_gso_size(seg) == (0, 0)


def test_set_gso_size_kat():
    oob = np.full(64, 0xEE, dtype=np.uint8)
    n = oracle.set_gso_size(oob, 40, 1452)
    assert n == 64
    assert bytes(oob[40:58]) == (18).to_bytes(8, "little") + (17).to_bytes(4, "little") + \
        (103).to_bytes(4, "little") + (1452).to_bytes(2, "little")
    assert bytes(oob[58:64]) == b"\xee" * 6  # padding keeps its old contents
    assert oracle.set_gso_size(oob, 41, 7) == 41  # no room: unchanged


def test_split_kat_two_gro_datagrams():
    """readAt = 126: two 45-segment datagrams -> 90 packets in msgs[0..90)."""
    rng = np.random.default_rng(1)
    msgs = [type("M", (), {})() for _ in range(128)]
    from conn_cases import Msg
    msgs = [Msg(rng.integers(0, 256, 65535, dtype=np.uint8)) for _ in range(128)]
    for s in (126, 127):
        msgs[s].n = 45 * 1452 - (0 if s == 126 else 100)
        c = gro_cmsg(1452)
        msgs[s].oob[: len(c)] = np.frombuffer(c, dtype=np.uint8)
        msgs[s].nn = len(c)
        msgs[s].addr = f"peer{s}"
    src = [m.buf.copy() for m in msgs]
    npk, rc = oracle.split_messages(msgs, 126)
    assert (npk, rc) == (90, 0)
    for k in range(90):
        s, j = (126, k) if k < 45 else (127, k - 45)
        want = src[s][j * 1452: min((j + 1) * 1452, 45 * 1452 - (0 if s == 126 else 100))]
        assert msgs[k].n == len(want)
        assert np.array_equal(msgs[k].buf[: len(want)], want)
        assert msgs[k].addr == f"peer{s}"
    assert msgs[126].n == 0 and msgs[127].n == 0  # consumed sources are zeroed (:589-594)


def test_split_kat_overflow_and_inplace_last():
    from conn_cases import Msg
    rng = np.random.default_rng(2)
    msgs = [Msg(rng.integers(0, 256, 1000, dtype=np.uint8)) for _ in range(4)]
    for s, (n, g) in {2: (300, 100), 3: (500, 100)}.items():
        msgs[s].n = n
        c = gro_cmsg(g)
        msgs[s].oob[: len(c)] = np.frombuffer(c, dtype=np.uint8)
        msgs[s].nn = len(c)
    src3 = msgs[3].buf.copy()
    npk, rc = oracle.split_messages(msgs, 2)
    # msg 2 -> slots 0,1,2 (the last one in place); msg 3 -> slot 3 (in place), then overflow
    assert (npk, rc) == (4, ERR_SPLIT_OVERFLOW)
    assert msgs[2].n == 100  # slot 2 is msg 2's own last packet: not zeroed
    assert msgs[3].n == 100 and np.array_equal(msgs[3].buf[:100], src3[:100])


def test_split_kat_n_below_gso():
    from conn_cases import Msg
    rng = np.random.default_rng(3)
    msgs = [Msg(rng.integers(0, 256, 4096, dtype=np.uint8)) for _ in range(2)]
    msgs[1].n = 10
    c = gro_cmsg(1000)
    msgs[1].oob[: len(c)] = np.frombuffer(c, dtype=np.uint8)
    msgs[1].nn = len(c)
    src = msgs[1].buf.copy()
    npk, rc = oracle.split_messages(msgs, 1)
    assert (npk, rc) == (1, 0)
    assert msgs[0].n == 1000  # Buffers[0][0:gsoSize]: packet 0 runs past N
    assert np.array_equal(msgs[0].buf[:1000], src[:1000])


def test_coalesce_kat_runs():
    rng = np.random.default_rng(4)
    bufs = [rng.integers(0, 256, 65535, dtype=np.uint8) for _ in range(128)]
    lens = [1452] * 128
    orig = [b.copy() for b in bufs]
    from conn_cases import Msg
    msgs = [Msg(np.zeros(1, np.uint8)) for _ in range(128)]
    nm = oracle.coalesce_messages(msgs, bufs, lens, b"", "ep", False)
    assert nm == 3  # 45 * 1452 = 65340 <= 65507 < 46 * 1452
    assert [m.buf_len for m in msgs[:3]] == [45 * 1452, 45 * 1452, 38 * 1452]
    for m, f in zip(msgs[:3], (0, 45, 90)):
        assert m.buf is bufs[f]
        assert m.oob_len == 24 and int.from_bytes(bytes(m.oob[16:18]), "little") == 1452
        for t in range((m.buf_len // 1452)):
            assert np.array_equal(m.buf[t * 1452:(t + 1) * 1452], orig[f + t][:1452])


# ---------------------------------------------------------------- cross-checks
@pytest.mark.parametrize("seed", range(24))
def test_split_oracle_vs_python(seed):
    rng = np.random.default_rng(1000 + seed)
    n_msgs = int(rng.choice([128, 8, 4, 16]))
    first = None if n_msgs == 128 else int(rng.integers(0, n_msgs))
    msgs, first = split_case(rng, n_msgs=n_msgs, first=first, buf_len=int(rng.choice([65535, 5000])))
    py = py_split(clone_msgs(msgs), first)
    npk, rc = oracle.split_messages(msgs, first)
    assert (npk, rc) == (py[0], py[1])
    for k, m in enumerate(msgs):
        assert m.n == py[3][k], k
        assert m.addr == py[4][k], k
        assert m.buf.tobytes() == bytes(py[2][k]), k


@pytest.mark.parametrize("seed", range(24))
def test_coalesce_oracle_vs_python(seed):
    rng = np.random.default_rng(2000 + seed)
    bufs, lens, src, v6, oob_cap = coalesce_case(rng)
    want_msgs, want_data = py_coalesce(bufs, lens, src, v6, oob_cap)
    from conn_cases import Msg
    msgs = [Msg(np.zeros(1, np.uint8), oob_cap) for _ in range(len(bufs))]
    nm = oracle.coalesce_messages(msgs, bufs, lens, src, "ep", v6)
    assert nm == len(want_msgs)
    for m, (f, ln, oob, olen) in zip(msgs, want_msgs):
        assert m.buf is bufs[f] and m.buf_len == ln
        assert m.oob_len == olen and m.oob.tobytes() == oob
    for b, d in zip(bufs, want_data):
        assert b.tobytes() == bytes(d)
