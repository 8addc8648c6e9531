"""CPU tests of the oracle (the C restatement of /root/reference/tun/checksum.go
and gro.go) against independent known answers and an independent closed form.

The reference ships no tests or fixtures and cannot run here (no Go
toolchain), so these pins are: RFC 1071 §3, the classic IPv4 header example,
a pseudo-header example, and the order-free word-sum closed
form checked against the faithful add-with-carry restatement.
"""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

import oracle
from wireguard_amd import synth

INITS = [0, 1, 0xFFFF, 0x10000, 2**32 - 1, 2**63, 2**64 - 1, 0x1234567890ABCDEF]


# ------------------------------------------------------------------- KATs
def test_rfc1071_example():
    # RFC 1071 §3: 00 01 f2 03 f4 f5 f6 f7 -> ones'-complement sum ddf2
    assert oracle.checksum(bytes([0x00, 0x01, 0xF2, 0x03, 0xF4, 0xF5, 0xF6, 0xF7]), 0) == 0xDDF2


def test_ipv4_header_example():
    hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    assert (~oracle.checksum(hdr, 0)) & 0xFFFF == 0xB861
    full = hdr[:10] + bytes.fromhex("b861") + hdr[12:]
    assert oracle.checksum(full, 0) == 0xFFFF  # a valid header sums to all ones


def test_pseudo_header_example():
    ph = oracle.pseudo_header_nofold(bytes([192, 168, 0, 1]), bytes([192, 168, 0, 199]), 17, 0x5F)
    assert ph == 0x80C101C800000000  # opaque big-endian-domain u64 (checksum.go:39-41,:118-119)
    assert oracle.checksum(b"", ph) == 0x8289


def test_nofold_byte_order_domain():
    assert oracle.checksum_nofold(b"\x01\x02", 0) == 0x0102000000000000
    assert oracle.checksum_nofold(b"", 0x0102) == 0x0102
    assert oracle.checksum_nofold(b"\xff" * 8, 0) == 2**64 - 1
    assert oracle.checksum_nofold(b"", 0) == 0


def test_zero_vs_ffff():
    # S == 0 -> 0x0000; S ≡ 0 (mod 0xFFFF), S != 0 -> 0xFFFF
    assert oracle.checksum(b"\0" * 100, 0) == 0
    assert oracle.checksum(b"\xff\xff", 0) == 0xFFFF
    assert oracle.checksum(b"", 2**64 - 1) == 0xFFFF
    assert oracle.checksum(b"\0" * 7, 0xFFFF) == 0xFFFF


# ------------------------------------------------- closed form vs faithful
@pytest.mark.parametrize("fill", [None, 0x00, 0xFF, 0x80, 0x01])
def test_closed_form_all_tail_paths(fill):
    rng = np.random.default_rng(0 if fill is None else fill)
    for n in list(range(0, 300)) + [511, 512, 513, 1023, 1500, 9000, 65535]:
        b = (rng.integers(0, 256, size=n, dtype=np.uint8) if fill is None else np.full(n, fill, np.uint8)).tobytes()
        for ini in INITS:
            assert oracle.checksum(b, ini) == oracle.closed_form_checksum(b, ini), (n, ini)


@settings(max_examples=400, deadline=None)
@given(st.binary(min_size=0, max_size=700), st.integers(min_value=0, max_value=2**64 - 1))
def test_closed_form_property(b, ini):
    assert oracle.checksum(b, ini) == oracle.closed_form_checksum(b, ini)


@settings(max_examples=200, deadline=None)
@given(st.binary(min_size=0, max_size=300), st.integers(min_value=0, max_value=299))
def test_split_additivity(b, cut):
    """checksum(b) == checksum(b[k:], checksumNoFold(b[:k], 0)) for even k."""
    k = min(cut, len(b)) & ~1
    assert oracle.checksum(b, 0) == oracle.checksum(b[k:], oracle.checksum_nofold(b[:k], 0))


# -------------------------------------------------------- checksumValid
@pytest.mark.parametrize("kinds", ["tcp4", "udp4", "tcp6", "udp6", "mixed"])
def test_synth_frames_validate(kinds):
    arena, pkts, k = synth.make_batch(300, 1500, kinds=kinds, stride=1503)
    v = oracle.checksum_batch(2, arena, pkts)
    assert v.all()
    bad, _, _ = synth.make_batch(300, 1500, kinds=kinds, stride=1503, valid=False)
    assert not oracle.checksum_batch(2, bad, pkts).any()
    # single-packet entry point agrees with the batch helper
    for i in range(10):
        o = int(synth.pkt_off(pkts)[i])
        pkt = arena[o: o + 1500].tobytes()
        v6 = bool(pkts["flags"][i] & 1)
        proto = int(pkts["proto"][i])
        assert oracle.checksum_valid(pkt, 40 if v6 else 20, proto, v6)


def test_fill_reproduces_stored_checksum():
    arena, pkts, _ = synth.make_batch(200, 1501, kinds="mixed")
    got = oracle.checksum_batch(1, arena, pkts)
    a = arena[: 200 * 1501].reshape(200, 1501)
    cs = pkts["csum_start"].astype(int) + pkts["csum_offset"]
    stored = (a[np.arange(200), cs].astype(np.uint16) << 8) | a[np.arange(200), cs + 1]
    assert np.array_equal(got, stored)


def test_multithreaded_batch_matches():
    arena, pkts, _ = synth.make_batch(2000, 1500, kinds="mixed")
    assert np.array_equal(oracle.checksum_batch_mt(2, arena, pkts, 4), oracle.checksum_batch(2, arena, pkts))
    assert np.array_equal(oracle.checksum_batch_mt(1, arena, pkts, 3), oracle.checksum_batch(1, arena, pkts))


# ------------------------------------------------------------- gsoSplit
def _split(vp, nbufs=128, size=65535, offset=16):
    rb = np.frombuffer(bytearray(vp), np.uint8).copy()
    bufs = [np.zeros(size, np.uint8) for _ in range(nbufs)]
    rc, n, sizes = oracle.handle_virtio_read(rb, bufs, offset)
    return rc, n, sizes, bufs, rb


def test_gso_split_tcp4_structure():
    vp = synth.make_super_packet(65535, 1460, tcp_flags=0x19)
    src = np.frombuffer(vp, np.uint8)[10:]
    rc, n, sizes, bufs, rb = _split(vp)
    assert rc == 0 and n == 45
    assert sizes[:n] == [1500] * 44 + [40 + 65495 - 44 * 1460]
    id0 = int(src[4]) << 8 | int(src[5])
    seq0 = int.from_bytes(src[24:28].tobytes(), "big")
    payload = b""
    for i in range(n):
        pkt = bufs[i][16: 16 + sizes[i]].tobytes()
        assert int.from_bytes(pkt[2:4], "big") == sizes[i]
        # quirk (gro.go:1426-1431): id0 + 1 for every segment after the first
        assert int.from_bytes(pkt[4:6], "big") == (id0 if i == 0 else (id0 + 1) & 0xFFFF)
        assert oracle.checksum(pkt[:20], 0) == 0xFFFF  # IPv4 header checksum valid
        assert int.from_bytes(pkt[24:28], "big") == (seq0 + 1460 * i) & 0xFFFFFFFF
        assert pkt[33] == (0x19 if i == n - 1 else 0x10)  # FIN|PSH only on the last segment
        assert oracle.checksum_valid(pkt, 20, 6, False)
        payload += pkt[40:]
    assert payload == src[40:].tobytes()
    # readBuf mutations (gro.go:1388,:1393)
    assert rb[10 + 10] == 0 and rb[10 + 11] == 0 and rb[10 + 36] == 0 and rb[10 + 37] == 0


@pytest.mark.parametrize("v6,udp", [(True, False), (False, True), (True, True)])
def test_gso_split_other_kinds_valid(v6, udp):
    vp = synth.make_super_packet(20000, 1232, v6=v6, udp=udp)
    rc, n, sizes, bufs, _ = _split(vp)
    assert rc == 0
    ih = 40 if v6 else 20
    for i in range(n):
        pkt = bufs[i][16: 16 + sizes[i]].tobytes()
        assert oracle.checksum_valid(pkt, ih, 17 if udp else 6, v6)
        if udp:
            assert int.from_bytes(pkt[ih + 4: ih + 6], "big") == sizes[i] - ih


def test_too_many_segments_semantics():
    vp = synth.make_super_packet(65535, 1460)
    rc, n, sizes, bufs, _ = _split(vp, nbufs=10)
    assert rc == oracle.OR_ERR_TOO_MANY if hasattr(oracle, "OR_ERR_TOO_MANY") else rc == -3
    assert n == 9  # i - 1 (gro.go:1409-1410)
    assert all(s == 1500 for s in sizes)


def test_virtio_read_errors():
    good = bytearray(synth.make_super_packet(3000, 1460))
    assert _split(bytes(good[:5]))[0] == -2
    b = bytearray(good); b[1] = 3
    assert _split(bytes(b))[0] == -5
    b = bytearray(good); b[1] = 4
    assert _split(bytes(b))[0] == -6
    b = bytearray(good); b[10] = 0x75
    assert _split(bytes(b))[0] == -7
    assert _split(bytes(good[:10 + 32]))[0] == -8
    b = bytearray(good); b[10 + 32] = 0x40
    assert _split(bytes(b))[0] == -9
    assert _split(bytes(good[:10 + 39]))[0] == -10
    b = bytearray(good); b[8:10] = (2980).to_bytes(2, "little")
    assert _split(bytes(b))[0] == -11
    none = bytearray(good); none[1] = 0; none[0] = 0
    assert _split(bytes(none), size=100)[0] == -12


def test_gso_none_checksum_odd_start():
    rng = np.random.default_rng(1)
    pkt = rng.integers(0, 256, size=777, dtype=np.uint8).tobytes()
    hdr = bytes([1, 0]) + (0).to_bytes(2, "little") + (0).to_bytes(2, "little") + (21).to_bytes(2, "little") + \
        (16).to_bytes(2, "little")
    rc, n, sizes, bufs, rb = _split(hdr + pkt)
    assert rc == 0 and n == 1 and sizes[0] == 777
    out = bufs[0][16: 16 + 777].tobytes()
    init = int.from_bytes(pkt[37:39], "big")
    body = bytearray(pkt[21:]); body[16:18] = b"\0\0"
    want = (~oracle.checksum(bytes(body), init)) & 0xFFFF
    assert int.from_bytes(out[37:39], "big") == want and out[:37] == pkt[:37] and out[39:] == pkt[39:]


# --------------------------------------------------------------- handleGRO
def _gro_batch(pkts, cap=65535, offset=16):
    bufs, lens = [], []
    for p in pkts:
        b = np.zeros(cap, np.uint8)
        b[offset: offset + len(p)] = np.frombuffer(p, np.uint8)
        bufs.append(b)
        lens.append(offset + len(p))
    return bufs, lens


def _tcp_stream(n, seg=1000, v6=False, seed=0, flags=0x10):
    """n in-order TCP segments of one flow (valid checksums)."""
    vp = synth.make_super_packet(40 + 20 * v6 + n * seg, seg, seed=seed, v6=v6, tcp_flags=flags)
    rc, cnt, sizes, bufs, _ = _split(vp, nbufs=max(n, 1), size=seg + 100)
    assert rc == 0 and cnt == n
    return [bufs[i][16: 16 + sizes[i]].tobytes() for i in range(n)]


def test_gro_coalesces_in_order_tcp_flow():
    segs = _tcp_stream(8)
    bufs, lens = _gro_batch(segs)
    rc, tw, order, nl = oracle.handle_gro(bufs, lens, 16, True)
    assert rc == 0 and tw == [0]
    b = bufs[order[0]]
    pkt = b[16: nl[0]].tobytes()
    assert len(pkt) == 40 + 8 * 1000
    assert pkt[40:] == b"".join(s[40:] for s in segs)
    vh = b[6:16].tobytes()
    assert vh[0] == 1 and vh[1] == 1 and int.from_bytes(vh[2:4], "little") == 40
    assert int.from_bytes(vh[4:6], "little") == 1000 and int.from_bytes(vh[6:8], "little") == 20
    assert oracle.checksum(pkt[:20], 0) == 0xFFFF
    ph = oracle.pseudo_header_nofold(pkt[12:16], pkt[16:20], 6, len(pkt) - 20)
    assert int.from_bytes(pkt[36:38], "big") == oracle.checksum(b"", ph)


def test_gro_invalid_checksum_not_coalesced():
    segs = _tcp_stream(6, seed=3)
    bad = bytearray(segs[3]); bad[-1] ^= 0xFF
    segs[3] = bytes(bad)
    bufs, lens = _gro_batch(segs)
    rc, tw, order, nl = oracle.handle_gro(bufs, lens, 16, True)
    assert rc == 0
    assert 3 in tw  # invalid packet written unmodified, with an empty virtio header
    assert bufs[order[3]][6:16].tobytes() == b"\0" * 10


def test_gro_prepend_out_of_order():
    segs = _tcp_stream(4, seed=5)
    bufs, lens = _gro_batch([segs[1], segs[0], segs[2], segs[3]])
    rc, tw, order, nl = oracle.handle_gro(bufs, lens, 16, True)
    assert rc == 0 and tw == [0]
    assert order[0] == 1 and order[1] == 0  # prepend swaps bufs (gro.go:696-697)
    pkt = bufs[order[0]][16: nl[0]].tobytes()
    assert pkt[40:] == b"".join(s[40:] for s in segs)


def test_gro_invalid_offset():
    segs = _tcp_stream(2)
    bufs, lens = _gro_batch(segs)
    assert oracle.handle_gro(bufs, lens, 5, True)[0] == -4
