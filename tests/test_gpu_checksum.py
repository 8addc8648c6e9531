"""GPU parity: the gfx950 checksum kernels vs the oracle (CPU restatement of
/root/reference/tun/checksum.go + gro.go), bit-exact, through the C ABI."""
import numpy as np
import pytest

import oracle
from wireguard_amd import synth
from wireguard_amd.tun import (MODE_FOLD, MODE_IP4HDR, MODE_L4_FILL, MODE_PARTIAL, MODE_VALIDATE, PKT_DTYPE, PKT_V6,
                               pkt_off, set_pkt_off)

pytestmark = pytest.mark.gpu

INITS = [0, 0xFFFF, 2**64 - 1, 1, 0x1234567890ABCDEF, 0xFFFF0000FFFF0000]


def _pkts(offs, lens, cs=0, co=0, flags=0, proto=6):
    p = np.zeros(len(offs), dtype=PKT_DTYPE)
    set_pkt_off(p, offs)
    p["len"] = lens
    p["csum_start"] = cs
    p["csum_offset"] = co
    p["flags"] = flags
    p["proto"] = proto
    return p


def _both(dev, mode, arena, pkts, initial=None, inplace=False):
    a_gpu = arena.copy()
    a_cpu = arena.copy()
    got = dev.checksum_batch_host(mode, a_gpu, pkts, initial=initial, inplace=inplace)
    want = oracle.checksum_batch(mode, a_cpu, pkts, initial=initial, inplace=inplace)
    return got, want, a_gpu, a_cpu


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fold_all_small_lengths_random_alignment(dev, seed):
    rng = np.random.default_rng(seed)
    arena = rng.integers(0, 256, size=1 << 18, dtype=np.uint8)
    lens = np.tile(np.arange(0, 301), 4)
    offs = rng.integers(0, len(arena) - 400, size=len(lens))
    init = rng.choice(np.array(INITS, dtype=np.uint64), size=len(lens))
    init[::7] = rng.integers(0, 2**63, size=len(init[::7]), dtype=np.uint64) * 2 + 1
    got, want, _, _ = _both(dev, MODE_FOLD, arena, _pkts(offs, lens), initial=init)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("fill", [0x00, 0xFF])
def test_fold_constant_arenas(dev, fill):
    arena = np.full(1 << 17, fill, dtype=np.uint8)
    lens = np.concatenate([np.arange(0, 200), [1023, 1024, 1025, 4096, 9000, 65535]])
    rng = np.random.default_rng(7)
    offs = rng.integers(0, len(arena) - 65536, size=len(lens))
    for ini in INITS:
        init = np.full(len(lens), ini, dtype=np.uint64)
        got, want, _, _ = _both(dev, MODE_FOLD, arena, _pkts(offs, lens), initial=init)
        assert np.array_equal(got, want), f"init={ini:#x}"
    if fill == 0:
        # S == 0 -> 0x0000 must stay distinct from S ≡ 0 (mod 0xFFFF) -> 0xFFFF
        got = dev.checksum_batch_host(MODE_FOLD, arena, _pkts(offs, lens))
        assert (got == 0).all()


def test_fold_large_lengths(dev):
    rng = np.random.default_rng(11)
    arena = rng.integers(0, 256, size=1 << 21, dtype=np.uint8)
    lens = rng.integers(0, 65536, size=300)
    lens[:4] = [65535, 65534, 8191, 8193]
    offs = rng.integers(0, len(arena) - 65536, size=len(lens))
    init = rng.integers(0, 2**64 - 1, size=len(lens), dtype=np.uint64)
    got, want, _, _ = _both(dev, MODE_FOLD, arena, _pkts(offs, lens), initial=init)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("kinds", ["tcp4", "udp4", "tcp6", "udp6", "mixed"])
@pytest.mark.parametrize("frame_len,stride", [(1500, None), (1501, 1509), (64, 67), (9000, 9003), (48, None)])
@pytest.mark.parametrize("valid", [True, False])
def test_validate_and_fill_synth(dev, kinds, frame_len, stride, valid):
    if frame_len < 60 and kinds in ("tcp6", "mixed"):
        pytest.skip("IPv6/TCP needs 60 bytes")
    arena, pkts, _ = synth.make_batch(512, frame_len, kinds=kinds, stride=stride, valid=valid, seed=frame_len)
    got, want, _, _ = _both(dev, MODE_VALIDATE, arena, pkts)
    assert np.array_equal(got, want)
    assert bool(got.all()) == valid and bool(got.any()) == valid
    got, want, _, _ = _both(dev, MODE_L4_FILL, arena, pkts)
    assert np.array_equal(got, want)
    got, want, ag, ac = _both(dev, MODE_L4_FILL, arena, pkts, inplace=True)
    assert np.array_equal(got, want) and np.array_equal(ag, ac)


def test_validate_random_descriptors(dev):
    """Arbitrary (even odd) csum_start / lengths / alignment on random bytes."""
    rng = np.random.default_rng(5)
    arena = rng.integers(0, 256, size=1 << 20, dtype=np.uint8)
    n = 4000
    flags = rng.integers(0, 2, size=n)
    proto = rng.integers(0, 256, size=n)  # checksumValid takes any protocol byte
    proto[::2] = np.where(rng.integers(0, 2, size=len(proto[::2])) == 1, 17, 6)
    lens = rng.integers(40, 3000, size=n)
    cs = np.minimum(rng.integers(0, 80, size=n), lens - 20)
    cs[::3] = np.where(flags[::3] & 1, 40, 20)
    offs = np.arange(n) * 3003 + rng.integers(0, 3, size=n)  # disjoint packets, odd alignments
    arena = rng.integers(0, 256, size=n * 3003 + 64, dtype=np.uint8)
    p = _pkts(offs, lens, cs, 0, flags, proto)
    got, want, _, _ = _both(dev, MODE_VALIDATE, arena, p)
    assert np.array_equal(got, want)
    co = np.where(proto == 17, 6, 16)
    ok = cs + co + 2 <= lens
    p = _pkts(offs[ok], lens[ok], cs[ok], co[ok], flags[ok], proto[ok])
    got, want, _, _ = _both(dev, MODE_L4_FILL, arena, p)
    assert np.array_equal(got, want)
    # force a valid checksum into every packet and validate
    _, _, filled, _ = _both(dev, MODE_L4_FILL, arena, p, inplace=True)
    v = dev.checksum_batch_host(MODE_VALIDATE, filled, p)
    assert np.array_equal(v, oracle.checksum_batch(MODE_VALIDATE, filled, p))
    even = (p["csum_start"] % 2 == 0) & (p["csum_start"] >= np.where(p["flags"] & PKT_V6, 40, 20))
    assert v[even].all()


def test_partial_gso_none(dev):
    rng = np.random.default_rng(9)
    n = 600
    lens = rng.integers(2, 4000, size=n)
    cs = rng.integers(0, 200, size=n) % lens
    co = rng.integers(0, 256, size=n)
    ok = cs + co + 2 <= lens
    lens, cs, co = lens[ok], cs[ok], co[ok]
    m = len(lens)
    arena = rng.integers(0, 256, size=m * 4003 + 64, dtype=np.uint8)
    p = _pkts(np.arange(m) * 4003 + rng.integers(0, 3, size=m), lens, cs, co)  # disjoint, odd alignments
    got, want, ag, ac = _both(dev, MODE_PARTIAL, arena, p, inplace=True)
    assert np.array_equal(got, want) and np.array_equal(ag, ac)
    got, want, _, _ = _both(dev, MODE_PARTIAL, arena, p)
    assert np.array_equal(got, want)


def test_partial_u16_offsets(dev):
    """gsoNoneChecksum's csumStart + csumOffset is a uint16 sum (gro.go:1503):
    offsets across 0..65535, including wrapped positions before csumStart."""
    rng = np.random.default_rng(13)
    n = 400
    lens = rng.integers(64, 65536, size=n)
    cs = rng.integers(0, 65536, size=n) % lens
    at = rng.integers(0, 2**16, size=n) % (lens - 1)  # field position inside the packet
    co = (at - cs) % 65536                             # any u16 offset, wrapping when at < cs
    co[:4] = [65535, 256, 4096, 40000]
    at[:4] = (cs[:4] + co[:4]) % 65536
    ok = at + 2 <= lens
    lens, cs, co = lens[ok], cs[ok], co[ok]
    m = len(lens)
    stride = 65539
    arena = rng.integers(0, 256, size=m * stride + 64, dtype=np.uint8)
    p = _pkts(np.arange(m) * stride + rng.integers(0, 3, size=m), lens, cs, co)
    assert (p["csum_offset"] > 255).sum() > m // 2
    got, want, ag, ac = _both(dev, MODE_PARTIAL, arena, p, inplace=True)
    assert np.array_equal(got, want) and np.array_equal(ag, ac)
    got, want, _, _ = _both(dev, MODE_L4_FILL, arena, p)
    assert np.array_equal(got, want)
    # the single-call drop-in with the same u16 offsets
    for i in range(8):
        pk = bytearray(arena[int(pkt_off(p)[i]): int(pkt_off(p)[i]) + int(lens[i])].tobytes())
        pk2 = bytearray(pk)
        assert dev.gso_none_checksum(pk, int(cs[i]), int(co[i])) is None
        oracle.lib().or_gso_none_checksum(np.frombuffer(pk2, np.uint8).ctypes.data, len(pk2), int(cs[i]), int(co[i]))
        assert pk == pk2


def test_partial_all_zero_is_zero_not_ffff(dev):
    arena = np.zeros(4096, dtype=np.uint8)
    p = _pkts([1, 100, 1001], [1000, 37, 3], [10, 3, 0], [6, 16, 1])
    got, want, _, _ = _both(dev, MODE_PARTIAL, arena, p)
    assert np.array_equal(got, want) and (got == 0xFFFF).all()  # ^checksum(zeros, 0) = ^0


def test_ip4hdr(dev):
    arena, pkts, _ = synth.make_batch(1000, 1500, kinds="tcp4", stride=1503)
    rng = np.random.default_rng(3)
    pkts["csum_start"] = rng.integers(5, 16, size=len(pkts)) * 4
    got, want, ag, ac = _both(dev, MODE_IP4HDR, arena, pkts, inplace=True)
    assert np.array_equal(got, want) and np.array_equal(ag, ac)
    arena2, pkts2, _ = synth.make_batch(1000, 1500, kinds="tcp4", stride=1501)
    got = dev.checksum_batch_host(MODE_IP4HDR, arena2, pkts2)
    a = arena2[: 1000 * 1501].reshape(1000, 1501)
    stored = (a[:, 10].astype(np.uint16) << 8) | a[:, 11]
    assert np.array_equal(got, stored)  # synth wrote valid header checksums


def test_reference_shaped_single_calls(dev):
    rng = np.random.default_rng(2)
    # RFC 1071 §3 example
    assert dev.checksum(bytes([0x00, 0x01, 0xF2, 0x03, 0xF4, 0xF5, 0xF6, 0xF7]), 0) == 0xDDF2
    hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    assert (~dev.checksum(hdr, 0)) & 0xFFFF == 0xB861
    for n in [0, 1, 2, 3, 7, 8, 15, 16, 17, 127, 128, 129, 1500, 65535]:
        b = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        for ini in INITS:
            assert dev.checksum(b, ini) == oracle.checksum(b, ini)
    arena, pkts, kinds = synth.make_batch(8, 1500, kinds="mixed")
    offs = pkt_off(pkts)
    for i in range(8):
        pkt = arena[offs[i]: offs[i] + 1500].tobytes()
        v6 = bool(pkts["flags"][i] & PKT_V6)
        proto = int(pkts["proto"][i])
        assert dev.checksum_valid(pkt, 40 if v6 else 20, proto, v6)
        bad = bytearray(pkt)
        bad[-1] ^= 1
        assert not dev.checksum_valid(bytes(bad), 40 if v6 else 20, proto, v6)
    # any protocol byte and any iphLen (checksumValid's uint8 arguments)
    for proto in (0, 1, 6, 17, 41, 58, 132, 255):
        for iph in (0, 19, 20, 21, 40, 255):
            b = rng.integers(0, 256, size=300, dtype=np.uint8).tobytes()
            for v6 in (False, True):
                assert dev.checksum_valid(b, iph, proto, v6) == oracle.checksum_valid(b, iph, proto, v6)
    rb = bytearray(rng.integers(0, 256, size=777, dtype=np.uint8).tobytes())
    rb2 = bytearray(rb)
    assert dev.gso_none_checksum(rb, 21, 16) is None
    oracle.lib().or_gso_none_checksum((np.frombuffer(rb2, np.uint8)).ctypes.data, len(rb2), 21, 16)
    assert rb == rb2


def test_checksum_valid_short_packets_spare_capacity(dev):
    """checksumValid on packets shorter than their addresses: the per-call
    form with cap (wgcs_checksum_valid_cap) reads them from the spare bytes
    or reports OUT_OF_RANGE where Go panics; the batch modes read them from
    the arena bytes after the packet (include/wgcsum.h), as the oracle does."""
    import gso_cases

    from wireguard_amd import WgcsError

    cases = list(gso_cases.short_valid_cases())
    for buf, n, iph, proto, v6 in cases:
        want = oracle.checksum_valid(buf, iph, proto, v6, n=n)
        if want is True or want is False:
            assert dev.checksum_valid(buf, iph, proto, v6, n=n) == want, (n, len(buf), iph, proto, v6)
        else:
            with pytest.raises(WgcsError) as ei:
                dev.checksum_valid(buf, iph, proto, v6, n=n)
            assert ei.value.code == want
    rng = np.random.default_rng(12)
    offs, pos = [], 0
    for buf, *_ in cases:
        pos += int(rng.integers(0, 5))
        offs.append(pos)
        pos += len(buf)
    arena = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    for o_, (buf, *_) in zip(offs, cases):
        arena[o_: o_ + len(buf)] = np.frombuffer(buf, np.uint8)
    p = _pkts(offs, [c[1] for c in cases], [c[2] for c in cases], 0, [PKT_V6 if c[4] else 0 for c in cases],
              [c[3] for c in cases])
    got, want, _, _ = _both(dev, MODE_VALIDATE, arena, p)
    assert np.array_equal(got, want)
    # L4_FILL where the checksum field and the addresses lie in the buffer
    # (gsoSplit's readBuf; no packet reads bytes another one writes)
    co = np.array([int(rng.integers(0, 8)) for _ in cases])
    keep = np.array([c[2] + k + 2 <= len(c[0]) and len(c[0]) >= (40 if c[4] else 20) for c, k in zip(cases, co)])
    assert keep.sum() >= 50
    p2 = p[keep].copy()
    p2["csum_offset"] = co[keep]
    for inplace in (False, True):
        got, want, ag, ac = _both(dev, MODE_L4_FILL, arena, p2, inplace=inplace)
        assert np.array_equal(got, want) and np.array_equal(ag, ac)


def test_host_batch_refuses_addresses_past_the_arena(dev):
    """wgcs_checksum_batch_host: a VALIDATE / L4_FILL packet whose pseudo-header
    addresses lie past the host arena (its capacity) is refused with
    OUT_OF_RANGE, where Go panics; FOLD does not read them."""
    from wireguard_amd import WgcsError
    from wireguard_amd._lib import ERR_OUT_OF_RANGE

    arena = np.arange(30, dtype=np.uint8)
    for mode in (MODE_VALIDATE, MODE_L4_FILL):
        for flags, n_ok in ((0, 10), (PKT_V6, -10)):  # v4 addresses end at 20, v6 at 40
            with pytest.raises(WgcsError) as ei:
                dev.checksum_batch_host(mode, arena.copy(), _pkts([15], [10], 4, 0, flags))
            assert ei.value.code == ERR_OUT_OF_RANGE
            if n_ok > 0:  # at offset 10 the v4 addresses end at 30 == the arena's end
                got = dev.checksum_batch_host(mode, arena.copy(), _pkts([10], [n_ok], 4, 0, flags))
                assert np.array_equal(got, oracle.checksum_batch(mode, arena.copy(), _pkts([10], [n_ok], 4, 0, flags)))
    assert dev.checksum_batch_host(MODE_FOLD, arena.copy(), _pkts([25], [5])).shape == (1,)
