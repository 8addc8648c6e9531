"""GPU parity of the resident per-call ring (include/wgcsum.h wgcs_ring_*,
wireguard_amd/csrc/ring.cpp + ring_kernel): checksumValid (tun/gro.go:554-612)
and handleVirtioRead (tun/tun.go:514-632) through the ring against the oracle,
byte for byte, on the same corpora as the per-call forms; inputs in pinned
host memory reused at one address with new content every call (a stale GPU
cache line would show); the kernel's idle exit and relaunch; and its stop on
destroy."""
import time

import numpy as np
import pytest

import gso_cases
import oracle
from wireguard_amd import WgcsError, synth
from wireguard_amd._lib import ERR_OUT_OF_RANGE, ERR_TOO_MANY_SEGMENTS
from wireguard_amd.tun import PKT_V6, Ring, pkt_off

pytestmark = pytest.mark.gpu

SENT = 0xA5


@pytest.fixture(scope="module")
def ring(dev):
    r = Ring(dev, idle_us=200000)
    yield r
    r.close()


def _code(err):
    return 0 if err is None else err.code


def test_ring_checksum_valid_matches_oracle(dev, ring):
    rng = np.random.default_rng(61)
    arena, pkts, _ = synth.make_batch(16, 1500, kinds="mixed")
    offs = pkt_off(pkts)
    for i in range(16):
        pkt = arena[offs[i]: offs[i] + 1500].tobytes()
        v6 = bool(pkts["flags"][i] & PKT_V6)
        proto = int(pkts["proto"][i])
        assert ring.checksum_valid(pkt, 40 if v6 else 20, proto, v6)
        bad = bytearray(pkt)
        bad[int(rng.integers(40, 1500))] ^= 1 << int(rng.integers(0, 8))
        assert not ring.checksum_valid(bytes(bad), 40 if v6 else 20, proto, v6)
    for proto in (0, 6, 17, 255):
        for iph in (0, 19, 20, 21, 40, 255):
            for n in (40, 41, 300, 1501, 9000):
                b = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
                for v6 in (False, True):
                    want = oracle.checksum_valid(b, iph, proto, v6)
                    if want is True or want is False:
                        assert ring.checksum_valid(b, iph, proto, v6) == want, (proto, iph, n, v6)
                    else:  # iphLen past the packet: Go panics, the ring reports OUT_OF_RANGE
                        with pytest.raises(WgcsError) as ei:
                            ring.checksum_valid(b, iph, proto, v6)
                        assert ei.value.code == want


def test_ring_checksum_valid_spare_capacity_and_errors(dev, ring):
    """Packets shorter than their addresses: read from the spare capacity, or
    OUT_OF_RANGE where Go panics -- as wgcs_checksum_valid_cap."""
    for buf, n, iph, proto, v6 in gso_cases.short_valid_cases():
        want = oracle.checksum_valid(buf, iph, proto, v6, n=n)
        if want is True or want is False:
            assert ring.checksum_valid(buf, iph, proto, v6, n=n) == want, (n, len(buf), iph, proto, v6)
        else:
            with pytest.raises(WgcsError) as ei:
                ring.checksum_valid(buf, iph, proto, v6, n=n)
            assert ei.value.code == want


def test_ring_pinned_reuse_same_address(dev, ring):
    """Zero-copy: the packet in wgcs_host_alloc memory, rewritten in place
    before every call (Tun.Read reuses one readBuf): every verdict matches the
    bytes of that call, valid and corrupted alternating."""
    buf = dev.host_alloc(2048)
    try:
        arena, pkts, _ = synth.make_batch(32, 1500, kinds="mixed", seed=5)
        offs = pkt_off(pkts)
        for k in range(64):
            i = k % 32
            buf[:1500] = arena[offs[i]: offs[i] + 1500]
            if k % 2:
                buf[100 + k] ^= 0x10
            v6 = bool(pkts["flags"][i] & PKT_V6)
            want = oracle.checksum_valid(buf[:1500].tobytes(), 40 if v6 else 20, int(pkts["proto"][i]), v6)
            assert want == (k % 2 == 0)
            assert ring.checksum_valid(buf[:1500], 40 if v6 else 20, int(pkts["proto"][i]), v6) == want, k
    finally:
        dev.host_free(buf)


def _virtio_both(ring, vpkt, nbufs, bufsize, offset, fill, read_buf=None):
    rb_o = np.frombuffer(bytearray(vpkt), dtype=np.uint8).copy()
    rb_p = rb_o.copy() if read_buf is None else read_buf
    if read_buf is not None:
        rb_p[: len(vpkt)] = rb_o
        rb_p = rb_p[: len(vpkt)]
    bo = [np.full(bufsize, fill, np.uint8) for _ in range(nbufs)]
    bp = [np.full(bufsize, fill, np.uint8) for _ in range(nbufs)]
    rc_o, n_o, sz_o = oracle.handle_virtio_read(rb_o, bo, offset)
    sz_p = [0] * nbufs
    n_p, err = ring.handle_virtio_read(rb_p, bp, sz_p, offset)
    return (rc_o, n_o, sz_o, bo, rb_o), (_code(err), n_p, sz_p, bp, np.array(rb_p))


def _assert_same(o, p):
    rc_o, n_o, sz_o, bo, rb_o = o
    rc_p, n_p, sz_p, bp, rb_p = p
    assert rc_p == rc_o and n_p == n_o, (rc_p, rc_o, n_p, n_o)
    if rc_o in (0, ERR_TOO_MANY_SEGMENTS):
        written = len(bo) if rc_o == ERR_TOO_MANY_SEGMENTS else max(n_o, 0)
        assert sz_p[:written] == sz_o[:written]
        assert np.array_equal(rb_p, rb_o), "readBuf mutation differs"
        for i in range(len(bo)):
            assert np.array_equal(bp[i], bo[i]), f"segment {i} differs"


@pytest.mark.parametrize("v6,udp", [(False, False), (True, False), (False, True), (True, True)])
def test_ring_handle_virtio_read_super_packets(dev, ring, v6, udp):
    for total, gso in ((65535, 1460), (65535, 1448), (9000, 1), (1500, 1460)):
        vp = synth.make_super_packet(total, gso, v6=v6, udp=udp)
        _assert_same(*_virtio_both(ring, vp, 128, 2048 if gso < 2000 else 65535, 16, SENT))


def test_ring_handle_virtio_read_fuzz(dev, ring):
    """The per-call fuzz corpus (tests/gso_cases.py, 1,100 mutated virtio reads)
    through the ring: every byte, size, count, error and readBuf edit."""
    compared = 0
    for trial, (vp, nbufs, bufsize, fill, offset, h, is_v6) in enumerate(gso_cases.fuzz_cases(False)):
        o, p = _virtio_both(ring, vp, nbufs, bufsize, offset, fill)
        if o[0] == ERR_OUT_OF_RANGE:
            assert p[0] == ERR_OUT_OF_RANGE, (trial, p[0])
            continue
        _assert_same(o, p)
        compared += 1
    assert compared >= 550


def test_ring_handle_virtio_read_pinned_reuse(dev, ring):
    """Zero-copy Tun.Read: one readBuf in wgcs_host_alloc memory, a different
    super-packet written into it before every call."""
    rb = dev.host_alloc(65535 + 64)
    try:
        for k in range(12):
            vp = synth.make_super_packet(65535 - 97 * k, 1460 - k, v6=bool(k & 1), udp=bool(k & 2), seed=100 + k)
            _assert_same(*_virtio_both(ring, vp, 64, 2048, 16, SENT, read_buf=rb))
    finally:
        dev.host_free(rb)


def test_ring_handle_virtio_read_direct_into_pinned_slab(dev, ring):
    """Zero-copy both ways: the readBuf and the Read buffers in wgcs_host_alloc
    memory, the buffers one slab on a fixed stride (a Read-buffer pool), so the
    kernel writes the segments straight into them; every byte of every buffer
    (the sentinel fill between and after the packets included) matches the
    oracle's, for split, GSO_NONE and error reads."""
    nb, stride, offset = 64, 2048, 16
    slab = dev.host_alloc(nb * stride)
    rb = dev.host_alloc(65535 + 64)
    try:
        bufs = [slab[i * stride:(i + 1) * stride] for i in range(nb)]
        cases = [synth.make_super_packet(65535 - 131 * k, 1460 - 3 * k, v6=bool(k & 1), udp=bool(k & 2), seed=300 + k)
                 for k in range(8)]
        cases += [vp for vp, nbufs, bufsize, fill, off, h, v6 in list(gso_cases.fuzz_cases(False))[:60]]
        for k, vp in enumerate(cases):
            slab[:] = SENT
            rb_o = np.frombuffer(bytearray(vp), np.uint8).copy()
            rb[: len(vp)] = rb_o
            bo = [np.full(stride, SENT, np.uint8) for _ in range(nb)]
            rc_o, n_o, sz_o = oracle.handle_virtio_read(rb_o, bo, offset)
            sz_p = [0] * nb
            n_p, err = ring.handle_virtio_read(rb[: len(vp)], bufs, sz_p, offset)
            if rc_o == ERR_OUT_OF_RANGE:
                assert _code(err) == ERR_OUT_OF_RANGE, k
                continue
            _assert_same((rc_o, n_o, sz_o, bo, rb_o), (_code(err), n_p, sz_p, [np.array(b) for b in bufs],
                                                         np.array(rb[: len(vp)])))
    finally:
        dev.host_free(rb)
        dev.host_free(slab)


def test_ring_idle_exit_relaunch_and_destroy(dev):
    """The kernel leaves after idle_us without a request (every wave reaches
    the deadline), a later call launches it again and is served, and destroy
    stops a running kernel."""
    r = Ring(dev, idle_us=3000)
    try:
        pkt = synth.make_batch(1, 1500, kinds="tcp4")[0][:1500].tobytes()
        assert r.checksum_valid(pkt, 20, 6, False)
        assert r.info()["launches"] == 1
        t0 = time.time()
        while r.info()["running"]:
            assert time.time() - t0 < 5, "ring kernel did not leave on its idle deadline"
            time.sleep(0.002)
        assert r.checksum_valid(pkt, 20, 6, False)
        inf = r.info()
        assert inf["launches"] == 2 and inf["requests"] == 2
    finally:
        r.close()
    r2 = Ring(dev, idle_us=10_000_000)
    assert r2.checksum_valid(pkt, 20, 6, False) and r2.info()["running"]
    t0 = time.time()
    r2.close()  # stop word: returns once the kernel has left
    assert time.time() - t0 < 5
