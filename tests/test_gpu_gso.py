"""GPU parity: GSO split (handleVirtioRead / gsoSplit, tun/tun.go:514-632 +
tun/gro.go:1373-1517) vs the oracle -- every output byte, size, count, error
code and the reference's readBuf mutations, through the C ABI."""
import struct

import numpy as np
import pytest

import gso_cases
import oracle
from wireguard_amd import synth
from wireguard_amd._lib import (ERR_BAD_IP_VERSION, ERR_CSUM_OFFSET, ERR_HDR_LEN, ERR_IP_GSO_MISMATCH,
                                ERR_OUT_OF_RANGE, ERR_PACKET_TOO_SHORT, ERR_READ_OVERFLOW, ERR_SHORT_BUFFER,
                                ERR_TCP_HDR_LEN, ERR_TOO_MANY_SEGMENTS, ERR_UNSUPPORTED_GSO, VirtioHdr)
from wireguard_amd.tun import GSO_JOB_DTYPE

pytestmark = pytest.mark.gpu

SENT = 0xA5


def _bufs(nbufs, size, fill=SENT):
    return [np.full(size, fill, dtype=np.uint8) for _ in range(nbufs)]


def _code(err):
    return 0 if err is None else err.code


def run_both(dev, vpkt: bytes, nbufs=128, bufsize=65535, offset=16, fill=SENT):
    rb_o = np.frombuffer(bytearray(vpkt), dtype=np.uint8).copy()
    rb_p = rb_o.copy()
    bo, bp = _bufs(nbufs, bufsize, fill), _bufs(nbufs, bufsize, fill)
    rc_o, n_o, sz_o = oracle.handle_virtio_read(rb_o, bo, offset)
    sz_p = [0] * nbufs
    n_p, err = dev.handle_virtio_read(rb_p, bp, sz_p, offset)
    return (rc_o, n_o, sz_o, bo, rb_o), (_code(err), n_p, sz_p, bp, rb_p)


def run_both_raw(dev, rb: bytes, hdr: tuple, is_v6: bool, nbufs=16, bufsize=9000, offset=16, fill=SENT):
    """gsoSplit(readBuf, hdr, ...) with the caller's header (gro.go:1373)."""
    rb_o = np.frombuffer(bytearray(rb), dtype=np.uint8).copy()
    rb_p = rb_o.copy()
    bo, bp = _bufs(nbufs, bufsize, fill), _bufs(nbufs, bufsize, fill)
    rc_o, n_o, sz_o = oracle.gso_split(rb_o, hdr, bo, offset, is_v6)
    sz_p = [0] * nbufs
    n_p, err = dev.gso_split(rb_p, VirtioHdr(*hdr), bp, sz_p, offset, is_v6)
    return (rc_o, n_o, sz_o, bo, rb_o), (_code(err), n_p, sz_p, bp, rb_p)


def assert_same(o, p, check_bufs=True, offset=16, fill=SENT):
    """Same return code, count, sizes and readBuf mutation; with check_bufs,
    every byte of every buffer -- including gsoSplit's header writes that land
    past a packet's end (a checksum or seq field beyond pktLen, gro.go:1426-
    1488) and the bytes it leaves alone."""
    rc_o, n_o, sz_o, bo, rb_o = o
    rc_p, n_p, sz_p, bp, rb_p = p
    assert rc_p == rc_o, (rc_p, rc_o)
    assert n_p == n_o
    written = len(bo) if rc_o == ERR_TOO_MANY_SEGMENTS else max(n_o, 0)
    if rc_o in (0, ERR_TOO_MANY_SEGMENTS):
        assert sz_p[:written] == sz_o[:written]
        assert np.array_equal(rb_p, rb_o), "readBuf mutation differs"
        if check_bufs:
            for i in range(len(bo)):
                assert np.array_equal(bp[i], bo[i]), f"segment {i} differs"


@pytest.mark.parametrize("v6,udp", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("total,gso", [(65535, 1460), (65535, 1448), (1500, 1460), (9000, 1), (60000, 7),
                                       (4000, 4000), (4001, 1000), (65535, 65000)])
def test_gso_split_matches_oracle(dev, v6, udp, total, gso):
    vp = synth.make_super_packet(total, gso, seed=total + gso, v6=v6, udp=udp)
    o, p = run_both(dev, vp, nbufs=128)
    assert_same(o, p)


@pytest.mark.parametrize("offset", [10, 16, 3, 0, 31])
def test_gso_offsets_and_alignment(dev, offset):
    vp = synth.make_super_packet(20000, 1460, seed=offset)
    o, p = run_both(dev, vp, nbufs=32, bufsize=2000, offset=offset)
    assert_same(o, p)


def test_too_many_segments(dev):
    vp = synth.make_super_packet(65535, 1460)
    o, p = run_both(dev, vp, nbufs=5)
    assert o[0] == ERR_TOO_MANY_SEGMENTS and o[1] == 4
    assert_same(o, p)
    vp = synth.make_super_packet(3000, 0)  # gsoSize 0: every buf gets a header-only segment
    o, p = run_both(dev, vp, nbufs=7)
    assert o[0] == ERR_TOO_MANY_SEGMENTS
    assert_same(o, p)


@pytest.mark.parametrize("flags", [0x10, 0x18, 0x19, 0x11, 0x01])
def test_fin_psh_only_on_last_segment(dev, flags):
    vp = synth.make_super_packet(10000, 1460, tcp_flags=flags)
    o, p = run_both(dev, vp, nbufs=16)
    assert_same(o, p)


def test_ipv4_options_and_tcp_options(dev):
    vp = bytearray(synth.make_super_packet(30000, 1400))
    rb = vp[10:]
    # IHL 6 (4 bytes of options) and TCP doff 8 (12 bytes of options): shift bytes
    pkt = bytes(rb[:20]) + b"\x01\x01\x01\x00" + bytes(rb[20:])
    pkt = bytearray(pkt[: len(rb)])
    pkt[0] = 0x46
    pkt[24 + 12] = 0x80
    hdr = bytearray(vp[:10])
    hdr[6:8] = (24).to_bytes(2, "little")
    o, p = run_both(dev, bytes(hdr) + bytes(pkt), nbufs=64)
    assert o[0] == 0
    assert_same(o, p)


def test_gso_none_paths(dev):
    """GSO_NONE (+ NEEDS_CSUM: gsoNoneChecksum with a uint16 csumStart +
    csumOffset anywhere in the packet, gro.go:1497-1517)."""
    rng = np.random.default_rng(4)
    big_offsets = 0
    for trial in range(120):
        plen = int(rng.integers(1, 3000)) if trial % 3 else int(rng.integers(3000, 65536))
        pkt = rng.integers(0, 256, size=plen, dtype=np.uint8)
        pkt[0] = 0x45
        cs = int(rng.integers(0, plen))
        if plen >= 2 and rng.random() < 0.8:
            at = int(rng.integers(0, plen - 1))  # field inside the packet, any u16 offset (wraps when at < cs)
            co = (at - cs) % 65536
        else:
            co = int(rng.integers(0, 65536))
        big_offsets += co > 255
        flags = int(rng.integers(0, 2))
        hdr = np.zeros(10, np.uint8)
        hdr[0] = flags
        hdr[6:8] = np.frombuffer(np.uint16(cs).tobytes(), np.uint8)
        hdr[8:10] = np.frombuffer(np.uint16(co).tobytes(), np.uint8)
        vp = hdr.tobytes() + pkt.tobytes()
        bufsize = int(rng.choice([65535 + 16, plen + 16, plen + 15, 100]))
        o, p = run_both(dev, vp, nbufs=4, bufsize=bufsize, offset=16)
        if o[0] == ERR_OUT_OF_RANGE:
            assert p[0] == ERR_OUT_OF_RANGE  # the reference panics on this input
            continue
        assert_same(o, p)
        if bufsize < plen + 16:
            assert o[0] == ERR_READ_OVERFLOW
    assert big_offsets > 50


def test_validation_errors(dev):
    good = bytearray(synth.make_super_packet(5000, 1460))
    cases = []
    cases.append((bytes(good[:9]), ERR_SHORT_BUFFER))
    for t in (2, 3, 0x80, 6):
        b = bytearray(good)
        b[1] = t
        cases.append((bytes(b), ERR_UNSUPPORTED_GSO))
    b = bytearray(good)
    b[1] = 4  # TCPV6 on an IPv4 packet
    cases.append((bytes(b), ERR_IP_GSO_MISMATCH))
    b = bytearray(good)
    b[10] = 0x55
    cases.append((bytes(b), ERR_BAD_IP_VERSION))
    b = bytearray(good[:10 + 32])
    cases.append((bytes(b), ERR_PACKET_TOO_SHORT))
    for doff in (0x40, 0x00, 0xF0):
        b = bytearray(good)
        b[10 + 20 + 12] = doff
        cases.append((bytes(b), ERR_TCP_HDR_LEN if doff != 0xF0 else 0))
    b = bytearray(good[:10 + 35])
    cases.append((bytes(b), ERR_HDR_LEN))
    b = bytearray(good)
    b[8:10] = (4990).to_bytes(2, "little")
    cases.append((bytes(b), ERR_CSUM_OFFSET))
    for vp, want in cases:
        o, p = run_both(dev, vp, nbufs=8, bufsize=70000)
        if want:
            assert o[0] == want, (o[0], want)
        if want != 0:
            assert p[0] == o[0]
        else:
            assert_same(o, p)


@pytest.mark.parametrize("raw", [False, True])
def test_fuzz_headers(dev, raw):
    """>= 1000 mutated headers per entry point.  The only cases not compared
    byte for byte are those where the ORACLE reports a reference panic
    (OUT_OF_RANGE); the product must report the same there."""
    compared = panics = 0
    trials = 0
    for trial, (vp, nbufs, bufsize, fill, offset, h, is_v6) in enumerate(gso_cases.fuzz_cases(raw)):
        trials += 1
        if raw:
            o, p = run_both_raw(dev, vp[10:], h, is_v6, nbufs, bufsize, offset, fill)
        else:
            o, p = run_both(dev, vp, nbufs, bufsize, offset, fill)
        if o[0] == ERR_OUT_OF_RANGE:
            assert p[0] == ERR_OUT_OF_RANGE, (trial, p[0])
            panics += 1
            continue
        assert_same(o, p, offset=offset, fill=fill)
        compared += 1
    assert compared >= 550 and compared + panics == trials == (1500 if raw else 1100)


def test_general_path_geometries(dev):
    """Targeted header geometries the row-streaming path does not take."""
    cases = []
    base4 = synth.make_super_packet(6000, 1000, seed=5)
    base6 = synth.make_super_packet(6000, 1000, seed=6, v6=True)
    for cs in (0, 1, 4, 5, 6, 11, 12, 19):  # IPv4 header shorter than 20 bytes (cs == 5: bufs' own byte 5)
        for co in (6, 16, 40, (65536 - cs + 3) % 65536):  # the last wraps the field to position 3
            h = bytearray(base4)
            h[6:8] = cs.to_bytes(2, "little")
            h[8:10] = co.to_bytes(2, "little")
            h[1] = 5  # UDP_L4: hdrLen = cs + 8
            cases.append(bytes(h))
    for cs in (300, 600):  # header over 240 bytes
        h = bytearray(base6)
        h[1] = 4
        h[6:8] = cs.to_bytes(2, "little")
        h[10 + cs + 12] = 0x80
        cases.append(bytes(h))
    for fill in (SENT, 0xFF, 0x00):
        for vp in cases:
            o, p = run_both(dev, vp, nbufs=16, bufsize=9000, fill=fill)
            if o[0] == ERR_OUT_OF_RANGE:
                assert p[0] == ERR_OUT_OF_RANGE
                continue
            assert_same(o, p, fill=fill)


def test_raw_gso_type_none_is_udp(dev):
    """gsoSplit itself treats any non-TCP gso_type (0 included) as UDP
    (gro.go:1398-1405): with gso_size 100 a 1000-byte packet splits into ~10
    segments (the packed output layout must size for them)."""
    rng = np.random.default_rng(8)
    rb = bytearray(rng.integers(0, 256, size=1000, dtype=np.uint8).tobytes())
    rb[0] = 0x45
    for gtype, gso in ((0, 100), (0, 1), (0, 0), (2, 333), (5, 100)):
        o, p = run_both_raw(dev, bytes(rb), (1, gtype, 28, gso, 20, 6), False, nbufs=32, bufsize=2000)
        assert o[0] in (0, ERR_TOO_MANY_SEGMENTS) and o[1] >= (9 if gso <= 100 else 3)
        assert_same(o, p)


def test_raw_gso_split(dev):
    """gsoSplit with the caller's header (no handleVirtioRead recomputation)."""
    vp = synth.make_super_packet(12000, 1460)
    for v6 in (False,):
        rb_o = np.frombuffer(bytearray(vp[10:]), np.uint8).copy()
        rb_p = rb_o.copy()
        h = VirtioHdr(1, 1, 40, 1460, 20, 16)
        bp = _bufs(16, 2000)
        sizes = [0] * 16
        n, err = dev.gso_split(rb_p, h, bp, sizes, 16, v6)
        # oracle: handleVirtioRead on the same bytes recomputes hdrLen = 40 too
        rb2 = np.frombuffer(bytearray(vp), np.uint8).copy()
        bo = _bufs(16, 2000)
        rc, n_o, sz_o = oracle.handle_virtio_read(rb2, bo, 16)
        assert err is None and rc == 0 and n == n_o and sizes[:n] == sz_o[:n]
        for i in range(16):
            assert np.array_equal(bp[i], bo[i])
        assert np.array_equal(rb_p, rb2[10:])


def test_device_batch_cfg4_like(dev):
    """Device-resident batch: 48 jobs of mixed kinds in one arena vs per-job oracle."""
    import torch

    rng = np.random.default_rng(3)
    jobs_bytes = []
    for j in range(48):
        total = int(rng.choice([65535, 30000, 1500, 9001]))
        gso = int(rng.choice([1460, 1448, 1200, 8948]))
        jobs_bytes.append(synth.make_super_packet(total, gso, seed=j, v6=bool(j % 2), udp=bool(j % 3 == 0)))
    offs, pos = [], 0
    for b in jobs_bytes:
        offs.append(pos)
        pos += len(b) + int(rng.integers(0, 7))
    arena = np.zeros(pos + 64, np.uint8)
    for o_, b in zip(offs, jobs_bytes):
        arena[o_: o_ + len(b)] = np.frombuffer(b, np.uint8)
    jobs = np.zeros(len(jobs_bytes), GSO_JOB_DTYPE)
    jobs["off"] = offs
    jobs["len"] = [len(b) for b in jobs_bytes]
    max_segs, stride, offset = 64, 9100, 16
    d_arena = torch.from_numpy(arena).cuda()
    d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
    d_out = torch.full((len(jobs) * max_segs * stride,), SENT, dtype=torch.uint8, device="cuda")
    d_sizes = torch.zeros(len(jobs) * max_segs, dtype=torch.int32, device="cuda")
    d_count = torch.zeros(len(jobs), dtype=torch.int32, device="cuda")
    d_status = torch.zeros(len(jobs), dtype=torch.int32, device="cuda")
    dev.gso_split_batch(d_arena, d_jobs, len(jobs), d_out, stride, offset, max_segs, d_sizes, d_count, d_status)
    dev.sync()
    out = d_out.cpu().numpy().reshape(len(jobs), max_segs, stride)
    sizes = d_sizes.cpu().numpy().reshape(len(jobs), max_segs)
    count, status = d_count.cpu().numpy(), d_status.cpu().numpy()
    for j, b in enumerate(jobs_bytes):
        rb = np.frombuffer(bytearray(b), np.uint8).copy()
        bo = _bufs(max_segs, stride)
        rc, n_o, sz_o = oracle.handle_virtio_read(rb, bo, offset)
        assert status[j] == rc and count[j] == n_o, j
        w = max_segs if rc == ERR_TOO_MANY_SEGMENTS else n_o
        assert list(sizes[j, :w]) == sz_o[:w]
        for i in range(max_segs):
            assert np.array_equal(out[j, i], bo[i]), (j, i)


@pytest.mark.parametrize("raw", [False, True])
def test_device_batch_fuzz_geometries(dev, raw):
    """The header-fuzz corpus as one device-resident batch (fixed slots of
    out_stride bytes standing in for bufs): every slot equals the oracle's
    buffer byte for byte -- the header writes gsoSplit leaves past a
    segment's end included -- and OUT_OF_RANGE where the reference panics."""
    import itertools

    import torch

    from wireguard_amd.tun import GSO_JOB_RAW, GSO_JOB_V6

    cases = list(itertools.islice(gso_cases.fuzz_cases(raw), 300))
    offs, pos = [], 0
    for vp, *_ in cases:
        offs.append(pos)
        pos += len(vp) + 5
    arena = np.zeros(pos + 64, np.uint8)
    for o_, (vp, *_) in zip(offs, cases):
        arena[o_: o_ + len(vp)] = np.frombuffer(vp, np.uint8)
    jobs = np.zeros(len(cases), GSO_JOB_DTYPE)
    jobs["off"] = offs
    jobs["len"] = [len(c[0]) for c in cases]
    if raw:
        jobs["flags"] = [GSO_JOB_RAW | (GSO_JOB_V6 if c[6] else 0) for c in cases]
    max_segs, stride, offset = 16, 9000, 16
    d_arena = torch.from_numpy(arena).cuda()
    d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
    d_out = torch.full((len(cases) * max_segs * stride,), SENT, dtype=torch.uint8, device="cuda")
    d_sizes = torch.zeros(len(cases) * max_segs, dtype=torch.int32, device="cuda")
    d_count = torch.zeros(len(cases), dtype=torch.int32, device="cuda")
    d_status = torch.zeros(len(cases), dtype=torch.int32, device="cuda")
    dev.gso_split_batch(d_arena, d_jobs, len(cases), d_out, stride, offset, max_segs, d_sizes, d_count, d_status)
    dev.sync()
    out = d_out.cpu().numpy().reshape(len(cases), max_segs, stride)
    sizes = d_sizes.cpu().numpy().reshape(len(cases), max_segs)
    count, status = d_count.cpu().numpy(), d_status.cpu().numpy()
    compared = 0
    for j, (vp, _, _, _, _, h, is_v6) in enumerate(cases):
        bo = _bufs(max_segs, stride)
        if raw:
            rb = np.frombuffer(bytearray(vp[10:]), np.uint8).copy()
            rc, n_o, sz_o = oracle.gso_split(rb, h, bo, offset, is_v6)
        else:
            rb = np.frombuffer(bytearray(vp), np.uint8).copy()
            rc, n_o, sz_o = oracle.handle_virtio_read(rb, bo, offset)
        assert status[j] == rc, (j, status[j], rc)
        if rc not in (0, ERR_TOO_MANY_SEGMENTS):
            continue
        assert count[j] == n_o, j
        w = max_segs if rc == ERR_TOO_MANY_SEGMENTS else n_o
        assert list(sizes[j, :w]) == list(sz_o[:w]), j
        for i in range(max_segs):
            assert np.array_equal(out[j, i], bo[i]), (j, i, np.nonzero(out[j, i] != bo[i])[0][:8])
        compared += 1
    assert compared >= 100


@pytest.mark.parametrize("raw", [False, True])
def test_short_packets_spare_capacity(dev, raw):
    """Packets shorter than their pseudo-header addresses read from a buffer
    with spare capacity (Tun.Read passes tun.readBuf[:n]): the address slices
    read the spare bytes (gro.go:1471-1477) or panic past cap -- through the
    per-call *_cap entry points and through the device batch with
    WGCS_GSO_JOB_SPARE, every buffer byte for byte against the oracle."""
    import itertools

    import torch

    from wireguard_amd.tun import GSO_JOB_RAW, GSO_JOB_V6, gso_job_spare

    cases = list(gso_cases.short_cases(raw))
    ok = 0
    for buf, n_read, nbufs, bufsize, fill, offset, h, is_v6 in cases:
        rb_o = np.frombuffer(bytearray(buf), np.uint8).copy()
        rb_p = rb_o.copy()
        bo, bp = _bufs(nbufs, bufsize, fill), _bufs(nbufs, bufsize, fill)
        sz_p = [0] * nbufs
        if raw:
            rc_o, n_o, sz_o = oracle.gso_split(rb_o, h, bo, offset, is_v6, n_read=n_read)
            n_p, err = dev.gso_split(rb_p, VirtioHdr(*h), bp, sz_p, offset, is_v6, n_read=n_read)
        else:
            rc_o, n_o, sz_o = oracle.handle_virtio_read(rb_o, bo, offset, n_read=n_read)
            n_p, err = dev.handle_virtio_read(rb_p, bp, sz_p, offset, n_read=n_read)
        assert_same((rc_o, n_o, sz_o, bo, rb_o), (_code(err), n_p, sz_p, bp, rb_p), offset=offset, fill=fill)
        ok += rc_o == 0
    assert ok >= 100
    # the same reads as one device batch (fixed slots), spare bytes after each job
    offs, pos = [], 0
    for buf, n_read, *_ in cases:
        offs.append(pos)
        pos += len(buf) + 3
    arena = np.zeros(pos + 64, np.uint8)
    for o_, (buf, *_) in zip(offs, cases):
        arena[o_: o_ + len(buf)] = np.frombuffer(buf, np.uint8)
    jobs = np.zeros(len(cases), GSO_JOB_DTYPE)
    jobs["off"] = offs
    jobs["len"] = [c[1] + (10 if raw else 0) for c in cases]
    if raw:  # a raw job's arena bytes are [virtio header | readBuf]: prepend the header
        arena, pos, offs2 = np.zeros(pos + 64 + 16 * len(cases), np.uint8), 0, []
        for buf, n_read, nbufs, bufsize, fill, offset, h, is_v6 in cases:
            vh = bytes([h[0], h[1]]) + b"".join(int(x).to_bytes(2, "little") for x in h[2:])
            b = vh + buf
            arena[pos: pos + len(b)] = np.frombuffer(b, np.uint8)
            offs2.append(pos)
            pos += len(b) + 3
        jobs["off"] = offs2
    jobs["flags"] = [(GSO_JOB_RAW | (GSO_JOB_V6 if c[7] else 0) if raw else 0) | gso_job_spare(len(c[0]) - c[1])
                     for c in cases]
    max_segs, stride, offset = 16, 256, 16
    d_arena = torch.from_numpy(arena).cuda()
    d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
    d_out = torch.full((len(cases) * max_segs * stride,), SENT, dtype=torch.uint8, device="cuda")
    d_sizes = torch.zeros(len(cases) * max_segs, dtype=torch.int32, device="cuda")
    d_count = torch.zeros(len(cases), dtype=torch.int32, device="cuda")
    d_status = torch.zeros(len(cases), dtype=torch.int32, device="cuda")
    dev.gso_split_batch(d_arena, d_jobs, len(cases), d_out, stride, offset, max_segs, d_sizes, d_count, d_status)
    dev.sync()
    out = d_out.cpu().numpy().reshape(len(cases), max_segs, stride)
    count, status = d_count.cpu().numpy(), d_status.cpu().numpy()
    for j, (buf, n_read, _, _, _, _, h, is_v6) in enumerate(cases):
        bo = _bufs(max_segs, stride)
        rb = np.frombuffer(bytearray(buf), np.uint8).copy()
        if raw:
            rc, n_o, _ = oracle.gso_split(rb, h, bo, offset, is_v6, n_read=n_read)
        else:
            rc, n_o, _ = oracle.handle_virtio_read(rb, bo, offset, n_read=n_read)
        assert status[j] == rc, (j, status[j], rc)
        if rc in (0, ERR_TOO_MANY_SEGMENTS):
            assert count[j] == n_o
            for i in range(max_segs):
                assert np.array_equal(out[j, i], bo[i]), (j, i)


@pytest.mark.parametrize("v6,udp", [(False, False), (True, False), (False, True)])
@pytest.mark.parametrize("total,gso", [(65535, 1460), (1500, 1460), (1460, 1460)])
def test_empty_bufs_split(dev, v6, udp, total, gso):
    """len(bufs) == 0: gsoSplit's loop returns (-1, ErrTooManySegments)
    before touching bufs (gro.go:1408-1410) after readBuf was prepared, or
    (0, nil) when the read holds no segment; validation errors come first."""
    vp = synth.make_super_packet(total, gso, seed=41, v6=v6, udp=udp)
    o, p = run_both(dev, vp, nbufs=0)
    assert_same(o, p)
    # the raw gsoSplit entry point, same header
    h = tuple(int(x) for x in struct.unpack("<BBHHHH", vp[:10]))
    o, p = run_both_raw(dev, vp[10:], h, v6, nbufs=0)
    assert_same(o, p)


def test_empty_bufs_gso_none(dev):
    """GSO_NONE with len(bufs) == 0 indexes bufs[0]: a Go panic, OUT_OF_RANGE."""
    pkt = synth.make_super_packet(1500, 1460, seed=42)[10:]
    n, err = dev.handle_virtio_read(bytes(10) + pkt, [], [], 16)
    assert err is not None and err.code == -13 and n == 0


def test_batch_rejects_huge_max_segs(dev):
    """len(bufs) is a Go int: wgcs_gso_split_batch refuses max_segs >= 2^31
    (INVALID_ARG, nothing launched) instead of letting the kernel's int
    segment bounds wrap."""
    import torch

    from wireguard_amd import WgcsError

    small = torch.zeros(64, dtype=torch.uint8, device="cuda")
    i32 = torch.zeros(4, dtype=torch.int32, device="cuda")
    with pytest.raises(WgcsError) as ei:
        dev.gso_split_batch(small, small, 1, small, 16, 0, 1 << 31, i32, i32, i32)
    assert ei.value.code == -1  # WGCS_ERR_INVALID_ARG


def test_batch_invalid_jobs_large_max_segs_return_promptly(dev):
    """A job that is not a split (GSO_NONE, bad gso type, IP-version mismatch,
    jlen < 14) under a large max_segs: the decoded path's verdict ends the
    block's group loop after the first group instead of running one decode +
    barrier round per 16 output slots.  Results vs the oracle,
    and the launch must take far less than the ~0.5 s those rounds would."""
    import time

    import torch

    pkt = bytearray(synth.make_super_packet(1500, 1460, seed=43))
    none_job = bytes([1, 0]) + bytes(pkt[2:10]) + bytes(pkt[10:])  # GSO_NONE + NEEDS_CSUM
    bad_type = bytes([1, 3]) + bytes(pkt[2:])
    v6_mismatch = bytes([1, 4]) + bytes(pkt[2:])  # TCPV6 on an IPv4 packet
    short = bytes(pkt[:12])
    vps = [none_job, bad_type, v6_mismatch, short]
    offs = np.cumsum([0] + [len(v) + 5 for v in vps])[:-1]
    arena = np.zeros(int(offs[-1]) + len(vps[-1]) + 64, np.uint8)
    for o_, v in zip(offs, vps):
        arena[o_: o_ + len(v)] = np.frombuffer(v, np.uint8)
    jobs = np.zeros(len(vps), GSO_JOB_DTYPE)
    jobs["off"] = offs
    jobs["len"] = [len(v) for v in vps]
    offset, stride = 16, 1600
    d_arena = torch.from_numpy(arena).cuda()
    d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
    d_count = torch.zeros(len(vps), dtype=torch.int32, device="cuda")
    d_status = torch.zeros(len(vps), dtype=torch.int32, device="cuda")
    for max_segs in (16, 1 << 24):
        # only job 0 (GSO_NONE) writes: bufs[0] at slot 0, sizes[0]
        d_out = torch.full((stride,), SENT, dtype=torch.uint8, device="cuda")
        d_sizes = torch.full((len(vps) * max_segs,), -7, dtype=torch.int32, device="cuda")
        dev.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.gso_split_batch(d_arena, d_jobs, len(vps), d_out, stride, offset, max_segs, d_sizes, d_count, d_status)
        dev.sync()
        dt = time.perf_counter() - t0
        assert dt < 0.1, (max_segs, dt)
        count, status = d_count.cpu().numpy(), d_status.cpu().numpy()
        for j, v in enumerate(vps):
            rb = np.frombuffer(bytearray(v), np.uint8).copy()
            bo = _bufs(min(max_segs, 4), stride)
            rc, n_o, sz_o = oracle.handle_virtio_read(rb, bo, offset)
            assert status[j] == rc and count[j] == n_o, (j, max_segs)
            if j == 0:
                assert rc == 0 and n_o == 1
                assert int(d_sizes[0].item()) == sz_o[0]
                assert np.array_equal(d_out.cpu().numpy(), bo[0])
        assert int((d_sizes[1:] != -7).sum().item()) == 0  # nothing else written
