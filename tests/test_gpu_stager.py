"""GPU parity: the Tun.Read batch stager (include/wgcsum.h wgcs_stager_*,
SURVEY.md §8f row 2).  Every read of a batch must leave bufs / sizes / n / err
exactly as the oracle's handleVirtioRead (tun/tun.go:514-632) does for that read
alone, across ring reuse, reserve/commit and the error paths."""
import numpy as np
import pytest

import oracle
from wireguard_amd import synth
from wireguard_amd._lib import ERR_BATCH_FULL, ERR_NOT_READY, ERR_TOO_MANY_SEGMENTS, WgcsError
from wireguard_amd.tun import Stager

pytestmark = pytest.mark.gpu

SENT = 0xA5
OFFSET = 16


def _reads(seed: int, count: int):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(count):
        kind = k % 7
        if kind == 0:
            out.append(synth.make_super_packet(65535, 1460, seed=seed * 100 + k))
        elif kind == 1:
            out.append(synth.make_super_packet(int(rng.integers(2000, 60000)), 1440, seed=seed * 100 + k, v6=True))
        elif kind == 2:
            out.append(synth.make_super_packet(int(rng.integers(1500, 30000)), 1200, seed=seed * 100 + k, udp=True))
        elif kind == 3:  # GSO_NONE + NEEDS_CSUM, odd csum start
            plen = int(rng.integers(60, 1500))
            pkt = rng.integers(0, 256, size=plen, dtype=np.uint8)
            pkt[0] = 0x45
            hdr = np.zeros(10, np.uint8)
            hdr[0] = 1
            hdr[6:8] = np.frombuffer(np.uint16(21).tobytes(), np.uint8)
            hdr[8:10] = np.frombuffer(np.uint16(16).tobytes(), np.uint8)
            out.append(hdr.tobytes() + pkt.tobytes())
        elif kind == 4:  # GSO_NONE without checksum
            plen = int(rng.integers(1, 9000))
            out.append(bytes(10) + rng.integers(0, 256, size=plen, dtype=np.uint8).tobytes())
        elif kind == 5:  # invalid: unsupported GSO type
            b = bytearray(synth.make_super_packet(5000, 1460, seed=k))
            b[1] = 3
            out.append(bytes(b))
        else:  # short buffer / tiny frame
            out.append(bytes(int(rng.integers(0, 12))))
    return out


def _oracle_read(vp: bytes, nbufs: int, bufsize: int):
    rb = np.frombuffer(bytearray(vp), np.uint8).copy()
    bo = [np.full(bufsize, SENT, np.uint8) for _ in range(nbufs)]
    rc, n, sz = oracle.handle_virtio_read(rb, bo, OFFSET)
    return rc, n, sz, bo


def _check_read(st: Stager, batch: int, idx: int, vp: bytes, nbufs: int, bufsize: int):
    rc_o, n_o, sz_o, bo = _oracle_read(vp, nbufs, bufsize)
    bp = [np.full(bufsize, SENT, np.uint8) for _ in range(nbufs)]
    sizes = [0] * nbufs
    n_p, err = st.copy_out(batch, idx, bp, sizes, OFFSET)
    rc_p = 0 if err is None else err.code
    assert rc_p == rc_o, (idx, rc_p, rc_o)
    assert n_p == n_o, (idx, n_p, n_o)
    if rc_o in (0, ERR_TOO_MANY_SEGMENTS):
        written = nbufs if rc_o == ERR_TOO_MANY_SEGMENTS else n_o
        assert sizes[:written] == list(sz_o[:written])
        for i in range(nbufs):
            assert np.array_equal(bp[i], bo[i]), (idx, i)
        n_r, err_r, sz_r = st.result(batch, idx)
        assert n_r == n_o and sz_r[:written] == list(sz_o[:written])


def test_stager_batch_matches_per_read_oracle(dev):
    nbufs, bufsize = 64, 9100
    st = Stager(dev, depth=2, max_reads=32, max_bytes=32 * 65552, max_segs=nbufs, seg_room=bufsize - OFFSET)
    reads = _reads(1, 28)
    idx = [st.push(r) for r in reads]
    assert idx == list(range(len(reads)))
    b = st.submit()
    st.wait(b)
    for i, r in enumerate(reads):
        _check_read(st, b, i, r, nbufs, bufsize)
    st.close()


def test_stager_ring_reuse_and_pipelining(dev):
    nbufs, bufsize = 48, 1600
    st = Stager(dev, depth=3, max_reads=8, max_bytes=8 * 65552, max_segs=nbufs, seg_room=bufsize - OFFSET)
    batches = []
    for k in range(7):  # more batches than ring slots: submit runs ahead, results stay per batch
        reads = [synth.make_super_packet(int(20000 + 5000 * j), 1460, seed=1000 * k + j, v6=bool(j & 1))
                 for j in range(5)]
        assert st.push_many(reads) == 0
        batches.append((st.submit(), reads))
        if len(batches) >= 2:  # depth-1 batches outstanding: consume the oldest before its slot is recycled
            bid, rs = batches.pop(0)
            st.wait(bid)
            for i, r in enumerate(rs):
                _check_read(st, bid, i, r, nbufs, bufsize)
    with pytest.raises(WgcsError):  # batch 1's slot was recycled by the third submit
        st.wait(1)
    for bid, rs in batches:
        st.wait(bid)
        for i, r in enumerate(rs):
            _check_read(st, bid, i, r, nbufs, bufsize)
    st.close()


def test_stager_too_many_segments_and_room(dev):
    nbufs, bufsize = 6, 1600
    st = Stager(dev, depth=2, max_reads=4, max_bytes=4 * 65552, max_segs=nbufs, seg_room=bufsize - OFFSET)
    reads = [synth.make_super_packet(65535, 1460, seed=5),  # 45 segments into 6 bufs
             synth.make_super_packet(5000, 1460, seed=6),
             bytes(10) + bytes(3000)]  # GSO_NONE larger than the room: READ_OVERFLOW
    for r in reads:
        st.push(r)
    b = st.submit()
    st.wait(b)
    for i, r in enumerate(reads):
        _check_read(st, b, i, r, nbufs, bufsize)
    n, err, _ = st.result(b, 0)
    assert err is not None and err.code == ERR_TOO_MANY_SEGMENTS and n == nbufs - 1
    st.close()


def test_stager_reserve_commit_and_errors(dev):
    nbufs, bufsize = 32, 1600
    st = Stager(dev, depth=2, max_reads=3, max_bytes=3 * 65552, max_segs=nbufs, seg_room=bufsize - OFFSET)
    vp = synth.make_super_packet(30000, 1460, seed=9)
    i0, view = st.reserve(65545)
    view[: len(vp)] = np.frombuffer(vp, np.uint8)  # stands in for read(2) into the pinned slot
    st.commit(i0, len(vp))
    i1, _ = st.reserve(100)
    st.commit(i1, 0)  # nothing read: dropped
    i2 = st.push(vp)
    assert (i0, i2) == (0, 1)
    st.push(vp)
    with pytest.raises(WgcsError) as ei:
        st.push(vp)
    assert ei.value.code == ERR_BATCH_FULL
    with pytest.raises(WgcsError) as ei:
        st.wait(12345)
    assert ei.value.code == ERR_NOT_READY
    b = st.submit()
    st.wait(b)
    for i in range(3):
        _check_read(st, b, i, vp, nbufs, bufsize)
    empty = st.submit()  # an empty batch completes too
    st.wait(empty)
    st.close()
    with pytest.raises(WgcsError):  # a one-slot ring could never hand back results
        Stager(dev, depth=1, max_reads=3, max_bytes=1 << 16, max_segs=nbufs, seg_room=bufsize - OFFSET)


def test_stager_fuzz_geometries(dev):
    """The handleVirtioRead header-fuzz corpus (tests/gso_cases.py: IP headers
    shorter than 6 / 20 bytes, checksum fields past hdrLen or past a short
    segment's end, wrapped u16 positions, errors) through the read stager:
    every read's bufs equal the oracle's byte for byte, including gsoSplit's
    header writes past a segment's end (copy_out runs such reads again through
    the per-call path with the caller's buffers staged)."""
    import itertools

    import gso_cases

    nbufs, bufsize = 16, 9000
    st = Stager(dev, depth=2, max_reads=32, max_bytes=32 * 65552, max_segs=nbufs, seg_room=bufsize - OFFSET)
    cases = [c[0] for c in itertools.islice(gso_cases.fuzz_cases(False), 400)]
    k = batches = 0
    while k < len(cases):
        chunk = []
        while k < len(cases) and len(chunk) < 32:
            try:
                st.push(cases[k])
            except WgcsError as e:
                if e.code != ERR_BATCH_FULL or not chunk:
                    raise
                break
            chunk.append(cases[k])
            k += 1
        b = st.submit()
        st.wait(b)
        batches += 1
        for i, vp in enumerate(chunk):
            _check_read(st, b, i, vp, nbufs, bufsize)
    st.close()
    assert batches >= 13
