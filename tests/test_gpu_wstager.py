"""GPU parity: the Tun.Write stager (wgcs_wstager_*) vs the oracle's
handleGRO per Write call -- status, toWrite and every byte Tun.Write hands to
write(2) (bufs[i][offset-10:len] for i in toWrite, tun/tun.go:687-698), for
many calls batched into one device handleGRO launch (one workgroup per call),
including invalid checksums, prepends, capacity limits, UDP GRO off, an
invalid offset, offsets other than 16 and Write calls with no buffers."""
import numpy as np
import pytest

import oracle
from wireguard_amd.tun import WriteStager

from test_gpu_gro import flow

pytestmark = pytest.mark.gpu
OFFSET = 16


def _mk(pkts, cap=65535, offset=OFFSET, lens_override=None):
    bufs, lens = [], []
    for p in pkts:
        b = np.full(cap if isinstance(cap, int) else cap(len(p)), 0x5A, np.uint8)
        b[offset: offset + len(p)] = np.frombuffer(p, np.uint8)
        bufs.append(b)
        lens.append(offset + len(p))
    for i, ln in (lens_override or {}).items():
        lens[i] = ln
    return bufs, lens


def _oracle_writes(pkts, cap, can_udp, offset, lens_override):
    bo, lo = _mk(pkts, cap, offset, lens_override)
    rc, tw, order, nl = oracle.handle_gro(bo, lo, offset, can_udp)
    if rc:
        return rc, [], []
    return 0, tw, [bo[order[i]][offset - 10: nl[i]].tobytes() for i in tw]


def _first_diff(got, want):
    """Where two lists of written packets first differ (for the assert message)."""
    if len(got) != len(want):
        return f"{len(got)} writes vs {len(want)}"
    for k, (g, w) in enumerate(zip(got, want)):
        if g != w:
            at = next((j for j in range(min(len(g), len(w))) if g[j] != w[j]), min(len(g), len(w)))
            return f"write {k}: len {len(g)} vs {len(w)}, first diff at byte {at}: {g[at:at + 8].hex()} vs {w[at:at + 8].hex()}"
    return "equal"


def _calls(seed):
    rng = np.random.default_rng(seed)
    calls = []
    for k in range(24):
        flows = [flow(int(rng.integers(1, 9)), seg=int(rng.choice([536, 1000, 1448])), v6=bool((k + j) % 2),
                      udp=bool((k + j) % 3 == 0), seed=1000 * seed + 10 * k + j,
                      last_flags=int(rng.choice([0x10, 0x18]))) for j in range(4)]
        batch = [p for f in flows for p in f]
        order = np.argsort(rng.random(len(batch)) + np.arange(len(batch)) * 0.1)
        pkts = [batch[i] for i in order][:128]
        cap, can_udp, lo = 65535, True, None
        if k % 5 == 1:  # bad checksums: the speculative plan is redone for this call
            for _ in range(3):
                i = int(rng.integers(0, len(pkts)))
                b = bytearray(pkts[i]); b[-1] ^= 0x21; pkts[i] = bytes(b)
        if k % 7 == 2:
            cap = lambda n: OFFSET + n + 1500  # noqa: E731  room for one more segment only
        if k % 6 == 3:
            can_udp = False
        if k % 11 == 4:
            lo = {len(pkts) // 2: OFFSET}  # invalid offset part-way: Write writes nothing
        if k % 4 == 0:  # a prepend: swap two neighbours of one flow
            f0 = flows[0]
            if len(f0) >= 2:
                pkts = [f0[1], f0[0]] + pkts[2:]
        calls.append((pkts, cap, can_udp, lo))
    return calls


@pytest.mark.parametrize("seed", [1, 2])
def test_write_stager_matches_handle_gro(dev, seed):
    calls = _calls(seed)
    ws = WriteStager(dev, depth=3, max_writes=16, max_pkts=16 * 128, max_bytes=16 * 128 * 1600)
    pending, expect = [], {}
    for ci, (pkts, cap, can_udp, lo) in enumerate(calls):
        bufs, lens = _mk(pkts, cap, OFFSET, lo)
        try:
            idx = ws.push(bufs, lens, OFFSET, can_udp)
        except Exception as e:  # BATCH_FULL: submit the open slot and push again
            assert getattr(e, "code", None) == -14, e
            pending.append(ws.submit())
            idx = ws.push(bufs, lens, OFFSET, can_udp)
        expect.setdefault(len(pending), []).append((ci, idx, len(pkts)))
    pending.append(ws.submit())
    checked = redone = 0
    for slot_k, batch in enumerate(pending):
        ws.wait(batch)
        for ci, idx, n in expect.get(slot_k, []):
            pkts, cap, can_udp, lo = calls[ci]
            rc, tw, writes = _oracle_writes(pkts, cap, can_udp, OFFSET, lo)
            err, tw_p, writes_p = ws.result(batch, idx, n)
            assert (0 if err is None else err.code) == rc, ci
            assert tw_p == tw, ci
            assert writes_p == writes, f"call {ci}: {_first_diff(writes_p, writes)}"
            checked += 1
    ws.close()
    assert checked == len(calls)


def test_write_stager_ring_reuse(dev):
    """More slots' worth of calls than the ring holds: every result is read
    before its slot is recycled (depth - 1 submits later)."""
    ws = WriteStager(dev, depth=2, max_writes=4, max_pkts=512, max_bytes=512 * 1600)
    calls = _calls(3)[:12]
    for r in range(0, len(calls), 4):
        idxs = []
        for pkts, cap, can_udp, lo in calls[r: r + 4]:
            bufs, lens = _mk(pkts, cap, OFFSET, lo)
            idxs.append(ws.push(bufs, lens, OFFSET, can_udp))
        b = ws.submit()
        ws.wait(b)
        for (pkts, cap, can_udp, lo), idx in zip(calls[r: r + 4], idxs):
            rc, tw, writes = _oracle_writes(pkts, cap, can_udp, OFFSET, lo)
            err, tw_p, writes_p = ws.result(b, idx, len(pkts))
            assert (0 if err is None else err.code, tw_p) == (rc, tw)
            assert writes_p == writes, _first_diff(writes_p, writes)
    ws.close()


@pytest.mark.parametrize("offset", [10, 13, 16, 40])
def test_write_stager_offsets(dev, offset):
    """Tun.Write offsets below and above the 16-byte headroom (the device slices
    put every packet on a 16-byte boundary whatever the offset), and an empty
    Write call between two real ones."""
    calls = _calls(4 + offset)[:6]
    ws = WriteStager(dev, depth=2, max_writes=8, max_pkts=8 * 128, max_bytes=8 * 128 * 1600)
    idxs = []
    for k, (pkts, cap, can_udp, lo) in enumerate(calls):
        if lo:  # the invalid-offset override is for OFFSET 16
            lo = {i: offset for i in lo}
        capk = cap if isinstance(cap, int) else (lambda n, c=cap: c(n) - OFFSET + offset)
        bufs, lens = _mk(pkts, capk, offset, lo)
        idxs.append(ws.push(bufs, lens, offset, can_udp))
        if k == 2:
            idxs.append(ws.push([], [], offset, True))
    b = ws.submit()
    ws.wait(b)
    j = 0
    for k, (pkts, cap, can_udp, lo) in enumerate(calls):
        if lo:
            lo = {i: offset for i in lo}
        capk = cap if isinstance(cap, int) else (lambda n, c=cap: c(n) - OFFSET + offset)
        rc, tw, writes = _oracle_writes(pkts, capk, can_udp, offset, lo)
        err, tw_p, writes_p = ws.result(b, idxs[j], len(pkts))
        assert (0 if err is None else err.code, tw_p) == (rc, tw), k
        assert writes_p == writes, f"call {k}: {_first_diff(writes_p, writes)}"
        j += 1
        if k == 2:
            err, tw_p, writes_p = ws.result(b, idxs[j], 0)
            assert err is None and tw_p == [] and writes_p == []
            j += 1
    ws.close()


def test_write_stager_rejects_oversized_call(dev):
    """A Write call holds at most conn.BatchSize (128) buffers (WGCS_GRO_MAX_CALL)."""
    ws = WriteStager(dev, depth=2, max_writes=4, max_pkts=512, max_bytes=512 * 1600)
    pkts = [p for _ in range(5) for p in flow(26, seed=7)][:129]
    bufs, lens = _mk(pkts)
    with pytest.raises(Exception) as ei:
        ws.push(bufs, lens, OFFSET, True)
    assert getattr(ei.value, "code", None) == -1, ei.value
    ws.close()


def test_write_stager_concurrent_pushes(dev):
    """Write calls pushed from 4 threads at once (the packet copies run outside
    the stager's lock): every call's results still match its own handleGRO."""
    import threading

    calls = _calls(5)[:16]
    ws = WriteStager(dev, depth=2, max_writes=16, max_pkts=16 * 128, max_bytes=16 * 128 * 1600)
    staged = [None] * len(calls)
    keep = []

    def worker(t):
        for k in range(t, len(calls), 4):
            pkts, cap, can_udp, lo = calls[k]
            bufs, lens = _mk(pkts, cap, OFFSET, lo)
            keep.append(bufs)
            staged[k] = ws.push(bufs, lens, OFFSET, can_udp)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert sorted(staged) == list(range(len(calls)))
    b = ws.submit()
    ws.wait(b)
    for k, (pkts, cap, can_udp, lo) in enumerate(calls):
        rc, tw, writes = _oracle_writes(pkts, cap, can_udp, OFFSET, lo)
        err, tw_p, writes_p = ws.result(b, staged[k], len(pkts))
        assert (0 if err is None else err.code, tw_p) == (rc, tw), k
        assert writes_p == writes, f"call {k}: {_first_diff(writes_p, writes)}"
    ws.close()


def _mk_pinned(pool, at, pkts, cap, offset, lens_override, phase):
    """The packets in Go-slice buffers carved out of pinned host memory
    (Device.host_alloc) at 16-byte phases `phase(i)`; returns (bufs, lens, at)."""
    bufs, lens = [], []
    for i, p in enumerate(pkts):
        c = cap if isinstance(cap, int) else cap(len(p))
        at += phase(i)
        b = pool[at: at + c]
        b[:] = 0x5A
        b[offset: offset + len(p)] = np.frombuffer(p, np.uint8)
        bufs.append(b)
        lens.append(offset + len(p))
        at = (at + c + 15) // 16 * 16
    for i, ln in (lens_override or {}).items():
        lens[i] = ln
    return bufs, lens, at


def test_write_stager_pinned_zero_copy(dev):
    """wgcs_wstager_push_pinned: the scatter kernel reads the packets straight
    from pinned host memory (buffers at every 16-byte phase), mixed in one slot
    with copying pushes; every call's write(2) images equal handleGRO's."""
    calls = _calls(6)[:12]
    total = sum(sum((c if isinstance(c, int) else c(len(p))) + 32 for p in pk) for pk, c, _, _ in calls)
    pool = dev.host_alloc(total + 4096)
    ws = WriteStager(dev, depth=2, max_writes=16, max_pkts=16 * 128, max_bytes=16 * 128 * 1600)
    at, idxs, keep = 0, [], []
    for k, (pkts, cap, can_udp, lo) in enumerate(calls):
        if k % 3 == 2:  # a copying push in between
            bufs, lens = _mk(pkts, cap, OFFSET, lo)
            keep.append(bufs)
            idxs.append(ws.push(bufs, lens, OFFSET, can_udp))
        else:
            bufs, lens, at = _mk_pinned(pool, at, pkts, cap, OFFSET, lo, lambda i, k=k: (i * 7 + k) % 16)
            idxs.append(ws.push_pinned(bufs, lens, OFFSET, can_udp))
    b = ws.submit()
    ws.wait(b)
    for k, (pkts, cap, can_udp, lo) in enumerate(calls):
        rc, tw, writes = _oracle_writes(pkts, cap, can_udp, OFFSET, lo)
        err, tw_p, writes_p = ws.result(b, idxs[k], len(pkts))
        assert (0 if err is None else err.code, tw_p) == (rc, tw), k
        assert writes_p == writes, f"call {k}: {_first_diff(writes_p, writes)}"
    ws.close()
    dev.host_free(pool)


def test_write_stager_pinned_rejects_pageable(dev):
    """push_pinned refuses buffers that are not wgcs_host_alloc memory."""
    ws = WriteStager(dev, depth=2, max_writes=4, max_pkts=512, max_bytes=512 * 1600)
    bufs, lens = _mk(flow(4, seed=9))
    with pytest.raises(Exception) as ei:
        ws.push_pinned(bufs, lens, OFFSET, True)
    assert getattr(ei.value, "code", None) == -1, ei.value
    ws.close()


def test_write_stager_concurrent_submits(dev):
    """Four pushing threads and two submitting threads at once (a
    submit that waited for copying pushes must not queue a stale slot): every
    submit returns a distinct batch, and the calls found in the submitted
    batches are exactly the pushed calls, each with its own handleGRO result."""
    import threading

    calls = _calls(8)[:16]
    ws = WriteStager(dev, depth=16, max_writes=4, max_pkts=4 * 128, max_bytes=4 * 128 * 1600)
    lock = threading.Lock()
    batches, keep = [], []
    stop = threading.Event()

    def submit():
        b = ws.submit()
        with lock:
            batches.append(b)

    def pusher(t):
        for k in range(t, len(calls), 4):
            pkts, cap, can_udp, lo = calls[k]
            bufs, lens = _mk(pkts, cap, OFFSET, lo)
            with lock:
                keep.append(bufs)
            while True:
                try:
                    ws.push(bufs, lens, OFFSET, can_udp)
                    break
                except Exception as e:  # BATCH_FULL: submit the open slot and push again
                    assert getattr(e, "code", None) == -14, e
                    submit()

    def submitter():
        for _ in range(3):
            if stop.wait(0.002):
                break
            submit()

    th = [threading.Thread(target=pusher, args=(t,)) for t in range(4)] + \
         [threading.Thread(target=submitter) for _ in range(2)]
    for x in th:
        x.start()
    for x in th[:4]:
        x.join()
    stop.set()
    for x in th[4:]:
        x.join()
    submit()
    assert len(batches) < 16, "results would have been recycled"
    assert len(set(batches)) == len(batches), f"a slot was submitted twice: {batches}"
    want = {}
    for k, (pkts, cap, can_udp, lo) in enumerate(calls):
        rc, tw, writes = _oracle_writes(pkts, cap, can_udp, OFFSET, lo)
        want[k] = (rc, tw, writes)
    found = []
    for b in batches:
        ws.wait(b)
        idx = 0
        while True:
            try:
                err, tw_p, writes_p = ws.result(b, idx, 128)
            except Exception as e:
                assert getattr(e, "code", None) == -1, e  # past the slot's last call
                break
            found.append((0 if err is None else err.code, tw_p, writes_p))
            idx += 1
    assert len(found) == len(calls)
    for k, w in want.items():  # the seeded flows make every call's writes distinct
        assert found.count(w) >= 1, f"call {k} missing from the submitted batches"
    ws.close()


def test_host_free_refused_while_a_slot_reads_it(dev):
    """wgcs_host_free refuses (NOT_READY) pinned memory that an open write-stager
    slot still reads through a zero-copy push; after the slot ran it succeeds."""
    pkts = flow(6, seed=11)
    pool = dev.host_alloc(8 * 65536)
    ws = WriteStager(dev, depth=2, max_writes=4, max_pkts=512, max_bytes=512 * 1600)
    bufs, lens, _ = _mk_pinned(pool, 0, pkts, 65535, OFFSET, None, lambda i: 0)
    idx = ws.push_pinned(bufs, lens, OFFSET, True)
    with pytest.raises(Exception) as ei:
        dev.host_free(pool)
    assert getattr(ei.value, "code", None) == -15, ei.value
    b = ws.submit()
    ws.wait(b)
    rc, tw, writes = _oracle_writes(pkts, 65535, True, OFFSET, None)
    err, tw_p, writes_p = ws.result(b, idx, len(pkts))
    assert (0 if err is None else err.code, tw_p, writes_p) == (rc, tw, writes)
    dev.host_free(pool)
    ws.close()


def test_write_stager_quirk_calls(dev):
    """The quirk calls (capacities above 64 KiB: items and their uint16 length
    fields grow past 65,535; a mid-flow PSH; sequence numbers wrapping) through
    the write stager, every write(2) image vs the oracle."""
    from test_gpu_gro_batch import quirk_calls

    calls = quirk_calls()
    ws = WriteStager(dev, depth=2, max_writes=16, max_pkts=16 * 128, max_bytes=16 * 128 * 1600)
    keep, idxs = [], []
    for pkts, cap, can_udp, lo in calls:
        bufs, lens = _mk(pkts, cap, OFFSET, lo)
        keep.append(bufs)
        idxs.append(ws.push(bufs, lens, OFFSET, can_udp))
    b = ws.submit()
    ws.wait(b)
    for k, (pkts, cap, can_udp, lo) in enumerate(calls):
        rc, tw, writes = _oracle_writes(pkts, cap, can_udp, OFFSET, lo)
        err, tw_p, writes_p = ws.result(b, idxs[k], len(pkts))
        assert (0 if err is None else err.code, tw_p) == (rc, tw), k
        assert writes_p == writes, f"call {k}: {_first_diff(writes_p, writes)}"
    ws.close()


def test_write_stager_field_fuzz(dev):
    """The header-field fuzz calls (tests/gro_cases.py) through the write
    stager, 16 calls per batch, every write(2) image vs the oracle."""
    import gro_cases

    calls = gro_cases.field_fuzz_calls()
    ws = WriteStager(dev, depth=2, max_writes=16, max_pkts=16 * 128, max_bytes=16 * 128 * 1600)
    for lo_k in range(0, len(calls), 16):
        part = calls[lo_k: lo_k + 16]
        keep, idxs = [], []
        for pkts, cap, can_udp, lo in part:
            bufs, lens = _mk(pkts, cap, OFFSET, lo)
            keep.append(bufs)
            idxs.append(ws.push(bufs, lens, OFFSET, can_udp))
        b = ws.submit()
        ws.wait(b)
        for k, (pkts, cap, can_udp, lo) in enumerate(part):
            rc, tw, writes = _oracle_writes(pkts, cap, can_udp, OFFSET, lo)
            err, tw_p, writes_p = ws.result(b, idxs[k], len(pkts))
            assert (0 if err is None else err.code, tw_p) == (rc, tw), lo_k + k
            assert writes_p == writes, f"call {lo_k + k}: {_first_diff(writes_p, writes)}"
    ws.close()
