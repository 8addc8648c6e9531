"""GPU tests of the C ABI's lifetime and thread-safety contract (VERDICT r3
items 6-7): include/wgcsum.h calls the entry points thread-safe, and Tun.Write
runs on many goroutines at once (/root/reference/tun/tun.go:654-700,
device/peer.go:191).

- a zero-copy push (wgcs_wstager_push_pinned) racing wgcs_host_free of the
  same pinned buffer: exactly one side fails, and a push that succeeded reads
  memory that is still allocated (its handleGRO result equals the oracle's);
- wgcs_destroy refuses while a read stager (or a write stager) is alive;
- wgcs_last_error is per thread: concurrent failing callers each read their
  own message."""
import ctypes as C
import threading

import numpy as np
import pytest

from wireguard_amd import WgcsError
from wireguard_amd.tun import Device, WriteStager

from test_gpu_gro import flow
from test_gpu_wstager import OFFSET, _mk_pinned, _oracle_writes

pytestmark = pytest.mark.gpu

INVALID_ARG, NOT_READY = -1, -15


def test_push_pinned_races_host_free(dev):
    """One thread pushes a Write call from a pinned buffer while another frees
    that buffer, released together by a barrier, 48 times: exactly one of the
    two fails (the push with INVALID_ARG, or the free with NOT_READY), no
    fault occurs, and every successful push's writes equal handleGRO's."""
    pkts = flow(6, seed=21)
    rc_o, tw_o, writes_o = _oracle_writes(pkts, 65535, True, OFFSET, None)
    ws = WriteStager(dev, depth=2, max_writes=4, max_pkts=512, max_bytes=512 * 1600)
    outcomes = {"push": 0, "free": 0}
    for it in range(48):
        pool = dev.host_alloc(8 * 65536)
        bufs, lens, _ = _mk_pinned(pool, 0, pkts, 65535, OFFSET, None, lambda i, it=it: (i + it) % 16)
        addr = pool.ctypes.data
        gate = threading.Barrier(2)
        res = {}

        def push():
            gate.wait()
            try:
                res["idx"] = ws.push_pinned(bufs, lens, OFFSET, True)
            except WgcsError as e:
                res["push_err"] = e.code

        def free():
            gate.wait()
            rc = dev.lib.wgcs_host_free(dev.h, C.c_void_p(addr))  # raw call: the view must not be touched after
            res["free_rc"] = rc

        th = [threading.Thread(target=push), threading.Thread(target=free)]
        if it % 2:
            th.reverse()
        for t in th:
            t.start()
        for t in th:
            t.join()
        pushed, freed = "idx" in res, res["free_rc"] == 0
        assert pushed != freed, (it, res)
        if pushed:
            assert res["free_rc"] == NOT_READY, res
            outcomes["push"] += 1
            b = ws.submit()
            ws.wait(b)
            err, tw_p, writes_p = ws.result(b, res["idx"], len(pkts))
            assert (0 if err is None else err.code, tw_p, writes_p) == (rc_o, tw_o, writes_o), it
            dev.host_free(pool)  # the slot has run: now the free succeeds
        else:
            assert res["push_err"] == INVALID_ARG, res
            outcomes["free"] += 1
        del bufs, pool
    ws.close()
    print("race outcomes", outcomes)


def test_destroy_refuses_live_read_stager():
    """wgcs_destroy with a live read stager returns INVALID_ARG and leaves the
    context usable; after the stager is destroyed it succeeds.  Device.close
    raises instead of dropping the context."""
    d = Device(0)
    lib = d.lib
    st = C.c_void_p()
    assert lib.wgcs_stager_create(d.h, 2, 4, 1 << 20, 16, 9000, C.byref(st)) == 0
    assert lib.wgcs_destroy(d.h) == INVALID_ARG
    assert b"read stager" in lib.wgcs_last_error(d.h)
    with pytest.raises(WgcsError) as ei:
        d.close()
    assert ei.value.code == INVALID_ARG and d.h  # the context is kept
    assert d.checksum(b"\x45\x00\x00\x1c") == (0x4500 + 0x001C)  # still usable
    assert lib.wgcs_stager_destroy(st) == 0
    d.close()
    assert d.h is None


def test_destroy_refuses_live_write_stager():
    d = Device(0)
    lib = d.lib
    ws = C.c_void_p()
    assert lib.wgcs_wstager_create(d.h, 2, 4, 512, 512 * 1600, C.byref(ws)) == 0
    assert lib.wgcs_destroy(d.h) == INVALID_ARG
    assert lib.wgcs_wstager_destroy(ws) == 0
    assert lib.wgcs_destroy(d.h) == 0
    d.h = None


def test_last_error_is_per_thread(dev):
    """Two threads fail on the same context at once, each with its own
    message, 2,000 times: each reads back exactly its own message."""
    lib = dev.lib
    ws = WriteStager(dev, depth=2, max_writes=4, max_pkts=512, max_bytes=512 * 1600)
    n = 129  # one more than conn.BatchSize: refused with a message naming the count
    ptrs = (C.c_void_p * n)()
    sz = (C.c_size_t * n)(*([100] * n))
    idx = C.c_int(0)
    bad = []
    gate = threading.Barrier(2)

    def mode_errors():
        gate.wait()
        for k in range(2000):
            rc = lib.wgcs_checksum_batch(dev.h, 90 + k % 7, 0, None, None, None, 1, None, None)
            msg = lib.wgcs_last_error(dev.h)
            if rc != INVALID_ARG or msg != f"bad mode {90 + k % 7}".encode():
                bad.append(("mode", k, rc, msg))

    def push_errors():
        gate.wait()
        for k in range(2000):
            rc = lib.wgcs_wstager_push(ws.h, ptrs, sz, sz, n, OFFSET, 1, C.byref(idx))
            msg = lib.wgcs_last_error(dev.h)
            if rc != INVALID_ARG or b"129 buffers" not in msg:
                bad.append(("push", k, rc, msg))

    th = [threading.Thread(target=mode_errors), threading.Thread(target=push_errors)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    ws.close()
    assert not bad, bad[:5]
    # a thread that has not failed on this context reads ""
    out = []
    t = threading.Thread(target=lambda: out.append(lib.wgcs_last_error(dev.h)))
    t.start()
    t.join()
    assert out == [b""]


def test_empty_calls_return_nothing(dev):
    """len(bufs) == 0 through every per-call entry point (the cgo shims'
    empty-call guards in INTEGRATION.md mirror this): handleGRO returns nil and
    writes nothing (gro.go:1334-1366, tun.go:654-700), gsoSplit returns
    (-1, ErrTooManySegments) or (0, nil) without touching bufs."""
    to_write, order, lens, err = dev.handle_gro([], [], OFFSET, True)
    assert (to_write, order, lens, err) == ([], [], [], None)
    tw = (C.c_int * 1)()
    ntw = C.c_int(-1)
    assert dev.lib.wgcs_handle_gro(dev.h, None, None, None, 0, OFFSET, 1, tw, C.byref(ntw)) == 0 and ntw.value == 0
    ws = WriteStager(dev, depth=2, max_writes=4, max_pkts=512, max_bytes=512 * 1600)
    i = ws.push([], [], OFFSET)
    b = ws.submit()
    ws.wait(b)
    assert ws.result(b, i, 0) == (None, [], [])
    ws.close()


def test_stream_wait_flag_doorbell(dev):
    """wgcs_stream_wait_flag: a batch posted behind the doorbell does not run
    until the host rings it, then runs exactly as an ungated one (bench.py
    posts its timed steps this way).  Non-mapped flags are refused."""
    import time

    import torch

    import oracle
    from wireguard_amd import synth
    from wireguard_amd.tun import MODE_VALIDATE

    arena, pkts, _ = synth.make_batch(512, 1500, kinds="mixed")
    d_arena = torch.from_numpy(arena).cuda()
    d_pkts = torch.from_numpy(pkts.view(np.uint8)).cuda()
    d_out = torch.full((512,), 7, dtype=torch.uint8, device="cuda")
    bell = dev.host_alloc(64).view(np.uint32)
    with pytest.raises(WgcsError):
        dev.stream_wait_flag(None, np.zeros(4, np.uint32), 1)  # pageable memory
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    bell[0] = 0
    dev.stream_wait_flag(s, bell, 1)
    dev.checksum_batch(MODE_VALIDATE, d_arena, d_pkts, 512, d_out, stream=s)
    ev = torch.cuda.Event()
    ev.record(s)
    time.sleep(0.05)
    gated = not ev.query()
    bell[0] = 1  # ring (always, before any wait on the stream)
    t0 = time.time()
    while not ev.query():
        assert time.time() - t0 < 10, "doorbell never released the stream"
        time.sleep(0.001)
    assert gated, "the batch ran before the doorbell was rung"
    want = oracle.checksum_batch(MODE_VALIDATE, arena, pkts)
    assert np.array_equal(d_out.cpu().numpy(), want) and want.all()
    dev.host_free(bell.view(np.uint8))


def test_doorbell_gates_every_stream_without_events(dev):
    """bench.py's gate with --no-event-timing and two launch streams: every
    launch stream waits on the doorbell itself, so no batch of the series runs
    before the ring even with no bracket events joining the streams (ADVICE
    r4: only stream 0 used to be gated).  The gate is bench.gate_streams, the
    helper bench.py's timed region calls."""
    import os
    import sys
    import time

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    import oracle
    from wireguard_amd import synth
    from wireguard_amd.tun import MODE_VALIDATE

    arena, pkts, _ = synth.make_batch(512, 1500, kinds="mixed")
    d_arena = torch.from_numpy(arena).cuda()
    d_pkts = torch.from_numpy(pkts.view(np.uint8)).cuda()
    outs = [torch.full((512,), 7, dtype=torch.uint8, device="cuda") for _ in range(4)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bell = dev.host_alloc(64).view(np.uint32)
    torch.cuda.synchronize()
    bell[0] = 0
    gated = bench.gate_streams(dev, bell, streams, use_events=False)
    assert len(gated) == len(streams)
    dev.checksum_batches(MODE_VALIDATE, dev.batch_list([(d_arena, d_pkts, 512, o) for o in outs]), streams)
    evs = [torch.cuda.Event() for _ in streams]
    for e, s in zip(evs, streams):
        e.record(s)
    time.sleep(0.05)
    ran = [e.query() for e in evs]
    bell[0] = 1  # ring before any assert: never leave a stream gated
    torch.cuda.synchronize()
    assert not any(ran), f"a stream ran before the doorbell: {ran}"
    want = oracle.checksum_batch(MODE_VALIDATE, arena, pkts)
    for o in outs:
        assert np.array_equal(o.cpu().numpy(), want)
    dev.host_free(bell.view(np.uint8))
