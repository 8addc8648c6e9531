"""Outer-UDP message batching measurement: device-resident
splitMessages / coalesceMessages (conn/bind.go:542-662) on one MI355X.
Called by bench.py --config udp_split | udp_coalesce.

udp_split:    1024 recvmmsg batches; each has the receive path's shape
              (BatchSize 128, readAt 126, conn/bind.go:293): two UDP_GRO
              datagrams of 45 x 1452-B WireGuard transport messages (MTU-1420
              tunnel + 32 B of header/tag) -> 90 packets per batch.
udp_coalesce: 1024 Send batches of 128 x 1452-B transport messages (IPv4
              peer) -> runs of 45 / 45 / 38 appended into 3 messages.
Algorithmic bytes per launch = payload bytes read + written (each packet byte
moves once: the first buffer of a coalesced run stays where it is).
"""
from __future__ import annotations

import json
import os
import time

import numpy as np

from . import shard, synth, traffic

HBM_PEAK_GBS = 8000.0
MSG = 1452  # transport message for a 1420-B tunnel MTU: 16-B header + 1420 + 16-B tag
SEGS = 45  # 45 * 1452 = 65340 <= maxIPv4PayloadLen 65507 < 46 * 1452


def _oracle():
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle  # cpu_baseline / host-call comparison only

    return oracle


def _gro_cmsg(g):
    return (18).to_bytes(8, "little") + (17).to_bytes(4, "little") + (104).to_bytes(4, "little") + \
        int(g).to_bytes(2, "little") + bytes(6)


def _time_steps(torch, streams, step, steps, warmup, barrier):
    """Step k runs on streams[k % S] (consecutive batches are independent);
    returns (wall seconds, GPU ms per launch over the timed region, the same
    on one stream or None)."""
    S = len(streams)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    joins = [torch.cuda.Event() for _ in streams[1:]]

    def timed(K, k0, ns):
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(streams[0])
        for st in streams[1:ns]:
            st.wait_event(e0)
        for k in range(K):
            step(k0 + k, ns)
        for j, st in zip(joins, streams[1:ns]):
            j.record(st)
            streams[0].wait_event(j)
        e1.record(streams[0])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        barrier()
        return el, e0.elapsed_time(e1) / K

    # the one-stream reference first (as bench.py: measured after a two-stream
    # burst, launches read slower, profiles/r2_probe_iso_order.txt), then the W
    # warmup steps through the same bracket as the K timed ones
    iso = None
    if S > 1:
        timed(min(warmup, 5), 0, 1)
        iso = timed(max(steps, 10), 0, 1)[1]
    if warmup > 0:
        timed(warmup, 0, S)
    el, ms = timed(steps, warmup, S)
    return el, ms, iso


def _copy_ms(torch, stream, dsts, srcs, nbytes, steps):
    """Calibration: the runtime's device copy kernel moving the same bytes,
    rotated over the bench's buffer copies like the kernel's steps (one fixed
    pair of ~134 MB buffers would be partly served by the 256 MB MALL)."""
    R = len(dsts)
    with torch.cuda.stream(stream):
        for k in range(3):
            dsts[k % R][:nbytes].copy_(srcs[k % R][:nbytes])
        c0 = torch.cuda.Event(enable_timing=True)
        c1 = torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        for k in range(steps):
            dsts[k % R][:nbytes].copy_(srcs[k % R][:nbytes])
        c1.record(stream)
    torch.cuda.synchronize()
    return c0.elapsed_time(c1) / steps


def run(args, torch, dev, dist, rank, world, local, barrier):
    if args.config == "udp_split":
        res = run_split(args, torch, dev, rank, world, barrier)
    else:
        res = run_coalesce(args, torch, dev, rank, world, barrier)
    elapsed = shard.max_over_ranks(res.pop("_elapsed"), dist)
    bps = res["roofline"]["algorithmic_bytes_per_launch"]
    res["value"] = round(bps * args.steps * world / elapsed / 2**30, 2)
    res["ms_per_step"] = round(elapsed / args.steps * 1e3, 5)
    res["n_gpus"] = world
    res["config"]["parallelism"] = f"shard{world} (no collective)"
    if rank == 0:
        print(json.dumps(res), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def _result(metric, args, workload, extra, kname, kern_ms, bps, copy_ms, elapsed, iso_ms=None, S=1):
    achieved = bps / (kern_ms * 1e-3) / 1e9
    res = {
        "metric": metric, "value": None, "unit": "GiB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic", "config": {"workload": workload, **extra},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic.per_launch(kname, bps), "kernel": kname,
                     "kernel_ms": round(kern_ms, 5),
                     "kernel_ms_is": ("GPU time per launch over the timed region (HIP events on the launch streams)"
                                      + (f"; {S} streams, consecutive launches overlap" if S > 1 else "")),
                     "algorithmic_bytes_per_launch": bps,
                     "d2d_copy_same_bytes_ms": round(copy_ms, 5)},
        "_elapsed": elapsed,
    }
    res["config"]["streams"] = S
    if iso_ms is not None:
        res["roofline"]["kernel_ms_one_stream"] = round(iso_ms, 5)
        res["roofline"]["frac_one_stream"] = round(bps / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    return res


# --------------------------------------------------------------------- split
def run_split(args, torch, dev, rank, world, barrier, B=1024, n_msgs=128, first=126):
    ns = n_msgs - first
    rng = np.random.default_rng(synth.SEED + 77 + rank)
    in_stride, out_stride, buf_len = 65536, 1456, 65535
    R = 2
    srcs = rng.integers(0, 256, (B * ns, SEGS * MSG), dtype=np.uint8)
    n_in = np.zeros(B * n_msgs, np.int32)
    gso = np.zeros(B * n_msgs, np.int32)
    for b in range(B):
        n_in[b * n_msgs + first: (b + 1) * n_msgs] = SEGS * MSG
        gso[b * n_msgs + first: (b + 1) * n_msgs] = MSG
    S = max(1, getattr(args, "streams", 1))
    streams = [torch.cuda.Stream() for _ in range(S)]
    stream = streams[0]
    R = max(R, S)
    d_in = []
    for _ in range(R):
        t = torch.zeros((B * ns, in_stride), dtype=torch.uint8, device="cuda")
        t[:, : SEGS * MSG].copy_(torch.from_numpy(srcs))
        d_in.append(t)
    d_n, d_g = torch.from_numpy(n_in).cuda(), torch.from_numpy(gso).cuda()
    d_out = [torch.empty((B * n_msgs, out_stride), dtype=torch.uint8, device="cuda") for _ in range(R)]
    # per-stream result arrays: launches on different streams may overlap
    d_nout = [torch.zeros(B * n_msgs, dtype=torch.int32, device="cuda") for _ in range(S)]
    d_src = [torch.zeros(B * n_msgs, dtype=torch.int32, device="cuda") for _ in range(S)]
    d_cnt = [torch.zeros(B, dtype=torch.int32, device="cuda") for _ in range(S)]
    d_st = [torch.zeros(B, dtype=torch.int32, device="cuda") for _ in range(S)]
    L, h = dev.lib, dev.h

    def step(k, ns):
        i, q = k % R, k % ns
        rc = L.wgcs_split_messages_batch(h, d_in[i].data_ptr(), in_stride, buf_len, d_n.data_ptr(), d_g.data_ptr(),
                                         n_msgs, first, B, d_out[i].data_ptr(), out_stride, d_nout[q].data_ptr(),
                                         d_src[q].data_ptr(), d_cnt[q].data_ptr(), d_st[q].data_ptr(),
                                         streams[q].cuda_stream)
        assert rc == 0

    elapsed, kern_ms, iso_ms = _time_steps(torch, streams, step, args.steps, args.warmup, barrier)
    cnt, st = d_cnt[0].cpu().numpy(), d_st[0].cpu().numpy()
    assert (st == 0).all() and (cnt == ns * SEGS).all(), (st[:4], cnt[:4])
    # size-independent property: packet k of batch b is bytes [k*1452, +1452) of its datagram
    out = d_out[0].view(B, n_msgs, out_stride)
    for b in (0, B // 2, B - 1):
        got = out[b, : ns * SEGS, :MSG].cpu().numpy().reshape(-1)
        assert np.array_equal(got, srcs[b * ns:(b + 1) * ns].reshape(-1)), b
    payload = B * ns * SEGS * MSG
    bps = 2 * payload
    copy_ms = _copy_ms(torch, stream, [o.view(-1) for o in d_out], [t.view(-1) for t in d_in], payload, args.steps)
    res = _result("device-resident UDP GRO split GiB/s (bytes read + written), 1024 recvmmsg batches x 2 x 45 x 1452 B",
                  args, f"{B} recvmmsg batches (BatchSize {n_msgs}, readAt {first}): {ns} UDP_GRO datagrams of "
                  f"{SEGS} x {MSG}-B transport messages each -> {ns * SEGS} packets per batch; splitMessages, "
                  "conn/bind.go:542-597 (SURVEY.md §8f row 3)",
                  {"batches": B, "packets_per_step": B * ns * SEGS, "payload_bytes": payload, "rotated_copies": R},
                  "udp_split_kernel<6>", kern_ms, bps, copy_ms, elapsed, iso_ms, S)
    if rank == 0 and world == 1 and not getattr(args, "no_e2e", False):
        res["host_call"] = split_host_call(dev, with_cpu=args.cpu_seconds > 0)
        if args.cpu_seconds > 0:
            res["cpu_baseline"] = split_cpu_baseline(srcs, args.cpu_seconds)
    return res


def split_host_call(dev, with_cpu: bool, reps: int = 200):
    """Latency of one reference-shaped splitMessages call (wgcs_split_messages:
    128 host buffers, 2 GRO datagrams at 126/127) -- one C call, prebuilt args."""
    import ctypes as C

    rng = np.random.default_rng(5)
    n_msgs, first = 128, 126
    bufs = [np.zeros(65535, np.uint8) for _ in range(n_msgs)]
    for s in (126, 127):
        bufs[s][: SEGS * MSG] = rng.integers(0, 256, SEGS * MSG, dtype=np.uint8)
    ctl = np.frombuffer(_gro_cmsg(MSG), np.uint8).copy()
    u8p = C.POINTER(C.c_uint8)
    cb = (u8p * n_msgs)(*[C.cast(b.ctypes.data, u8p) for b in bufs])
    oobs = (u8p * n_msgs)(*[C.cast(ctl.ctypes.data, u8p)] * n_msgs)
    nns = (C.c_size_t * n_msgs)(*([0] * first + [len(ctl)] * 2))
    ns = (C.c_int * n_msgs)()
    src = (C.c_int * n_msgs)()
    npk = C.c_int(0)

    def reset():
        for i in range(n_msgs):
            ns[i] = SEGS * MSG if i >= first else 0

    def timed(fn):
        ts = []
        for _ in range(reps):
            reset()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    gpu = timed(lambda: dev.lib.wgcs_split_messages(dev.h, cb, 65535, ns, oobs, nns, n_msgs, first, src,
                                                    C.byref(npk)))
    assert npk.value == 90
    out = {"call": "wgcs_split_messages, one recvmmsg batch (2 x 45 x 1452 B -> 90 packets), host buffers",
           "median_us": round(gpu * 1e6, 1)}
    if with_cpu:
        oracle = _oracle()
        O = oracle._conn_lib()
        arr = (oracle._OrMsg * n_msgs)()

        def cpu():
            for i in range(n_msgs):
                arr[i] = oracle._OrMsg(bufs[i].ctypes.data, 65535, 65535, ns[i], ctl.ctypes.data, len(ctl), len(ctl),
                                       nns[i], i)
            O.or_split_messages(arr, n_msgs, first, C.byref(npk))

        out["cpu_oracle_median_us"] = round(timed(cpu) * 1e6, 1)
        out["cpu_oracle_note"] = "includes ~128 ctypes struct fills per call"
    return out


def _threaded_rate(make_pass, threads, seconds):
    """All-cores leg: `threads` Python threads, each running passes of its own
    state (make_pass() -> (one_pass, bytes_per_pass)); the oracle's C calls
    release the GIL (ctypes), so the threads run on separate cores.  Rate =
    sum over threads of bytes / time inside its passes."""
    import threading

    out = [None] * threads
    go = threading.Barrier(threads)

    def work(t):
        one, nbytes = make_pass()
        go.wait()
        busy, reps, t_end = 0.0, 0, time.perf_counter() + seconds
        while time.perf_counter() < t_end:
            t0 = time.perf_counter()
            one()
            busy += time.perf_counter() - t0
            reps += 1
        out[t] = (nbytes * reps / busy if busy > 0 else 0.0, reps)

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    return sum(r for r, _ in out), sum(n for _, n in out)


def split_cpu_baseline(srcs, seconds, B=16, n_msgs=128, first=126):
    """The oracle (C restatement of splitMessages) on B batches of the same
    shape: 1 thread for `seconds`, then every host thread (all_cores)."""
    import ctypes as C

    oracle = _oracle()
    L = oracle._conn_lib()
    L.or_split_batch.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                 C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    L.or_split_batch.restype = None
    ns_ = n_msgs - first
    bps = 2 * B * ns_ * SEGS * MSG

    def make_pass():
        bufs = np.zeros((B * n_msgs, 65535), np.uint8)
        ns0 = np.zeros(B * n_msgs, np.int32)
        oobs = np.zeros((B * n_msgs, 24), np.uint8)
        nns = np.zeros(B * n_msgs, np.int32)
        for b in range(B):
            for t in range(ns_):
                q = b * n_msgs + first + t
                bufs[q, : SEGS * MSG] = srcs[b * ns_ + t]
                ns0[q] = SEGS * MSG
                oobs[q] = np.frombuffer(_gro_cmsg(MSG), np.uint8)
                nns[q] = 24
        cnt = np.zeros(B, np.int32)
        st = np.zeros(B, np.int32)

        def one():
            ns = ns0.copy()
            L.or_split_batch(bufs.ctypes.data, 65535, 65535, ns.ctypes.data, oobs.ctypes.data, 24, nns.ctypes.data,
                             n_msgs, first, B, cnt.ctypes.data, st.ctypes.data)
            assert (cnt == ns_ * SEGS).all() and (st == 0).all()
        return one, bps

    rate, reps = _threaded_rate(make_pass, 1, seconds)
    threads = oracle.host_threads()
    arate, areps = _threaded_rate(make_pass, threads, seconds)
    return {"value": round(rate / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{reps} passes over {B} recvmmsg batches of the same shape, {seconds:.1f} s, "
                      "C restatement of splitMessages (bytes read + written)",
            "all_cores": {"value": round(arate / 2**30, 3), "unit": "GiB/s", "cores": threads,
                          "host_nproc": os.cpu_count(),
                          "sample": f"{areps} passes, one private copy of the {B} batches per thread"}}


# ------------------------------------------------------------------ coalesce
def run_coalesce(args, torch, dev, rank, world, barrier, B=1024, max_bufs=128):
    import os

    stride, cap = int(os.environ.get("WGCS_UDP_STRIDE", 65536)), 65535
    rng = np.random.default_rng(synth.SEED + 88 + rank)
    S = max(1, getattr(args, "streams", 1))
    streams = [torch.cuda.Stream() for _ in range(S)]
    stream = streams[0]
    R = max(2, S)
    pk = rng.integers(0, 256, (B * max_bufs, MSG), dtype=np.uint8)
    d_bufs = []
    for _ in range(R):
        t = torch.zeros((B * max_bufs, stride), dtype=torch.uint8, device="cuda")
        t[:, :MSG].copy_(torch.from_numpy(pk))
        d_bufs.append(t)
    d_lens = torch.full((B * max_bufs,), MSG, dtype=torch.int32, device="cuda")
    d_nb = torch.full((B,), max_bufs, dtype=torch.int32, device="cuda")
    d_nm = [torch.zeros(B, dtype=torch.int32, device="cuda") for _ in range(S)]
    d_first, d_len, d_gso = ([torch.zeros(B * max_bufs, dtype=torch.int32, device="cuda") for _ in range(S)]
                             for _ in range(3))
    L, h = dev.lib, dev.h

    def step(k, ns):
        i, q = k % R, k % ns
        rc = L.wgcs_coalesce_messages_batch(h, d_bufs[i].data_ptr(), stride, cap, None, d_lens.data_ptr(),
                                            d_nb.data_ptr(), max_bufs, B, 0, d_nm[q].data_ptr(), d_first[q].data_ptr(),
                                            d_len[q].data_ptr(), d_gso[q].data_ptr(), streams[q].cuda_stream)
        assert rc == 0

    elapsed, kern_ms, iso_ms = _time_steps(torch, streams, step, args.steps, args.warmup, barrier)
    nm = d_nm[0].cpu().numpy()
    assert (nm == 3).all(), nm[:4]
    runs = [SEGS, SEGS, max_bufs - 2 * SEGS]
    ml = d_len[0].view(B, max_bufs)[:, :3].cpu().numpy()
    assert (ml == np.array(runs) * MSG).all()
    for b in (0, B // 2, B - 1):  # the first buffer of run r holds packets f..f+n-1 back to back
        f = 0
        for n in runs:
            got = d_bufs[0][b * max_bufs + f, : n * MSG].cpu().numpy()
            assert np.array_equal(got, pk[b * max_bufs + f: b * max_bufs + f + n].reshape(-1)), (b, f)
            f += n
    moved = B * (max_bufs - 3) * MSG
    bps = 2 * moved
    flat = d_bufs[1].view(-1)  # disjoint regions of the (multi-GB) buffer: 4 x moved bytes, beyond the MALL
    copy_ms = _copy_ms(torch, stream, [flat[moved:], flat[3 * moved:]], [flat, flat[2 * moved:]], moved, args.steps)
    res = _result("device-resident UDP GSO coalesce GiB/s (bytes read + written), 1024 Send batches x 128 x 1452 B",
                  args, f"{B} Send batches of {max_bufs} x {MSG}-B transport messages to an IPv4 peer -> "
                  f"3 UDP_SEGMENT messages ({'/'.join(map(str, runs))} packets) each; coalesceMessages, "
                  "conn/bind.go:599-662, in place (SURVEY.md §8f row 3)",
                  {"batches": B, "packets_per_step": B * max_bufs, "moved_bytes": moved, "rotated_copies": R,
                   "slot_stride": stride},
                  "udp_coalesce_kernel<6,16>", kern_ms, bps, copy_ms, elapsed, iso_ms, S)
    if rank == 0 and args.cpu_seconds > 0:  # every N: north_star wants it in the same run
        res["cpu_baseline"] = coalesce_cpu_baseline(pk, args.cpu_seconds)
    return res


def coalesce_cpu_baseline(pk, seconds, B=16, max_bufs=128):
    """The oracle (C restatement of coalesceMessages) on B Send batches of the
    same shape: 1 thread for `seconds`, then every host thread (all_cores)."""
    import ctypes as C

    oracle = _oracle()
    L = oracle._conn_lib()
    L.or_coalesce_batch.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                    C.c_int, C.c_void_p]
    L.or_coalesce_batch.restype = None
    bps = 2 * B * (max_bufs - 3) * MSG

    def make_pass():
        bufs = np.zeros((B * max_bufs, 65536), np.uint8)
        bufs[:, :MSG] = pk[: B * max_bufs]
        lens = np.full(B * max_bufs, MSG, np.uint64)
        caps = np.full(B * max_bufs, 65535, np.uint64)
        nb = np.full(B, max_bufs, np.int32)
        nm = np.zeros(B, np.int32)

        def one():
            L.or_coalesce_batch(bufs.ctypes.data, 65536, lens.ctypes.data, caps.ctypes.data, nb.ctypes.data, max_bufs,
                                B, 0, nm.ctypes.data)
            assert (nm == 3).all()
        return one, bps

    rate, reps = _threaded_rate(make_pass, 1, seconds)
    threads = oracle.host_threads()
    arate, areps = _threaded_rate(make_pass, threads, seconds)
    return {"value": round(rate / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{reps} passes over {B} Send batches of the same shape, {seconds:.1f} s, "
                      "C restatement of coalesceMessages (bytes read + written)",
            "all_cores": {"value": round(arate / 2**30, 3), "unit": "GiB/s", "cores": threads,
                          "host_nproc": os.cpu_count(),
                          "sample": f"{areps} passes, one private copy of the {B} batches per thread"}}
