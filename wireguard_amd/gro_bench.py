"""Tun.Write measurement: handleGRO
(tun/gro.go:1326-1367) over one device.RoutineSendToInternet batch of 128
packets from host buffers, the reference's Write granularity (conn/conn.go:12-15).
Called by bench.py --config gro.

Batch: 4 TCP/IPv4 flows x 32 in-order 1448-B MSS segments (1488-B packets), the
common bulk-transfer case; every segment coalesces into 4 packets of 32 x 1448 B.
One step = one wgcs_handle_gro C call (argument arrays prebuilt): stage into
pinned memory, H2D, the VALIDATE checksum kernel, the host flow planner, the
coalesce kernel, D2H and the copy back into the Go-slice buffers.
Unit: packets/s (higher is better).
"""
from __future__ import annotations

import json
import time

import numpy as np

from . import shard, synth, traffic

OFFSET = 16
CAP = 65535 + OFFSET
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, MI355X_MICROARCH.md


def flow_segments(dev, n_pkts: int, mss: int = 1448, seed: int = synth.SEED, tcp_flags: int = 0x10):
    """n_pkts in-order TCP/IPv4 segments of ONE flow (any count: the flow is cut
    into super-packets of at most 45 segments that share the IP/TCP header and
    continue its sequence numbers), each made by the product's GSO split."""
    out, seq_step, first = [], 0, None
    while len(out) < n_pkts:
        k = min(45, n_pkts - len(out))
        vp = bytearray(synth.make_super_packet(40 + k * mss, mss, seed=seed + 7919 * len(out), tcp_flags=tcp_flags))
        if first is None:
            first = bytes(vp[10:50])
        else:  # the flow's header, sequence number continued
            vp[10:50] = first
            vp[12:14] = (40 + k * mss).to_bytes(2, "big")
            seq = (int.from_bytes(first[24:28], "big") + seq_step) & 0xFFFFFFFF
            vp[34:38] = seq.to_bytes(4, "big")
        bufs = [np.zeros(mss + 200, np.uint8) for _ in range(k + 2)]
        sizes = [0] * len(bufs)
        n, err = dev.handle_virtio_read(np.frombuffer(vp, np.uint8).copy(), bufs, sizes, OFFSET)
        assert err is None and n == k, (n, err)
        out += [bufs[i][OFFSET: OFFSET + sizes[i]].tobytes() for i in range(n)]
        seq_step += k * mss
    return out


def udp_flow_segments(dev, n_pkts: int, mss: int = 1448, seed: int = synth.SEED):
    """n_pkts UDP/IPv4 datagrams of ONE flow (UDP GSO super-packets of at most
    45 segments sharing the IP/UDP header), each made by the product's GSO split."""
    out, first = [], None
    while len(out) < n_pkts:
        k = min(45, n_pkts - len(out))
        vp = bytearray(synth.make_super_packet(28 + k * mss, mss, seed=seed + 7919 * len(out), udp=True))
        if first is None:
            first = bytes(vp[10:38])
        else:  # the flow's header, lengths for this super-packet
            vp[10:38] = first
            vp[12:14] = (28 + k * mss).to_bytes(2, "big")
            vp[34:36] = (8 + k * mss).to_bytes(2, "big")
        bufs = [np.zeros(mss + 200, np.uint8) for _ in range(k + 2)]
        sizes = [0] * len(bufs)
        n, err = dev.handle_virtio_read(np.frombuffer(vp, np.uint8).copy(), bufs, sizes, OFFSET)
        assert err is None and n == k, (n, err)
        out += [bufs[i][OFFSET: OFFSET + sizes[i]].tobytes() for i in range(n)]
    return out


def make_batch(dev, flows: int = 4, per_flow: int = 32, mss: int = 1448, seed: int = synth.SEED):
    """128 segmented TCP/IPv4 packets, produced by the product's GSO split of
    one super-packet per flow (flows interleaved round-robin, in order per flow)."""
    segs = [flow_segments(dev, per_flow, mss, seed + f) for f in range(flows)]
    return [segs[f][k] for k in range(per_flow) for f in range(flows)]


# Write-call shapes of the gro_device bench (the per-flow walk is
# one thread per flow, so one long flow or prepend chains are its worst case).
CALL_SHAPES = {
    "4x32": "4 TCP/IPv4 flows x 32 in-order 1448-B MSS segments, interleaved (bulk transfer)",
    "1x128": "one TCP/IPv4 flow of 128 in-order 1448-B segments (one walker does all 128 steps)",
    "4x32rev": "4 flows x 32 segments, each flow in reverse order: every packet prepends to its item (gro.go:648-697)",
    "1x128rev": "one flow of 128 segments in reverse order (a 128-step prepend chain)",
    "shuffled": "4 flows x 32 segments in a seeded random order (appends, prepends and new items mixed)",
    "4x32udp": "4 UDP/IPv4 flows x 32 1448-B datagrams, interleaved (UDP GRO: every datagram appends)",
    "1x128udp": "one UDP/IPv4 flow of 128 1448-B datagrams",
    "16x8": "16 TCP/IPv4 flows x 8 in-order segments, interleaved (many short flows)",
    "32x4": "32 TCP/IPv4 flows x 4 in-order segments, interleaved",
}


def shape_batch(dev, shape: str):
    if shape == "4x32":
        return make_batch(dev)
    if shape in ("1x128", "1x128rev"):
        f = flow_segments(dev, 128)
        return f[::-1] if shape.endswith("rev") else f
    if shape == "4x32rev":
        segs = [flow_segments(dev, 32, seed=synth.SEED + f)[::-1] for f in range(4)]
        return [segs[f][k] for k in range(32) for f in range(4)]
    if shape in ("16x8", "32x4"):
        f, k = (int(x) for x in shape.split("x"))
        return make_batch(dev, flows=f, per_flow=k)
    if shape == "4x32udp":
        segs = [udp_flow_segments(dev, 32, seed=synth.SEED + f) for f in range(4)]
        return [segs[f][k] for k in range(32) for f in range(4)]
    if shape == "1x128udp":
        return udp_flow_segments(dev, 128)
    if shape == "shuffled":
        pk = make_batch(dev)
        order = np.random.default_rng(synth.SEED).permutation(len(pk))
        return [pk[i] for i in order]
    raise ValueError(shape)


class Batch:
    """The 128 packets as Go-slice style buffers (cap CAP, len OFFSET+len(p))
    inside one arena, with the C argument arrays prebuilt, so a timed step is
    exactly one C call; reset() restores bytes, pointers and lengths."""

    def __init__(self, pkts, arena=None):
        import ctypes as C

        self.C = C
        n = len(pkts)
        self.n = n
        self.arena = np.zeros((n, CAP), np.uint8) if arena is None else arena.reshape(n, CAP)
        self.orig = np.zeros((n, OFFSET + max(len(p) for p in pkts) + 16), np.uint8)
        for i, p in enumerate(pkts):
            self.orig[i, OFFSET: OFFSET + len(p)] = np.frombuffer(p, np.uint8)
        u8p = C.POINTER(C.c_uint8)
        self.ptrs0 = (u8p * n)(*[C.cast(self.arena[i].ctypes.data, u8p) for i in range(n)])
        self.ptrs = (u8p * n)()
        self.lens0 = (C.c_size_t * n)(*[OFFSET + len(p) for p in pkts])
        self.lens = (C.c_size_t * n)()
        self.caps = (C.c_size_t * n)(*([CAP] * n))
        self.tw = (C.c_int * n)()
        self.ntw = C.c_int(0)
        self.width = self.orig.shape[1]

    def reset(self):
        C = self.C
        self.arena[:, : self.width] = self.orig
        C.memmove(self.ptrs, self.ptrs0, C.sizeof(self.ptrs0))
        C.memmove(self.lens, self.lens0, C.sizeof(self.lens0))


def run(args, torch, dev, dist, rank, world, local, barrier):
    pkts = make_batch(dev)
    n = len(pkts)
    payload = sum(len(p) for p in pkts)
    b = Batch(pkts)
    L, h = dev.lib, dev.h

    def call():
        return L.wgcs_handle_gro(h, b.ptrs, b.lens, b.caps, b.n, OFFSET, 1, b.tw, b.C.byref(b.ntw))

    for _ in range(args.warmup):
        b.reset()
        assert call() == 0 and b.ntw.value == 4, b.ntw.value
    barrier()
    t_total = 0.0
    for _ in range(args.steps):
        b.reset()  # Write gets fresh bufs: restored outside the timed call
        t0 = time.perf_counter()
        call()
        t_total += time.perf_counter() - t0
    barrier()
    t_total = shard.max_over_ranks(t_total, dist)
    per = t_total / args.steps
    result = {
        "metric": "Tun.Write handleGRO packets/s (host buffers, 128-packet batch)",
        "value": round(n * world / per, 1),
        "unit": "packets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(per * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": "128 TCP/IPv4 packets (4 flows x 32 x 1448-B MSS) per wgcs_handle_gro call, "
                        "coalesced to 4 packets; host buffers in and out",
            "packets_per_step": n,
            "payload_bytes": payload,
            "parallelism": f"replica{world} (one context per GPU, no collective)",
            "gib_per_s": round(payload / per / 2**30, 3),
        },
    }
    if rank == 0 and args.cpu_seconds > 0:  # every N: north_star wants it in the same run
        result["cpu_baseline"] = cpu_baseline(pkts, min(args.cpu_seconds, 5.0))
    if rank == 0:
        print(json.dumps(result), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def run_staged(args, torch, dev, dist, rank, world, local, barrier, calls_per_slot: int = 64, depth: int = 3):
    """bench.py --config gro_staged: the Tun.Write stager (wgcs_wstager_*).
    One step = one ring slot of `calls_per_slot` Write calls (128 packets
    each, the batch above): push (pinned staging, no host planning), submit
    (H2D, scatter into Go-sized slices, ONE device handleGRO launch over every
    call, gather of the write(2) images, D2H), and -- depth-1 slots later
    -- wait + per-call results (the write(2) images).  Host buffers in, host
    buffers out: PCIe-inclusive packets/s."""
    import ctypes as C
    import os

    from .tun import WriteStager

    L = dev.lib
    calls_per_slot = int(os.environ.get("WGCS_WS_CALLS", calls_per_slot))
    depth = int(os.environ.get("WGCS_WS_DEPTH", depth))
    # zero-copy: the Write buffers live in pinned host memory (wgcs_host_alloc)
    # and the slot's scatter kernel reads them over PCIe (wgcs_wstager_push_pinned)
    pinned = bool(getattr(args, "pinned", False)) or os.environ.get("WGCS_WS_PINNED", "0") == "1"
    pkts = make_batch(dev)
    n = len(pkts)
    # Every Write call of the timed region gets its own buffers (distinct host
    # addresses, so neither the CPU caches nor the GPU's see a packet twice):
    # R sets of calls_per_slot x 128 buffers, 2 KiB apart, >= 512 MiB in all,
    # rotated so a set is reused only after its slot has been settled.  Each
    # buffer is declared with the Go pool's capacity (CAP); only
    # bufs[i][offset-10:len] is ever read.
    SB = 2048
    per_set = calls_per_slot * n
    R = max(depth + 1, -(-(512 << 20) // (per_set * SB)))
    nbytes = R * per_set * SB
    b_pool = dev.host_alloc(nbytes) if pinned else None
    mem = b_pool if pinned else np.empty(nbytes, np.uint8)
    img = np.zeros((n, SB), np.uint8)
    for i, p in enumerate(pkts):
        img[i, OFFSET: OFFSET + len(p)] = np.frombuffer(p, np.uint8)
    mem.reshape(R * calls_per_slot, n, SB)[:] = img
    base = mem.ctypes.data
    call_ptrs = [(C.c_void_p * n)(*[base + ((r * calls_per_slot + c) * n + i) * SB for i in range(n)])
                 for r in range(R) for c in range(calls_per_slot)]
    lens0 = (C.c_size_t * n)(*[OFFSET + len(p) for p in pkts])
    caps = (C.c_size_t * n)(*([CAP] * n))
    push_fn = L.wgcs_wstager_push_pinned if pinned else L.wgcs_wstager_push
    ws = WriteStager(dev, depth=depth, max_writes=calls_per_slot, max_pkts=calls_per_slot * n,
                     max_bytes=calls_per_slot * sum(len(p) + 32 for p in pkts))
    nstep = [0]
    st, nw = C.c_int(0), C.c_int(0)
    tw = (C.c_int * n)()
    outp = (C.c_void_p * n)()
    outl = (C.c_size_t * n)()
    bt = C.c_uint64(0)
    inflight = []

    def settle(batch):
        assert L.wgcs_wstager_wait(ws.h, batch) == 0
        for k in range(calls_per_slot):
            L.wgcs_wstager_result(ws.h, batch, k, C.byref(st), C.byref(nw), tw, outp, outl)
            assert st.value == 0 and nw.value == 4, (st.value, nw.value)

    # Write calls arrive from many goroutines (one RoutineSendToInternet per
    # peer): `threads` host threads push concurrently (ctypes releases the GIL;
    # the stager copies outside its lock)
    import concurrent.futures as cf

    threads = max(1, int(getattr(args, "push_threads", 0) or os.environ.get("WGCS_PUSH_THREADS", 4)))
    pool = cf.ThreadPoolExecutor(threads) if threads > 1 else None
    share = [calls_per_slot // threads + (1 if t < calls_per_slot % threads else 0) for t in range(threads)]

    def pusher(c0, k):
        i = C.c_int(0)
        for c in range(c0, c0 + k):
            assert push_fn(ws.h, call_ptrs[c], lens0, caps, n, OFFSET, 1, C.byref(i)) == 0

    phase = [0.0, 0.0, 0.0]  # push, wait + results, submit (host seconds)

    def step():
        t0 = time.perf_counter()
        c0 = (nstep[0] % R) * calls_per_slot
        nstep[0] += 1
        if pool is None:
            pusher(c0, calls_per_slot)
        else:
            starts = [c0 + sum(share[:t]) for t in range(threads)]
            for f in [pool.submit(pusher, a, k) for a, k in zip(starts, share)]:
                f.result()
        t1 = time.perf_counter()
        if len(inflight) == depth - 1:
            settle(inflight.pop(0))
        t2 = time.perf_counter()
        assert L.wgcs_wstager_submit(ws.h, C.byref(bt)) == 0
        inflight.append(bt.value)
        t3 = time.perf_counter()
        phase[0] += t1 - t0
        phase[1] += t2 - t1
        phase[2] += t3 - t2

    for _ in range(max(args.warmup, depth + 1)):
        step()
    barrier()
    phase[:] = [0.0, 0.0, 0.0]
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    while inflight:
        settle(inflight.pop(0))
    dt = time.perf_counter() - t0
    barrier()
    dt = shard.max_over_ranks(dt, dist)
    per = dt / args.steps
    ws.close()
    if pool is not None:
        pool.shutdown()
    if b_pool is not None:
        dev.host_free(b_pool)
    # the written images are correct: one slot checked against the oracle in tests/test_gpu_wstager.py
    result = {
        "metric": "Tun.Write handleGRO packets/s through the write stager (host buffers in, write(2) images out)",
        "value": round(calls_per_slot * n * world / per, 1),
        "unit": "packets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(per * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": f"{calls_per_slot} Tun.Write calls of 128 TCP/IPv4 packets (4 flows x 32 x 1448-B MSS) per "
                        f"ring slot, depth {depth}; each call coalesced to 4 super-packets"
                        + f"; every call its own buffers ({R} rotated sets, {nbytes >> 20} MiB)"
                        + ("; buffers in pinned host memory, read by the GPU (zero-copy push)" if pinned else ""),
            "packets_per_step": calls_per_slot * n,
            "payload_bytes_per_step": calls_per_slot * sum(len(p) for p in pkts),
            "push_threads": threads,
            "zero_copy": pinned,
            "host_ms_per_step": {"push": round(phase[0] / args.steps * 1e3, 4),
                                 "wait_and_results": round(phase[1] / args.steps * 1e3, 4),
                                 "submit": round(phase[2] / args.steps * 1e3, 4)},
            "parallelism": f"replica{world} (one stager per GPU, no collective)",
            "gib_per_s": round(calls_per_slot * sum(len(p) for p in pkts) / per / 2**30, 3),
        },
    }
    if rank == 0 and args.cpu_seconds > 0:  # every N: north_star wants it in the same run
        result["cpu_baseline"] = cpu_baseline(pkts, min(args.cpu_seconds, 5.0))
    if rank == 0:
        print(json.dumps(result), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(pkts, seconds):
    """The oracle's handleGRO (C restatement of tun/gro.go) on the same
    128-packet batch: one core, then all host cores (pthreads,
    wg_oracle_bench.c); only the calls are timed (not the batch refills)."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle  # cpu_baseline leg only

    rate1, calls1 = oracle.gro_bench_mt(pkts, OFFSET, True, 1, seconds)
    threads = oracle.host_threads()
    rate_mt, calls_mt = oracle.gro_bench_mt(pkts, OFFSET, True, threads, max(seconds / 2, 1.0))
    return {"value": round(len(pkts) * rate1, 1), "unit": "packets/s", "cores": 1, "kind": "port",
            "sample": f"{calls1} handleGRO calls on the same {len(pkts)}-packet batch in {seconds:.0f} s, "
                      "C restatement of tun/gro.go, calls timed (not the refills)",
            "all_cores": {"value": round(len(pkts) * rate_mt, 1), "unit": "packets/s", "cores": threads,
                          "host_nproc": os.cpu_count(),
                          "sample": f"{calls_mt} calls on {threads} pthreads, each on a private copy of the batch"}}


def run_device(args, torch, dev, dist, rank, world, local, barrier, calls: int = 1792, rotate: int = 4):
    """bench.py --config gro_device: the device-resident batch of Tun.Write
    calls (wgcs_handle_gro_batch).  One step = one launch over `calls` calls
    of the 128-packet batch above, every buffer a Go-sized slice (cap 65,551 B)
    in HBM, handleGRO in place.  The packets must be pristine for every step
    (handleGRO rewrites headers), so the bench keeps `rotate` copies and
    restores them between bursts of `rotate` launches, outside the timed
    region; the timed region is the launches, bracketed by a device sync."""
    import os

    from .tun import GRO_BUF_DTYPE, GRO_CALL_DTYPE, GRO_CAN_UDP

    calls = int(os.environ.get("WGCS_GRO_CALLS", calls))
    shape = getattr(args, "gro_shape", "4x32")
    pkts = shape_batch(dev, shape)
    n = len(pkts)
    N = calls * n
    # Buffer k at shift + k * stride.  --gro-buf-align A (default 128): stride
    # a multiple of A and the arena shifted so that every bufs[k][offset]
    # starts on an A-byte line, as cfg4 places its slots (the reference's bufs
    # are separate Go allocations at whatever address; here the device batch's
    # layout is ours to choose).  0: back to back at 16-byte multiples.
    align = int(getattr(args, "gro_buf_align", 0) or 16)
    stride = int(os.environ.get("WGCS_GRO_STRIDE", (CAP + align - 1) // align * align))
    shift = (align - OFFSET % align) % align
    W = (OFFSET + max(len(p) for p in pkts) + 31) // 16 * 16  # bytes restored per buffer
    img = np.zeros((n, W), np.uint8)
    for i, p in enumerate(pkts):
        img[i, OFFSET: OFFSET + len(p)] = np.frombuffer(p, np.uint8)
    d_img = torch.from_numpy(np.tile(img, (calls, 1))).cuda()
    # rotated copies (each launch's packets alone exceed the 256 MiB MALL), at
    # most ~64 GiB of slices in all, at least 2 (consecutive launches overlap)
    R = max(2, min(rotate, (64 << 30) // (N * stride)))
    arenas = [torch.empty(N * stride + shift, dtype=torch.uint8, device="cuda") for _ in range(R)]
    gb = np.zeros(N, GRO_BUF_DTYPE)
    gb["off"] = np.arange(N, dtype=np.uint64) * np.uint64(stride) + np.uint64(shift)
    gb["len"] = np.tile(np.array([OFFSET + len(p) for p in pkts], np.uint32), calls)
    gb["cap"] = CAP
    d_bufs0 = torch.from_numpy(gb.view(np.uint8)).cuda()
    d_bufs = [d_bufs0.clone() for _ in range(R)]
    gc = np.zeros(calls, GRO_CALL_DTYPE)
    gc["first"] = np.arange(calls, dtype=np.uint32) * n
    gc["n"] = n
    gc["offset"] = OFFSET
    gc["flags"] = GRO_CAN_UDP
    d_calls = torch.from_numpy(gc.view(np.uint8)).cuda()
    st = [torch.zeros(calls, dtype=torch.int32, device="cuda") for _ in range(R)]
    nw = [torch.zeros(calls, dtype=torch.int32, device="cuda") for _ in range(R)]
    tw = [torch.zeros(N, dtype=torch.int32, device="cuda") for _ in range(R)]
    S = max(1, getattr(args, "streams", 1))  # consecutive launches (independent batches) round-robin
    streams = [torch.cuda.Stream() for _ in range(S)]
    stream = streams[0]

    def restore():
        for r in range(R):
            arenas[r][shift: shift + N * stride].view(N, stride)[:, :W].copy_(d_img)
            d_bufs[r].copy_(d_bufs0)
        torch.cuda.synchronize()

    def launch(r):
        dev.handle_gro_batch(arenas[r], d_bufs[r], d_calls, calls, st[r], nw[r], tw[r], stream=streams[r % S])

    restore()
    launch(0)
    torch.cuda.synchronize()
    # every call is the same batch: the same status and write count everywhere
    # (the per-byte parity of each shape is tests/test_gpu_gro_batch.py's)
    assert bool((st[0] == 0).all()) and bool((nw[0] == nw[0][0]).all()), (st[0][:4], nw[0][:4])
    n_write = int(nw[0][0].item())
    # bytes the reference's appends and prepend copies move (gro.go:648-697):
    # every copy grows len(bufs[j]) of its destination, and lengths only grow,
    # so the copied volume is the growth of all slice lengths (a prepend chain
    # copies its whole item at every step: quadratic in the chain length)
    lens0 = d_bufs0.cpu().numpy().view(GRO_BUF_DTYPE)["len"].astype(np.int64)
    lens1 = d_bufs[0].cpu().numpy().view(GRO_BUF_DTYPE)["len"].astype(np.int64)
    copied = int(lens1.sum() - lens0.sum())
    if shape == "4x32":
        heads = d_bufs[0].cpu().numpy().view(GRO_BUF_DTYPE)["len"].reshape(calls, n)[:, :4]
        assert n_write == 4 and (heads == OFFSET + 40 + 32 * 1448).all(), heads[0]
    for _ in range(max(0, args.warmup - 1)):
        restore()
        for r in range(R):
            launch(r)
        torch.cuda.synchronize()
    barrier()
    t_total, ev_ms, done = 0.0, 0.0, 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    while done < args.steps:
        k = min(R, args.steps - done)
        restore()  # fresh Write batches: not timed
        t0 = time.perf_counter()
        e0.record(stream)
        for q in streams[1:]:
            q.wait_event(e0)
        for r in range(k):
            launch(r)
        for q in streams[1:]:
            j = torch.cuda.Event()
            j.record(q)
            stream.wait_event(j)
        e1.record(stream)
        torch.cuda.synchronize()
        t_total += time.perf_counter() - t0
        ev_ms += e0.elapsed_time(e1)
        done += k
    barrier()
    t_total = shard.max_over_ranks(t_total, dist)
    per = t_total / args.steps
    kern_ms = ev_ms / args.steps
    payload = sum(len(p) for p in pkts) * calls
    # algorithmic bytes per launch: every candidate byte read once (checksumValid),
    # every appended payload read and written once, the rewritten headers
    # every copied byte read and written once (`copied`, above)
    algo = payload + 2 * copied + n_write * calls * (10 + 40)
    achieved = algo / (kern_ms * 1e-3) / 1e9
    result = {
        "metric": "device-resident Tun.Write handleGRO packets/s (batch of Write calls in HBM)",
        "value": round(N * world / per, 1),
        "unit": "packets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(per * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": f"{calls} Tun.Write calls per launch, each 128 packets: {CALL_SHAPES[shape]}; coalesced to "
                        f"{n_write} packets, buffers of cap 65,551 B in HBM, in place",
            "call_shape": shape,
            "writes_per_call": n_write,
            "packets_per_step": N,
            "payload_bytes_per_step": payload,
            "rotated_copies": R,
            "streams": S,
            "buffer_stride": stride,
            "buf_align": align,
            "parallelism": f"replica{world} (one batch per GPU, no collective)",
            "gib_per_s": round(payload / per / 2**30, 3),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic.per_launch("gro_batch_kernel", algo),
            "kernel": "gro_batch_kernel",
            "kernel_ms": round(kern_ms, 5),
            "kernel_ms_is": "GPU time per launch (HIP events around each burst of launches"
                            + (f"; {S} streams, consecutive launches overlap)" if S > 1 else ")"),
            "algorithmic_bytes_per_launch": algo,
            "copied_bytes_per_launch": copied,
            "note": "algorithmic bytes: every candidate byte read once (checksumValid) + every byte the "
                    "reference's append / prepend copies move, read and written (the growth of all slice "
                    "lengths) + the rewritten headers; one thread per flow runs handleGRO's flow-table walk",
        },
    }
    if rank == 0 and args.cpu_seconds > 0:  # every N: north_star wants it in the same run
        result["cpu_baseline"] = cpu_baseline(pkts, min(args.cpu_seconds, 5.0))
    if rank == 0:
        print(json.dumps(result), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()
