"""BASELINE.json configs[3] measurement: GSO split of 256 × 64-KiB TCP/IPv4
super-segments into 1500-B MSS segments with per-segment checksums, on one
MI355X (device-resident).  Called by bench.py --config cfg4.

Per super-packet: 65,535 bytes read (the virtio header's 10 bytes included),
45 segments written (44 × 1500 B + 1 × 1335 B; hdrLen 40, gsoSize 1460).
Algorithmic bytes per launch = bytes read + bytes written.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import time

import numpy as np

from . import shard, synth, traffic
from .tun import GSO_JOB_DTYPE

HBM_PEAK_GBS = 8000.0


def run(args, torch, dev, dist, rank, world, local, barrier):
    n_jobs, total, gso = 256, 65535, 1460
    # output slots per read: len(bufs) of the reference's Read = conn.BatchSize = 128
    # (/root/reference/device/send.go:239-245, tun/tun.go:870); --max-segs 64 for the round-2 line
    max_segs, stride, offset = getattr(args, "max_segs", 128), 1536, 16
    R = max(args.rotate, 8)  # (16.8 MB in + 25 MB out) per copy: rotate past the 256 MiB MALL
    pkts = [synth.make_super_packet(total, gso, seed=synth.SEED + 1000 * rank + k) for k in range(n_jobs)]
    jlen = len(pkts[0])
    in_align = getattr(args, "gso_in_align", 0) or 1
    jpitch = -(-jlen // in_align) * in_align
    arena = np.zeros(n_jobs * jpitch + 64, np.uint8)  # 64 B of slack past the last job
    for k, p in enumerate(pkts):
        arena[k * jpitch: k * jpitch + jlen] = np.frombuffer(p, np.uint8)
    jobs = np.zeros(n_jobs, GSO_JOB_DTYPE)
    jobs["off"] = np.arange(n_jobs, dtype=np.uint64) * np.uint64(jpitch)
    jobs["len"] = jlen
    out_align = getattr(args, "gso_out_align", 0)
    # slot base shift so that bufs[i][offset] lands on an out_align boundary (stride is a multiple of 128)
    oshift = (out_align - offset % out_align) % out_align if out_align else 0
    S = max(1, getattr(args, "streams", 1))
    streams = [torch.cuda.Stream() for _ in range(S)]
    R = max(R, 2 * S)
    d_arena = [torch.from_numpy(arena).cuda() for _ in range(R)]
    d_jobs = torch.from_numpy(jobs.view(np.uint8)).cuda()
    # slack past the slots covers the base shift (< out_align) as well as 256 B
    # (a fixed 256 B let an --gso-out-align above 256 cut the view short)
    d_out = [torch.empty(n_jobs * max_segs * stride + max(out_align, 256), dtype=torch.uint8, device="cuda")[oshift:]
             for _ in range(R)]
    assert all(d.numel() >= n_jobs * max_segs * stride for d in d_out)
    # per-stream result arrays: launches on different streams may overlap
    d_sizes = [torch.zeros(n_jobs * max_segs, dtype=torch.int32, device="cuda") for _ in range(S)]
    d_count = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(S)]
    d_status = [torch.zeros(n_jobs, dtype=torch.int32, device="cuda") for _ in range(S)]

    def step(k, ns=S):
        i, q = k % R, k % ns
        dev.gso_split_batch(d_arena[i], d_jobs, n_jobs, d_out[i], stride, offset, max_segs, d_sizes[q], d_count[q],
                            d_status[q], stream=streams[q])

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

    # The one-stream reference (untimed for `value`) runs first, as in bench.py
    # (measured after a two-stream burst, cfg2's launches read 2-3 us slower,
    # profiles/r2_probe_iso_order.txt).
    iso_ms = None
    if S > 1:
        timed(min(args.warmup, 5), 0, 1)
        iso_ms = timed(max(args.steps, 20), 0, 1)[1]
    if args.warmup > 0:  # the W warmup steps go through the same bracket as the timed ones
        timed(args.warmup, 0, S)
    torch.cuda.synchronize()
    count = d_count[0].cpu().numpy()
    status = d_status[0].cpu().numpy()
    assert (status == 0).all() and (count == 45).all(), (status[:4], count[:4])
    sizes = d_sizes[0].cpu().numpy().reshape(n_jobs, max_segs)
    bytes_out = int(sizes.astype(np.int64).sum())
    bytes_in = int(jobs["len"].astype(np.int64).sum())
    bytes_per_step = bytes_in + bytes_out
    elapsed, kern_ms = timed(args.steps, args.warmup, S)
    elapsed = shard.max_over_ranks(elapsed, dist)
    stream = streams[0]
    achieved = bytes_per_step / (kern_ms * 1e-3) / 1e9
    # the kernel and grid as the library was compiled (wgcs_gso_kernel_shape)
    nw, parts, uu, rows = (C.c_int(0) for _ in range(4))
    dev.lib.wgcs_gso_kernel_shape(C.byref(nw), C.byref(parts), C.byref(uu), C.byref(rows))
    if rows.value:  # the round-4 grid (WGCS_GSO_KERNEL=rows, A/B)
        kname = f"gso_rows_kernel<{uu.value},true>"
        grid = (f"({n_jobs}, {min((max_segs + 15) // 16, 3)}) blocks of 256: one block per (job, group lane), "
                "looping over segment groups")
    elif parts.value == 1:
        kname = f"gso_lds_kernel<{nw.value},{uu.value},true>"
        grid = (f"{n_jobs} blocks of {nw.value * 64}: one workgroup per read, staging it in LDS by LDS-DMA, "
                "16-lane rows stream its segments out")
    else:
        kname = f"gso_lds_kernel<{nw.value},{uu.value},true,{parts.value}>"
        grid = (f"{(n_jobs + 7) // 8 * 8 * parts.value} blocks of {nw.value * 64}: {parts.value} workgroups per read "
                f"(dealt to one XCD), each staging about 1/{parts.value} of the read in LDS by LDS-DMA, 16-lane rows "
                "stream its segments out")
    # calibration: a plain device-to-device copy of the super-packet bytes
    # (same read + write volume, same rotation) with the runtime's copy kernel
    with torch.cuda.stream(stream):
        for k in range(5):
            d_out[k % R][:bytes_in].copy_(d_arena[k % R][:bytes_in])
        c0 = torch.cuda.Event(enable_timing=True)
        c1 = torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        for k in range(args.steps):
            d_out[k % R][:bytes_in].copy_(d_arena[k % R][:bytes_in])
        c1.record(stream)
    torch.cuda.synchronize()
    copy_ms = c0.elapsed_time(c1) / args.steps
    result = {
        "metric": "device-resident GSO split GiB/s (bytes read + written), 256×64KiB TCP/IPv4 → 1500-B MSS",
        "value": round(bytes_per_step * args.steps * world / elapsed / 2**30, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": "256 x 65535-B TCP/IPv4 super-packets -> 45 x <=1500-B segments each (gsoSize 1460), "
                        "BASELINE.json configs[3]",
            "segments_per_step": int((count).sum()),
            "max_segs": max_segs,
            "bytes_in": bytes_in,
            "bytes_out": bytes_out,
            "rotated_copies": R,
            "out_align": out_align,
            "in_align": in_align,
            "streams": S,
            "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
            "parallelism": f"shard{world} (no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic.per_launch(kname, bytes_per_step),
            "kernel": kname,
            "grid": grid,
            "kernel_ms": round(kern_ms, 5),
            "kernel_ms_is": ("GPU time per launch over the timed region (HIP events on the launch streams)"
                             + (f"; {S} streams, consecutive launches overlap" if S > 1 else "")),
            "algorithmic_bytes_per_launch": bytes_per_step,
            "d2d_copy_same_bytes_ms": round(copy_ms, 5),
        },
    }
    if iso_ms is not None:
        result["roofline"]["kernel_ms_one_stream"] = round(iso_ms, 5)
        result["roofline"]["frac_one_stream"] = round(bytes_per_step / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if not getattr(args, "no_e2e", False):
        result["end_to_end"] = end_to_end(dev, pkts, bytes_in, bytes_out, steps=max(10, min(args.steps, 40)))
        result["host_call"] = host_call(dev, pkts[0], with_cpu=rank == 0 and world == 1 and args.cpu_seconds > 0)
    if rank == 0 and args.cpu_seconds > 0:  # every N: north_star wants it in the same run
        result["cpu_baseline"] = cpu_baseline(pkts, args.cpu_seconds, bytes_per_step)
    if rank == 0:
        print(json.dumps(result), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def end_to_end(dev, pkts, bytes_in, bytes_out, steps: int, depth: int = 3):
    """Host-memory-in / host-memory-out rate through the Tun.Read stager
    (wgcs_stager_*): per batch, the 256 reads are copied into the pinned ring
    slot (standing in for read(2) into tun.readBuf), then H2D -> split -> D2H
    of the packed segments on the slot's stream; `depth` batches in flight."""
    from .tun import Stager

    arrs = [np.frombuffer(p, np.uint8) for p in pkts]
    st = Stager(dev, depth=depth, max_reads=len(arrs), max_bytes=sum(len(a) + 16 for a in arrs), max_segs=64,
                seg_room=1536 - 16)
    inflight = []
    push_t = [0.0]

    def one():
        t = time.perf_counter()
        st.push_many(arrs)
        push_t[0] += time.perf_counter() - t
        if len(inflight) == depth - 1:  # the next submit recycles the oldest slot: consume it first
            b = inflight.pop(0)
            st.wait(b)
            n, err, _ = st.result(b, len(arrs) - 1)
            assert err is None and n == 45
        inflight.append(st.submit())

    for _ in range(depth + 2):
        one()
    push_t[0] = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    while inflight:
        st.wait(inflight.pop(0))
    dt = (time.perf_counter() - t0) / steps
    st.close()
    return {"value": round((bytes_in + bytes_out) / dt / 2**30, 2), "unit": "GiB/s",
            "ms_per_batch": round(dt * 1e3, 4), "bytes_in_plus_out": bytes_in + bytes_out,
            "host_push_ms_per_batch": round(push_t[0] / steps * 1e3, 4),
            "what": f"Tun.Read stager, depth {depth}: host memcpy of the reads into pinned staging + H2D + "
                    "split kernel + D2H of the packed segments (PCIe-inclusive)"}


def host_call(dev, vp: bytes, with_cpu: bool, reps: int = 200):
    """Latency of one reference-shaped call, wgcs_handle_virtio_read on one
    65,535-B read (Tun.Read granularity, host buffers in and out), as one C
    call with prebuilt arguments; the oracle's time for the same call beside it."""
    import ctypes as C

    nb = 64
    bufs = [np.zeros(1536, np.uint8) for _ in range(nb)]
    u8p = C.POINTER(C.c_uint8)
    arr = (u8p * nb)(*[C.cast(b.ctypes.data, u8p) for b in bufs])
    lens = (C.c_size_t * nb)(*([1536] * nb))
    sizes = (C.c_int * nb)()
    n = C.c_int(0)
    src = np.frombuffer(vp, np.uint8)
    rb = src.copy()

    def timed(fn):
        ts = []
        for _ in range(reps):
            rb[:] = src  # handleVirtioRead edits readBuf in place: restore outside the timed call
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    L, h = dev.lib, dev.h
    gpu = timed(lambda: L.wgcs_handle_virtio_read(h, rb.ctypes.data, len(rb), arr, lens, nb, sizes, 16, C.byref(n)))
    assert n.value == 45
    out = {"call": "wgcs_handle_virtio_read, one 65,535-B TSO read -> 45 segments, host buffers",
           "median_us": round(gpu * 1e6, 1)}
    if with_cpu:
        import os
        import sys

        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
        import oracle  # cpu_baseline leg only

        OL = oracle.lib()
        cpu = timed(lambda: OL.or_handle_virtio_read(rb.ctypes.data, len(rb), arr, lens, nb, sizes, 16, C.byref(n)))
        out["cpu_oracle_median_us"] = round(cpu * 1e6, 1)
    return out


def cpu_baseline(pkts, seconds, bytes_per_step):
    """The oracle's handleVirtioRead (C restatement of tun/tun.go:514-632 +
    gsoSplit) over the same 256 reads: one core for `seconds`, then all host
    cores (pthreads, wg_oracle_bench.c) for a quarter of that."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle  # cpu_baseline leg only

    per_read = bytes_per_step / len(pkts)
    rate1, calls1 = oracle.gso_bench_mt(pkts, 64, 1536, 16, 1, seconds)
    threads = oracle.host_threads()
    rate_mt, calls_mt = oracle.gso_bench_mt(pkts, 64, 1536, 16, threads, max(seconds / 4, 1.0))
    return {"value": round(per_read * rate1 / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{calls1} handleVirtioRead calls over the 256 super-packets in {seconds:.0f} s, C restatement "
                      "of tun/tun.go:514-632 + gsoSplit, 1 thread, calls timed (not the readBuf refills)",
            "all_cores": {"value": round(per_read * rate_mt / 2**30, 3), "unit": "GiB/s", "cores": threads,
                          "host_nproc": os.cpu_count(),
                          "sample": f"{calls_mt} calls on {threads} pthreads, each on private copies"}}
