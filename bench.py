#!/usr/bin/env python3
"""bench.py -- device-resident Internet-checksum throughput on MI355X.

Metric (BASELINE.json): "device-resident payload GiB/s, Internet checksum,
64k×1500B batch".  One step = one pass of the hot path (one kernel launch of
WGCS_MODE_VALIDATE = checksumValid, /root/reference/tun/gro.go:554-612) over
one batch of 65,536 × 1500-B TCP/IPv4 frames already resident in HBM.  Payload
bytes = sum of frame lengths (every byte of a frame is read: addresses for the
pseudo-header, the L4 header and the payload).

Contract: `python bench.py --gpus N --steps K --warmup W`; for N>1 it is run
under torch.distributed.run, one rank per GPU.  Each rank checksums its own
batch (weak scaling, no data-path collective -- per-packet checksums are
independent).  The timed region is bracketed by a barrier +
device sync on both sides; the max time over ranks is used; rank 0 prints ONE
JSON line.

Infinity Cache: a 98.3 MB batch fits the 256 MiB MALL, so the bench rotates
over R distinct copies (default 4 = 393 MB) so every launch reads HBM.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md

CONFIGS = {
    # name: (n_packets, frame_len, kinds, BASELINE.json configs index)
    "cfg2": (65536, 1500, "tcp4", 1),
    "cfg3": (65536, 9000, "tcp4", 2),
    "cfg5": (131072, 1500, "mixed", 4),  # per-GPU shard of 1,048,576 mixed frames at 8 GPUs
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS) + ["cfg4"])
    ap.add_argument("--mode", default="validate", choices=["validate", "fill"])
    ap.add_argument("--rotate", type=int, default=4, help="distinct batch copies (defeat the 256 MiB MALL)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-event-timing", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check the GPU results against the synth ground truth")
    return ap.parse_args()


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(0)

    def barrier():
        if dist is not None:
            dist.barrier()

    from wireguard_amd import synth
    from wireguard_amd.tun import Device, MODE_VALIDATE, MODE_L4_FILL

    dev = Device(local if world > 1 else 0)
    if args.config == "cfg4":
        from wireguard_amd import gso_bench

        return gso_bench.run(args, torch, dev, dist, rank, world, local, barrier)

    n, flen, kinds, cfg_idx = CONFIGS[args.config]
    mode = MODE_VALIDATE if args.mode == "validate" else MODE_L4_FILL
    # each rank gets its own seeded shard (weak scaling)
    arena_np, pkts_np, _ = synth.make_batch(n, flen, kinds=kinds, seed=synth.SEED + rank)
    bytes_per_step = int(pkts_np["len"].astype(np.int64).sum())
    stream = torch.cuda.Stream()  # dedicated stream: kernel launches and events share it
    arenas = [torch.from_numpy(arena_np).to("cuda") for _ in range(args.rotate)]
    pkts = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
    outs = [torch.empty(n, dtype=torch.uint8 if mode == MODE_VALIDATE else torch.int16, device="cuda")
            for _ in range(args.rotate)]
    torch.cuda.synchronize()

    def step(k):
        i = k % args.rotate
        dev.checksum_batch(mode, arenas[i], pkts, n, outs[i], stream=stream)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    if args.verify:
        if mode == MODE_VALIDATE:
            assert bool(outs[0].all().item()), "VALIDATE: synthetic frames must all be valid"
        else:
            # L4 fill of a valid frame reproduces the stored checksum field
            got = outs[0].cpu().numpy().view(np.uint16)
            a = arena_np[: n * flen].reshape(n, flen)
            cs = pkts_np["csum_start"].astype(np.int64) + pkts_np["csum_offset"]
            want = (a[np.arange(n), cs].astype(np.uint16) << 8) | a[np.arange(n), cs + 1]
            assert np.array_equal(got, want), "L4_FILL mismatch vs stored checksums"

    # HIP events on the launch stream bracket the timed region (one pair: an
    # event between launches would add a ~10 µs gap per step); launches are
    # back-to-back on one stream, so elapsed / steps = the average launch
    # duration rocprofv3 reports for the kernel (profiles/).
    use_events = not args.no_event_timing
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if use_events:
        e0.record(stream)
    for k in range(args.steps):
        step(args.warmup + k)
    if use_events:
        e1.record(stream)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = e0.elapsed_time(e1) / args.steps if use_events else None
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # timing only, not on the data path
        elapsed = float(t.item())

    total_bytes = bytes_per_step * args.steps * world
    value = total_bytes / elapsed / 2**30
    result = {
        "metric": "device-resident payload GiB/s, Internet checksum, 64k×1500B batch",
        "value": round(value, 2),
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
            "workload": f"{n} x {flen}-B {kinds} frames per GPU, {args.mode} (checksumValid) per step, "
                        f"BASELINE.json configs[{cfg_idx}]",
            "packets_per_gpu": n,
            "frame_len": flen,
            "global_batch_bytes": bytes_per_step * world,
            "mode": args.mode,
            "rotated_copies": args.rotate,
            "parallelism": f"shard{world} (no collective)",
        },
    }
    if kern_ms is not None:
        achieved = bytes_per_step / (kern_ms * 1e-3) / 1e9
        result["roofline"] = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": "checksum_batch_kernel<VALIDATE>" if mode == MODE_VALIDATE else "checksum_batch_kernel<L4_FILL>",
            "kernel_ms": round(kern_ms, 5),
            "algorithmic_bytes_per_launch": bytes_per_step,
        }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(arena_np, pkts_np, mode, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(arena_np, pkts_np, mode, seconds):
    """The oracle (C restatement of tun/checksum.go, 1 thread) on the same batch,
    repeated until `seconds` of CPU time have elapsed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg: allowed use of the oracle

    nbytes = int(pkts_np["len"].astype(np.int64).sum())
    oracle.checksum_batch_mt(mode, arena_np, pkts_np, 1)  # warm
    reps = 0
    t0 = time.perf_counter()
    while True:
        oracle.checksum_batch_mt(mode, arena_np, pkts_np, 1)
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {
        "value": round(nbytes * reps / dt / 2**30, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{reps} passes over the same {len(pkts_np)}-frame batch ({nbytes/1e6:.1f} MB), "
                  f"{dt:.1f} s, C -O3 restatement of tun/checksum.go + checksumValid, 1 thread",
    }


if __name__ == "__main__":
    main()
