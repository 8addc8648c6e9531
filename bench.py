#!/usr/bin/env python3
"""bench.py -- device-resident Internet-checksum throughput on MI355X.

Metric (BASELINE.json): "device-resident payload GiB/s, Internet checksum,
64k×1500B batch".  One step = one pass of the hot path (one launch of
WGCS_MODE_VALIDATE = checksumValid, /root/reference/tun/gro.go:554-612) over
one batch of 65,536 × 1500-B TCP/IPv4 frames already resident in HBM.  Payload
bytes = sum of frame lengths (every byte of a frame is read: addresses for the
pseudo-header, the L4 header and the payload).

Contract: `python bench.py --gpus N --steps K --warmup W`; for N>1 it runs
under torch.distributed.run, one rank per GPU.  Default config (cfg2): each
rank checksums its own 64k batch (weak scaling, no data-path collective --
per-packet checksums are independent).  --config cfg5 runs
the 1,048,576-frame mixed batch split across the ranks (strong scaling).  The
timed region is bracketed by a barrier + device sync on both sides; the max
time over ranks is used; rank 0 prints ONE JSON line.

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

# Host completion wait: spin on the HIP completion signal instead of sleeping
# on the interrupt after the runtime's default 10 us, as a latency-bound
# packet datapath would (busy-poll).  Host-side only: the GPU work is the same.
# Must be set before the HIP runtime initialises (torch import).
os.environ.setdefault("ROC_ACTIVE_WAIT_TIMEOUT", "100000")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md

CONFIGS = {
    # name: (packets, frame_len, kinds, BASELINE.json configs index, scaling)
    "cfg1": (1024, 1500, "udp4", 0, "weak"),  # the reference's CPU plumbing case; GPU leg as context
    "cfg2": (65536, 1500, "tcp4", 1, "weak"),
    "cfg3": (65536, 9000, "tcp4", 2, "weak"),
    "cfg5": (1048576, 1500, "mixed", 4, "strong"),  # global batch, split across the ranks
}
MODE_DESC = {"validate": "validate (checksumValid, gro.go:554-612)",
             "fill": "L4 fill (gsoNoneChecksum, gro.go:1500-1516)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg2",
                    choices=sorted(CONFIGS) + ["cfg4", "gro", "gro_staged", "gro_device", "udp_split", "udp_coalesce"])
    ap.add_argument("--mode", default="validate", choices=["validate", "fill"])
    ap.add_argument("--rotate", type=int, default=4, help="distinct batch copies (defeat the 256 MiB MALL)")
    ap.add_argument("--streams", type=int, default=0,
                    help="launch streams, consecutive batches round-robin (0: 2; 4 for cfg4 and the launch-bound cfg1; 1 for cfg5, whose 0.26-ms launches gain nothing from overlapping boundaries)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-event-timing", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive end-to-end measurement")
    ap.add_argument("--push-threads", type=int, default=0,
                    help="gro_staged: host threads pushing Write calls concurrently (default 4)")
    ap.add_argument("--pinned", action="store_true",
                    help="gro_staged: Write buffers in pinned host memory, zero-copy pushes")
    ap.add_argument("--gro-shape", default="4x32", choices=["4x32", "1x128", "4x32rev", "1x128rev", "shuffled", "4x32udp", "1x128udp", "16x8", "32x4"],
                    help="gro_device: the packets of each Write call (wireguard_amd/gro_bench.py CALL_SHAPES)")
    ap.add_argument("--max-segs", type=int, default=128,
                    help="cfg4: output slots per read = len(bufs) (the reference's Read passes conn.BatchSize = 128)")
    ap.add_argument("--frame-stride", type=int, default=0,
                    help="cfg1-3: frame k at k * stride in the arena (0: back to back, the frame length)")
    ap.add_argument("--gso-out-align", type=int, default=128,
                    help="cfg4: output slots placed so that bufs[i][offset] starts on this many bytes (0: as allocated)")
    ap.add_argument("--gso-in-align", type=int, default=128,
                    help="cfg4: each read's buffer at a multiple of this many bytes in the arena (0: packed)")
    ap.add_argument("--gro-buf-align", type=int, default=128,
                    help="gro_device: buffers placed so that bufs[k][offset] starts on this many bytes (0: 16-byte "
                         "multiples back to back)")
    ap.add_argument("--verify", action="store_true", help="check the GPU results against the synth ground truth")
    ap.add_argument("--no-strong", action="store_true",
                    help="cfg2: skip the configs[4] block (the 1M mixed batch split over the ranks, `cfg5_strong`)")
    ap.add_argument("--no-gate", action="store_true",
                    help="enqueue the K steps inside the timed region instead of posting them behind a doorbell")
    ap.add_argument("--poll", action="store_true",
                    help="poll the closing event before torch.cuda.synchronize() (slower: profiles/r4_probe_poll_ab.jsonl)")
    ap.add_argument("--no-affinity", action="store_true", help="do not bind each rank to its GPU's NUMA-local CPUs")
    ap.add_argument("--warm-ms", type=float, default=40.0,
                    help="configs[4] legs (cfg5_strong, --config cfg5): AFTER the contract region (K steps behind "
                         "exactly W warmup steps, which is `value`), keep issuing untimed steps for at least this "
                         "much wall time and time the K steps again as the diagnostic `value_warm` (the chip streams "
                         "~15 %% slower for ~25 ms after idling; profiles/r5_cfg5_regions.jsonl); 0 = no warm re-time")
    ap.add_argument("--repeat", type=int, default=1,
                    help="diagnostics: time the K-step region this many times; `value` stays the FIRST region, "
                         "the others are listed under timing.repeats")
    return ap.parse_args()


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher_cmd(gpus: int, argv: list[str], port: int) -> list[str]:
    """The torch.distributed.run command that runs this bench as `gpus` ranks
    (one process per GPU) with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def launch_ranks(args, argv: list[str]) -> int | None:
    """`--gpus N` without a launcher: run N ranks under torch.distributed.run as
    a CHILD process (started before torch or HIP is touched in this process;
    never exec) and return its exit code.  Under a launcher, WORLD_SIZE must
    equal --gpus.  Returns None when this process is itself the (only) rank."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import subprocess

    return subprocess.run(launcher_cmd(args.gpus, argv, _free_port())).returncode


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    rc = launch_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if args.streams <= 0:
        # cfg4: four launch streams, each on its own hardware queue (below) --
        # 7.5 us per GSO launch against 7.9 with two (profiles/r4_probe_streams3.jsonl);
        # cfg1's 1.5-MB launches are launch-bound: four streams overlap them, 1.24 us
        # per launch against 3.23 on one (profiles/r4_probe_cfg1_streams.jsonl); the
        # 98-MB checksum configs are fastest on two, cfg5's 0.26-ms launches on one
        args.streams = {"cfg5": 1, "cfg4": 4, "cfg1": 4}.get(args.config, 2)
    # HIP's default of 4 hardware queues per process would put two of the launch
    # streams on one queue once the context's and torch's streams are counted:
    # raise it (before HIP initialises) when the streams need more
    hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    if args.streams + 2 > hwq:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(8, args.streams + 2)))
    import torch  # before wireguard_amd: one HIP runtime per process

    from wireguard_amd import shard, synth
    from wireguard_amd.tun import Device, MODE_VALIDATE, MODE_L4_FILL

    world, rank, local = shard.dist_env()
    dist = None
    # WGCS_DIST_BACKEND=gloo rehearses the N>1 bench on a box with fewer GPUs
    # than ranks (ranks then share devices round-robin); the driver's runs use
    # RCCL ("nccl") with one GPU per rank.
    backend = os.environ.get("WGCS_DIST_BACKEND", "nccl")
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl" and torch.cuda.device_count() < world:
            sys.exit(f"bench.py: {world} RCCL ranks need {world} GPUs, {torch.cuda.device_count()} visible "
                     "(WGCS_DIST_BACKEND=gloo rehearses ranks sharing a GPU)")
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    red_dev = "cuda" if backend == "nccl" else "cpu"

    def barrier():
        if dist is not None:
            dist.barrier()

    # N > 1: each rank on its GPU's NUMA-local cores before anything pins host
    # memory (the Device's staging, the end-to-end leg), so the node's ranks
    # do not cross sockets; one rank keeps the whole CPU share it was given
    affinity = None
    if world > 1 and not args.no_affinity:
        affinity = shard.bind_numa_local(torch, local)
    dev = Device(local if world > 1 else 0)
    if args.config == "cfg4":
        from wireguard_amd import gso_bench

        return gso_bench.run(args, torch, dev, dist, rank, world, local, barrier)
    if args.config == "gro":
        from wireguard_amd import gro_bench

        return gro_bench.run(args, torch, dev, dist, rank, world, local, barrier)
    if args.config == "gro_staged":
        from wireguard_amd import gro_bench

        return gro_bench.run_staged(args, torch, dev, dist, rank, world, local, barrier)
    if args.config == "gro_device":
        from wireguard_amd import gro_bench

        return gro_bench.run_device(args, torch, dev, dist, rank, world, local, barrier)
    if args.config in ("udp_split", "udp_coalesce"):
        from wireguard_amd import udp_bench

        return udp_bench.run(args, torch, dev, dist, rank, world, local, barrier)

    n_cfg, flen, kinds, cfg_idx, scaling = CONFIGS[args.config]
    mode = MODE_VALIDATE if args.mode == "validate" else MODE_L4_FILL
    if scaling == "strong":
        arena_np, pkts_np, _, lo, hi = shard.make_global_shard(n_cfg, rank, world, flen, kinds)
    else:  # every rank its own seeded 64k batch
        arena_np, pkts_np, _ = synth.make_batch(n_cfg, flen, kinds=kinds, seed=synth.SEED + rank,
                                                stride=args.frame_stride or None)
    n = len(pkts_np)
    bytes_per_step = int(pkts_np["len"].astype(np.int64).sum())
    use_events = not args.no_event_timing
    leg = checksum_leg(torch, dev, arena_np, pkts_np, mode, args.steps, args.warmup, args.streams, args.rotate,
                       barrier, use_events, repeat=args.repeat, verify=args.verify, gate=not args.no_gate,
                       poll=args.poll, warm_ms=args.warm_ms if scaling == "strong" else 0.0)
    local_elapsed, kern_ms, iso_ms, S, R = leg["elapsed"], leg["kern_ms"], leg["iso_ms"], leg["streams"], leg["R"]
    elapsed = shard.max_over_ranks(local_elapsed, dist, device=red_dev)
    kern_all = shard.gather_floats(kern_ms if kern_ms is not None else -1.0, dist, device=red_dev)

    total_bytes = bytes_per_step * args.steps * world  # every rank processed bytes_per_step per step
    if scaling == "strong":
        total_bytes = int(n_cfg) * flen * args.steps
    value = total_bytes / elapsed / 2**30
    kname = kernel_name(mode)
    # also the L4-segment-only rate (frame bytes past csum_start)
    l4_frac = float((pkts_np["len"].astype(np.int64) - pkts_np["csum_start"].astype(np.int64)).sum()) / bytes_per_step
    result = {
        "metric": "device-resident payload GiB/s, Internet checksum, 64k×1500B batch",
        "value": round(value, 2),
        "unit": "GiB/s",
        "value_l4_only": round(value * l4_frac, 2),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": (f"{n} x {flen}-B {kinds} frames per GPU" if scaling == "weak" else
                         f"{n_cfg} x {flen}-B {kinds} frames split over {world} GPU(s)") +
                        f", {MODE_DESC[args.mode]} per step, BASELINE.json configs[{cfg_idx}]",
            "packets_per_gpu": n,
            "frame_len": flen,
            "global_batch_bytes": bytes_per_step * world if scaling == "weak" else n_cfg * flen,
            "mode": args.mode,
            "rotated_copies": R,
            "frame_stride": args.frame_stride or flen,
            "streams": S,
            "parallelism": f"shard{world} (no collective)",
        },
    }
    if world > 1:
        result["config"]["dist"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                                    "gpus_visible": torch.cuda.device_count(), "device_of_rank0": local}
    if affinity is not None:
        result["config"]["affinity"] = affinity
    if kern_ms is not None:
        # host-side time inside the timed region beyond the GPU's event span:
        # first-launch latency + the completion wait (this rank; `value` uses the max over ranks)
        result["timing"] = {"wall_us": round(local_elapsed * 1e6, 2), "event_span_us": round(kern_ms * args.steps * 1e3, 2),
                            "wall_minus_span_us": round((local_elapsed - kern_ms * args.steps * 1e-3) * 1e6, 2),
                            "enqueue": ("one wgcs_checksum_batches call for the K steps" +
                                        ("" if args.no_gate else ", posted behind a doorbell (wgcs_stream_wait_flag) "
                                         "rung when the clock starts") +
                                        ("; completion polled on the closing event, then torch.cuda.synchronize()"
                                         if args.poll else ""))}
        if leg.get("ungated"):
            uw, um = leg["ungated"]
            result["timing"]["ungated"] = {
                "what": "the same K steps enqueued inside the clock (no doorbell), timed after the region; "
                        "how rounds 1-3 timed; never `value`",
                "wall_us": round(uw * 1e6, 2), "GiB_per_s": round(bytes_per_step * args.steps / uw / 2**30, 2)}
            if um is not None:
                result["timing"]["ungated"]["event_span_us"] = round(um * args.steps * 1e3, 2)
        if leg.get("warm"):
            ww, wm = leg["warm"]
            wel = shard.max_over_ranks(ww, dist, device=red_dev)
            result["value_cold"] = result["value"]
            result["value_warm"] = round(total_bytes / wel / 2**30, 2)
            result["timing"]["warm"] = warm_block(args.warm_ms, leg["prewarm"], ww, wm, args.steps)
        if leg["repeats"]:
            result["timing"]["repeats"] = [{"wall_us": round(w * 1e6, 1), "event_span_us": round(m * args.steps * 1e3, 1)}
                                           for w, m in leg["repeats"]]
        result["roofline"] = roofline(kname, bytes_per_step, flen, n, kern_ms, S, iso_ms, kern_all)
    if not args.no_e2e:  # every rank moves its own shard over its own PCIe link; rank 0 reports the aggregate
        e2e = end_to_end(torch, dev, arena_np, pkts_np, mode, barrier, dist, red_dev, world)
        if rank == 0:
            result["end_to_end"] = e2e
    if rank == 0 and world == 1 and args.config == "cfg1" and not args.no_e2e:
        result["host_call"] = host_call(dev, arena_np, pkts_np, mode)
    del leg
    # BASELINE.json configs[4] in the same run: the 1,048,576-frame mixed batch
    # split over the N ranks by bytes (strong scaling), its own roofline
    if args.config == "cfg2" and not args.no_strong:
        strong = strong_leg(torch, dev, args, mode, rank, world, barrier, dist, red_dev, use_events)
        if rank == 0:
            result["cfg5_strong"] = strong
    # the CPU baseline on rank 0 at every N (north_star: "reported in the same run")
    if rank == 0 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(arena_np, pkts_np, mode, args.cpu_seconds)
    barrier()  # the other ranks wait for rank 0's CPU leg before tearing down
    if rank == 0:
        print(json.dumps(result), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


REQUIRED_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                 "scaling", "vs_baseline", "dtype", "data", "config")


def line_problems(line: dict, require_cold: bool = True) -> list[str]:
    """What is missing from a cfg2 result line (the driver's default
    invocation), per the bench contract: the required keys, `roofline`,
    `cpu_baseline` at every N, and for N > 1 every rank's kernel time, the
    process group's world size and the `cfg5_strong` block (BASELINE.json
    configs[4]) with its own roofline and (round 6) its
    cold value -- the K steps behind exactly W warmup steps -- as `value` and
    `value_cold`, any warm re-time only beside them.  Empty = complete.
    require_cold=False reads lines recorded before round 6."""
    bad = [f"missing {k}" for k in REQUIRED_KEYS if k not in line]
    if bad:
        return bad
    n = line["n_gpus"]
    rf = line.get("roofline")
    if not rf:
        bad.append("missing roofline")
    else:
        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
            if k not in rf:
                bad.append(f"roofline missing {k}")
        if n > 1 and len(rf.get("kernel_ms_per_rank", [])) != n:
            bad.append("roofline.kernel_ms_per_rank must list every rank")
    cb = line.get("cpu_baseline")
    if not cb or not all(k in cb for k in ("value", "unit", "cores", "kind", "sample")):
        bad.append("cpu_baseline missing or incomplete")
    if n > 1:
        d = line["config"].get("dist", {})
        if d.get("world_size") != n:
            bad.append("config.dist.world_size must equal n_gpus")
    st = line.get("cfg5_strong")
    if st is None:
        bad.append("missing cfg5_strong")
    else:
        if st.get("n_gpus") != n or st.get("scaling") != "strong" or not st.get("value"):
            bad.append("cfg5_strong: n_gpus / scaling / value")
        if len(st.get("packets_per_rank", [])) != n or sum(st.get("packets_per_rank", [])) != CONFIGS["cfg5"][0]:
            bad.append("cfg5_strong.packets_per_rank must cover the 1M batch")
        if require_cold:
            if st.get("value_cold") != st.get("value"):
                bad.append("cfg5_strong.value_cold must be the contract value (K steps behind exactly W warmups)")
            if "value_warm" in st and "warm" not in st:
                bad.append("cfg5_strong.value_warm without its warm block")
        srf = st.get("roofline")
        if not srf or "frac" not in srf or (n > 1 and len(srf.get("kernel_ms_per_rank", [])) != n):
            bad.append("cfg5_strong.roofline missing or without every rank")
    return bad


def kernel_name(mode) -> str:
    from wireguard_amd.tun import MODE_VALIDATE

    return f"checksum_batch_kernel<{'VALIDATE' if mode == MODE_VALIDATE else 'L4_FILL'},{_tune_tag()},nt>"


def roofline(kname, bytes_per_step, flen, n, kern_ms, S, iso_ms, kern_all=None) -> dict:
    """The line's `roofline` object for one rank's checksum launches (kern_ms =
    HIP-event GPU time per launch); kern_all = every rank's kern_ms (N > 1)."""
    from wireguard_amd import traffic

    achieved = bytes_per_step / (kern_ms * 1e-3) / 1e9
    r = {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic.per_launch(kname, bytes_per_step),
        "kernel": kname,
        "kernel_ms": round(kern_ms, 5),
        "kernel_ms_is": ("GPU time per launch over the timed region (HIP events on the launch streams)"
                         + (f"; {S} streams, consecutive launches overlap" if S > 1 else "")
                         + ("; rank 0's, every rank's in kernel_ms_per_rank" if kern_all and len(kern_all) > 1 else "")),
        "algorithmic_bytes_per_launch": bytes_per_step,
        "algorithmic_bytes_per_unit": flen,
        "units_per_launch": n,
    }
    if kern_all and len(kern_all) > 1:
        r["kernel_ms_per_rank"] = [round(k, 5) for k in kern_all]
        r["kernel_ms_min"] = round(min(kern_all), 5)
        r["kernel_ms_max"] = round(max(kern_all), 5)
        r["frac_slowest_rank"] = round(bytes_per_step / (max(kern_all) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    if iso_ms is not None:
        r["kernel_ms_one_stream"] = round(iso_ms, 5)
        r["frac_one_stream"] = round(bytes_per_step / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    return r


def gate_streams(dev, bell, streams, use_events) -> list:
    """Post the doorbell wait (wgcs_stream_wait_flag on bell[0] == 1) on the
    launch streams of a gated region and return the streams that wait on it.
    With the bracket events on, streams[1:] wait on e0, which is recorded on
    stream 0 behind the bell, so stream 0 alone is gated; without events
    nothing else would hold them before the clock starts, so each waits on the
    bell itself (tests/test_gpu_abi_safety.py drives this helper)."""
    gated = list(streams[:1]) if use_events else list(streams)
    for s in gated:
        dev.stream_wait_flag(s, bell, 1)
    return gated


def checksum_leg(torch, dev, arena_np, pkts_np, mode, steps, warmup, streams, rotate, barrier, use_events,
                 repeat=1, verify=False, iso=True, gate=True, poll=False, warm_ms=0.0):
    """Time `steps` checksum launches (one batch each, inputs resident in HBM)
    after `warmup` untimed ones.  Returns {elapsed (this rank's wall s),
    kern_ms (HIP events, GPU ms per launch), iso_ms (one-stream reference),
    repeats, streams, R}."""
    from wireguard_amd.tun import MODE_VALIDATE

    n = len(pkts_np)
    flen = int(pkts_np["len"][0]) if n else 0
    bytes_per_step = int(pkts_np["len"].astype(np.int64).sum())
    # Consecutive steps are independent batches (their own rotated arena and
    # output), launched round-robin over S streams: step k+1's kernel streams
    # while step k's drains and pays its end-of-kernel L2 writeback, which a
    # single stream serialises (~1.7 us per boundary, MI355X_MICROARCH.md).
    S = max(1, streams)
    strm = [torch.cuda.Stream() for _ in range(S)]
    R = rotate if bytes_per_step * rotate > (300 << 20) else max(rotate, (400 << 20) // max(bytes_per_step, 1))
    R = max(R, 2 * S)
    arenas = [torch.from_numpy(arena_np).to("cuda") for _ in range(R)]
    pkts = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
    outs = [torch.empty(max(n, 1) * 2, dtype=torch.uint8, device="cuda") for _ in range(R)]
    torch.cuda.synchronize()

    def batches(K, k0):  # steps k0 .. k0+K-1: each its own rotated arena and output
        return dev.batch_list([(arenas[(k0 + k) % R], pkts, n, outs[(k0 + k) % R]) for k in range(K)])

    # The K steps are enqueued by ONE library call (wgcs_checksum_batches: step k
    # on stream k % S), which also records the HIP bracket events on the launch
    # streams: e0 on stream 0 before the first launch (the others wait on it),
    # every other stream joined to stream 0 before e1, so (e1 - e0) / K is the
    # GPU time per launch over the timed region.  One call instead of K Python
    # calls: the first launch leaves the host ~10 us sooner and no per-step
    # ctypes/torch path runs inside the region.
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(strm[0])  # torch creates the HIP events on their first record
    e1.record(strm[0])

    # The doorbell (gate): the K launches are posted behind a device-side wait
    # on a pinned flag (wgcs_stream_wait_flag) before the clock starts, and the
    # clock starts when the host rings it -- as a receive ring posts batches
    # ahead and releases them when due.  The timed region then holds the K
    # launches' GPU work and the completion wait, not the host's enqueue calls.
    bell = dev.host_alloc(64).view(np.uint32) if gate else None

    def timed(K, k0, ns, gated=True):
        bl = batches(K, k0)  # the step list (pointers only) is built before the clock starts
        barrier()
        torch.cuda.synchronize()
        evs = (e0 if use_events else None, e1 if use_events else None)
        if bell is not None and gated:
            bell[0] = 0
            gate_streams(dev, bell, strm[:ns], use_events)
            try:
                dev.checksum_batches(mode, bl, strm[:ns], *evs)
            finally:
                t0 = time.perf_counter()
                bell[0] = 1  # ring: never leave the streams gated
        else:
            t0 = time.perf_counter()
            dev.checksum_batches(mode, bl, strm[:ns], *evs)
        # Completion: torch.cuda.synchronize().  Polling the closing event
        # first (--poll) was measured slower: 30-35 us of wall time beyond the
        # GPU's event span against 11-12 us (profiles/r4_probe_poll_ab.jsonl).
        if poll and use_events:
            while not e1.query():
                pass
        torch.cuda.synchronize()
        el = time.perf_counter() - t0  # the closing barrier is not timed: max over ranks covers skew
        barrier()
        return el, (e0.elapsed_time(e1) / K if use_events else None)

    # The one-stream reference (untimed for `value`) runs first, before the
    # timed region's own W warmup steps: measured after a two-stream burst, the
    # same launches read ~2-3 us slower per launch than in a one-stream
    # process (profiles/r2_probe_iso_order.txt).  Then W warmup steps and
    # exactly K timed steps, as the bench contract has it.
    iso_first = os.environ.get("WGCS_ISO_FIRST", "1") == "1"
    iso_ms = None
    if iso and use_events and S > 1 and iso_first:
        dev.checksum_batches(mode, batches(min(warmup, 5), 0), strm[:1])
        _, iso_ms = timed(max(steps, 20), 0, 1)
    # W warmup steps, enqueued exactly as the timed steps are (one call, the
    # same streams, the same bracket events): the first cross-stream wait and
    # join on a stream costs ~40 us once per process (profiles/r3_probe_first_region.txt)
    if warmup > 0:
        dev.checksum_batches(mode, batches(warmup, 0), strm, e0 if use_events else None,
                             e1 if use_events else None)
    torch.cuda.synchronize()
    if verify:
        if mode == MODE_VALIDATE:
            assert bool(outs[0][:n].all().item()), "VALIDATE: synthetic frames must all be valid"
        else:  # L4 fill of a valid frame reproduces the stored checksum field
            got = outs[0].cpu().numpy().view(np.uint16)[:n]
            a = arena_np[: n * flen].reshape(n, flen)
            cs = pkts_np["csum_start"].astype(np.int64) + pkts_np["csum_offset"]
            want = (a[np.arange(n), cs].astype(np.uint16) << 8) | a[np.arange(n), cs + 1]
            assert np.array_equal(got, want), "L4_FILL mismatch vs stored checksums"

    local_elapsed, kern_ms = timed(steps, warmup, S)
    repeats = [timed(steps, warmup + r * steps, S) for r in range(1, repeat)]
    # Large launches (configs[4]: 1.57 GB each at N = 1) run ~15 % slower for
    # the first ~25 ms of sustained streaming after the GPU sat idle (the
    # process builds the 1 M-frame batch on the CPU first): the same 20-step
    # region timed 4 times in a row reads 267 / 258 / 238 / 227 us per launch
    # (profiles/r5_cfg5_regions.jsonl).  The contract region above ran after
    # exactly W warmup steps (`value`, cold); such legs then keep issuing
    # untimed steps, in the same enqueue shape, for at least warm_ms of wall
    # time and time the same K steps again (`value_warm`, a diagnostic).
    prewarm, warm = 0, None
    if warm_ms > 0:
        k0 = warmup + repeat * steps
        t_end = time.perf_counter() + warm_ms / 1e3
        while time.perf_counter() < t_end:
            dev.checksum_batches(mode, batches(8, k0 + prewarm), strm)
            torch.cuda.synchronize()
            prewarm += 8
        warm = timed(steps, k0 + prewarm, S)
    # The same K steps enqueued inside the clock (no doorbell), after the
    # timed region: the rounds before round 4 timed this way, so the line
    # carries both wall times for comparison (never `value`)
    ungated = None
    if bell is not None and iso:
        ungated = timed(steps, warmup + repeat * steps, S, gated=False)
    if iso and use_events and S > 1 and not iso_first:  # the same launches one at a time on one stream
        _, iso_ms = timed(max(steps, 20), warmup + steps, 1)
    del arenas, outs, pkts
    return {"elapsed": local_elapsed, "kern_ms": kern_ms, "iso_ms": iso_ms, "repeats": repeats, "streams": S, "R": R,
            "ungated": ungated, "prewarm": prewarm, "warm": warm}


def strong_leg(torch, dev, args, mode, rank, world, barrier, dist, red_dev, use_events) -> dict:
    """BASELINE.json configs[4]: the seeded 1,048,576 x 1500-B mixed
    TCP4/UDP4/TCP6/UDP6 batch split over the `world` ranks by bytes
    (shard.make_global_shard; no collective), K launches per rank dealt over
    two streams like the headline's (at N = 8 a rank's launch is ~35 us, and
    consecutive launches then overlap their ramp and drain; at N = 1 the
    0.27-ms launches neither gain nor lose).  Value = the whole batch's
    bytes x K / the slowest rank's wall time, over the K steps behind exactly
    W warmup steps (`value_cold`, the same number); `value_warm` re-times them
    after --warm-ms of untimed steps."""
    from wireguard_amd import shard

    n_cfg, flen, kinds, cfg_idx, _ = CONFIGS["cfg5"]
    arena_np, pkts_np, _, lo, hi = shard.make_global_shard(n_cfg, rank, world, flen, kinds)
    bytes_rank = int(pkts_np["len"].astype(np.int64).sum())
    S = 2
    leg = checksum_leg(torch, dev, arena_np, pkts_np, mode, args.steps, args.warmup, S, 2, barrier, use_events,
                       iso=False, gate=not args.no_gate, poll=args.poll, warm_ms=args.warm_ms)
    del arena_np
    elapsed = shard.max_over_ranks(leg["elapsed"], dist, device=red_dev)
    kern_all = shard.gather_floats(leg["kern_ms"] if leg["kern_ms"] is not None else -1.0, dist, device=red_dev)
    ranges = shard.gather_floats(float(hi - lo), dist, device=red_dev)
    out = {
        "value": round(n_cfg * flen * args.steps / elapsed / 2**30, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5),
        "scaling": "strong",
        "workload": f"{n_cfg} x {flen}-B {kinds} (25 % each TCP4/UDP4/TCP6/UDP6) frames split by bytes over "
                    f"{world} GPU(s), {MODE_DESC[args.mode]} per step, BASELINE.json configs[{cfg_idx}]",
        "packets_per_rank": [int(x) for x in ranges],
        "streams": leg["streams"],
        "rotated_copies": leg["R"],
    }
    out["value_cold"] = out["value"]
    if leg["kern_ms"] is not None:
        out["roofline"] = roofline(kernel_name(mode), bytes_rank, flen, hi - lo, leg["kern_ms"], leg["streams"], None,
                                   kern_all)
    if leg.get("warm"):  # the diagnostic re-time after --warm-ms of untimed steps (every rank takes part)
        ww, wm = leg["warm"]
        wel = shard.max_over_ranks(ww, dist, device=red_dev)
        wk_all = shard.gather_floats(wm if wm is not None else -1.0, dist, device=red_dev)
        out["value_warm"] = round(n_cfg * flen * args.steps / wel / 2**30, 2)
        out["warm"] = warm_block(args.warm_ms, leg["prewarm"], ww, wm, args.steps)
        if wm is not None:
            out["warm"]["roofline"] = roofline(kernel_name(mode), bytes_rank, flen, hi - lo, wm, leg["streams"], None,
                                               wk_all)
    return out


def warm_block(warm_ms, launches, wall, kern_ms, steps) -> dict:
    """timing of the K steps re-run after `launches` untimed prewarm steps
    (--warm-ms): a diagnostic beside the contract's cold `value`."""
    b = {"warm_ms": warm_ms, "prewarm_launches": launches, "wall_us": round(wall * 1e6, 2),
         "what": "the same K steps timed again after the contract region and --warm-ms of untimed steps "
                 "(a warm chip); `value` is the region after exactly W warmup steps"}
    if kern_ms is not None:
        b["event_span_us"] = round(kern_ms * steps * 1e3, 2)
    return b


def _tune_tag():
    """G,U of the launched checksum kernel: the library defaults (wgcs_kernels.h
    LaunchTuning: 32 lanes per packet, 4 loads in flight per lane) or the
    WGCS_LANES_PER_PKT / WGCS_UNROLL overrides api.cpp reads."""
    g = int(os.environ.get("WGCS_LANES_PER_PKT", "32"))
    x = "" if os.environ.get("WGCS_XCD", "1") != "0" else ",noxcd"
    u = int(os.environ.get("WGCS_UNROLL", "4"))
    if g == 32:
        u = 6 if u >= 6 else (4 if u >= 4 else 3)
    elif g == 64:
        u = 4 if u >= 4 else 2
    else:
        g, u = 16, (8 if u >= 8 else (6 if u >= 6 else 4))
    return f"{g},{u}{x}"


def end_to_end(torch, dev, arena_np, pkts_np, mode, barrier, dist, red_dev, world, iters=10, chunks=8):
    """Host -> device -> host rate (the path starts and ends in host memory,
    tun/tun.go:490, :688): pinned H2D of the batch, the kernel, D2H of the
    per-packet results, pipelined -- the batch goes in `chunks` pieces whose
    H2D copies run back to back on a copy stream, so chunk k+1's H2D overlaps
    chunk k's kernel and D2H on the compute stream.  Every rank runs it at once on its own GPU and PCIe link; the
    aggregate is all ranks' bytes over the slowest rank's time."""
    from wireguard_amd import tun

    n = len(pkts_np)
    nbytes = int(pkts_np["len"].astype(np.int64).sum())
    out_b = 1 if mode == tun.MODE_VALIDATE else 2
    h_arena = torch.from_numpy(arena_np).pin_memory()
    h_out = torch.empty(n * 2, dtype=torch.uint8).pin_memory()
    d_arena = torch.empty(len(arena_np), dtype=torch.uint8, device="cuda")
    d_out = torch.empty(n * 2, dtype=torch.uint8, device="cuda")
    offs = tun.pkt_off(pkts_np)
    # chunk c: packets [lo, hi), arena bytes [offs[lo], end of packet hi-1), descriptors rebased to the chunk
    bounds = [n * c // chunks for c in range(chunks + 1)]
    parts = []
    for c in range(chunks):
        lo, hi = bounds[c], bounds[c + 1]
        if lo == hi:
            continue
        a0 = int(offs[lo])
        a1 = len(arena_np) if hi == n else int(offs[hi])
        sub = pkts_np[lo:hi].copy()
        tun.set_pkt_off(sub, offs[lo:hi] - np.uint64(a0))
        parts.append((lo, hi, a0, a1, torch.from_numpy(sub.view(np.uint8)).to("cuda")))
    copy_s, comp_s = torch.cuda.Stream(), torch.cuda.Stream()
    evs = [torch.cuda.Event() for _ in parts]
    torch.cuda.synchronize()

    def pipelined():  # H2D chunks back to back on one copy stream; kernel + D2H of chunk k once it has landed
        for k, (lo, hi, a0, a1, d_p) in enumerate(parts):
            with torch.cuda.stream(copy_s):
                d_arena[a0:a1].copy_(h_arena[a0:a1], non_blocking=True)
                evs[k].record(copy_s)
            comp_s.wait_event(evs[k])
            with torch.cuda.stream(comp_s):
                dev.checksum_batch(mode, d_arena[a0:], d_p, hi - lo, d_out[lo * out_b:], stream=comp_s)
                h_out[lo * out_b: hi * out_b].copy_(d_out[lo * out_b: hi * out_b], non_blocking=True)

    def serialized():  # whole batch: H2D, kernel, D2H on one stream
        with torch.cuda.stream(comp_s):
            d_arena.copy_(h_arena, non_blocking=True)
            dev.checksum_batch(mode, d_arena, d_pkts_all, n, d_out, stream=comp_s)
            h_out[: n * out_b].copy_(d_out[: n * out_b], non_blocking=True)

    d_pkts_all = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
    from wireguard_amd import shard

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        barrier()
        return shard.max_over_ranks(dt, dist, device=red_dev)

    dt_pipe = timed(pipelined)
    dt_ser = timed(serialized)
    dt = min(dt_pipe, dt_ser)
    return {"value": round(world * nbytes / dt / 2**30, 2), "unit": "GiB/s", "ms_per_batch": round(dt * 1e3, 4),
            "n_gpus": world, "strategy": "serialized" if dt_ser <= dt_pipe else "pipelined",
            "serialized_GiB_per_s": round(world * nbytes / dt_ser / 2**30, 2),
            "pipelined_GiB_per_s": round(world * nbytes / dt_pipe / 2**30, 2),
            "what": "pinned H2D of the batch + kernel + D2H of the per-packet results, every rank at once "
                    "(aggregate; PCIe bound); the faster of: serialized (whole batch H2D -> kernel -> D2H on one "
                    f"stream) and pipelined ({len(parts)} chunks, H2D back to back on a copy stream, each chunk's "
                    "kernel + D2H on a compute stream once it has landed)"}


def host_call(dev, arena_np, pkts_np, mode, reps=50):
    """The reference-shaped host entry (wgcs_checksum_batch_host: host arena
    in, results out, one round trip) on the whole batch, median per call."""
    arena = arena_np.copy()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dev.checksum_batch_host(mode, arena, pkts_np)
        ts.append(time.perf_counter() - t0)
    med = float(np.median(ts))
    nbytes = int(pkts_np["len"].astype(np.int64).sum())
    return {"call": "wgcs_checksum_batch_host on the whole batch (host buffers, one PCIe round trip)",
            "median_us": round(med * 1e6, 1), "GiB_per_s": round(nbytes / med / 2**30, 3)}


def _time_oracle(oracle, mode, arena_np, pkts_np, threads, seconds):
    oracle.checksum_batch_mt(mode, arena_np, pkts_np, threads)  # warm
    reps = 0
    t0 = time.perf_counter()
    while True:
        oracle.checksum_batch_mt(mode, arena_np, pkts_np, threads)
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return reps, time.perf_counter() - t0


def _go_note() -> str:
    """north_star asks for the pure-Go CPU baseline: say whether a Go toolchain
    exists on this host (none on the GPU boxes: profiles/r3_go_probe.txt)."""
    import shutil

    found = [t for t in ("go", "gccgo", "tinygo") if shutil.which(t)]
    if found:
        return f"Go toolchain present ({', '.join(found)}) but no pure-Go leg is built"
    return "no Go toolchain on this host (go, gccgo, tinygo absent), so the pure-Go baseline cannot run here"


def cpu_baseline(arena_np, pkts_np, mode, seconds):
    """The oracle (C restatement of tun/checksum.go) on the same batch: one
    thread for `seconds`, plus an all-host-cores leg for a quarter of that --
    pthreads over packet ranges of the one batch, or, for batches under 64 MB
    (cfg1: a pass is too short to split), every thread running whole passes
    over its own copy."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg: allowed use of the oracle

    nbytes = int(pkts_np["len"].astype(np.int64).sum())
    reps, dt = _time_oracle(oracle, mode, arena_np, pkts_np, 1, seconds)
    threads = oracle.host_threads()
    mt_seconds = max(seconds / 4, 0.5)
    if arena_np.nbytes < (64 << 20):
        rate, passes = oracle.checksum_bench_mt(mode, arena_np, pkts_np, threads, mt_seconds)
        mt = {"value": round(nbytes * rate / 2**30, 3),
              "sample": f"{passes} whole-batch passes on {threads} pthreads, each on its own copy, {mt_seconds:.1f} s"}
    else:
        reps_mt, dt_mt = _time_oracle(oracle, mode, arena_np, pkts_np, threads, mt_seconds)
        mt = {"value": round(nbytes * reps_mt / dt_mt / 2**30, 3),
              "sample": f"{reps_mt} passes, {dt_mt:.1f} s, {threads} pthreads over packet ranges"}
    return {
        "value": round(nbytes * reps / dt / 2**30, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{reps} passes over the same {len(pkts_np)}-frame batch ({nbytes/1e6:.1f} MB), "
                  f"{dt:.1f} s, C -O3 restatement of tun/checksum.go + checksumValid, 1 thread; "
                  + _go_note(),
        "all_cores": dict(mt, unit="GiB/s", cores=threads, host_nproc=os.cpu_count()),
    }


if __name__ == "__main__":
    main()
