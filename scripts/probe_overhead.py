#!/usr/bin/env python3
"""Where does the bench's wall-clock time go beyond the kernel? (round 2)

Times the bench's exact bracket (sync; t0; K launches; sync; t1) for several
K, the host-side enqueue cost of one launch, and a hipGraph replay of the K
launches, so the fixed (first-launch + completion-wait) overhead and the
per-step cost separate.  Run it once per host wait policy, e.g.
  python scripts/probe_overhead.py
  ROC_ACTIVE_WAIT_TIMEOUT=100000 python scripts/probe_overhead.py
(ROC_ACTIVE_WAIT_TIMEOUT: how long the HIP runtime spins on a completion
signal before it sleeps on the interrupt, microseconds.)
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import Device, MODE_VALIDATE  # noqa: E402


def main():
    tag = os.environ.get("ROC_ACTIVE_WAIT_TIMEOUT", "default")
    torch.cuda.set_device(0)
    dev = Device(0)
    arena_np, pkts_np, _ = synth.make_batch(65536, 1500, kinds="tcp4")
    n = len(pkts_np)
    R = 4
    arenas = [torch.from_numpy(arena_np).to("cuda") for _ in range(R)]
    pkts = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
    outs = [torch.empty(n * 2, dtype=torch.uint8, device="cuda") for _ in range(R)]
    stream = torch.cuda.Stream()
    lib, h = dev.lib, dev.h
    sp = stream.cuda_stream
    a_ptr = [a.data_ptr() for a in arenas]
    o_ptr = [o.data_ptr() for o in outs]
    p_ptr = pkts.data_ptr()

    def step_py(k):  # what bench.py does per step
        i = k % R
        dev.checksum_batch(MODE_VALIDATE, arenas[i], pkts, n, outs[i], stream=stream)

    def step_raw(k):  # the bare ctypes call
        i = k % R
        lib.wgcs_checksum_batch(h, MODE_VALIDATE, 0, a_ptr[i], p_ptr, None, n, o_ptr[i], sp)

    for k in range(30):
        step_py(k)
    torch.cuda.synchronize()

    # idle completion wait
    idle = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        idle.append((time.perf_counter() - t0) * 1e6)
    print(json.dumps({"probe": "idle_sync_us", "wait": tag, "median": statistics.median(idle)}), flush=True)

    # host cost of enqueueing one launch (queue kept shallow: sync every 8)
    for name, fn in (("py", step_py), ("raw", step_raw)):
        ts = []
        for rep in range(50):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(8):
                fn(k)
            ts.append((time.perf_counter() - t0) / 8 * 1e6)
        torch.cuda.synchronize()
        print(json.dumps({"probe": "enqueue_us", "fn": name, "wait": tag, "median": statistics.median(ts)}),
              flush=True)

    def bracket(K, fn, trials=9):
        walls, evs, loops = [], [], []
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        for t in range(trials):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(stream)
            for k in range(K):
                fn(t * K + k)
            e1.record(stream)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            walls.append((t2 - t0) * 1e6)
            loops.append((t1 - t0) * 1e6)
            evs.append(e0.elapsed_time(e1) * 1e3)
        return statistics.median(walls), statistics.median(evs), statistics.median(loops)

    for K in (1, 2, 5, 20, 100):
        for name, fn in (("py", step_py), ("raw", step_raw)):
            w, ev, lp = bracket(K, fn)
            print(json.dumps({"probe": "bracket", "K": K, "fn": name, "wait": tag, "wall_us": round(w, 2),
                              "event_us": round(ev, 2), "loop_us": round(lp, 2),
                              "wall_per_step_us": round(w / K, 3), "event_per_step_us": round(ev / K, 3),
                              "overhead_us": round(w - ev, 2)}), flush=True)

    # hipGraph of 20 launches (captured on the bench stream), replayed
    for K in (20, 100):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            step_py(0)  # warm on the stream
            torch.cuda.current_stream().synchronize()
            with torch.cuda.graph(g, stream=stream):
                for k in range(K):
                    step_py(k)
        torch.cuda.synchronize()
        walls, evs = [], []
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        for t in range(9):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(stream)
            with torch.cuda.stream(stream):
                g.replay()
            e1.record(stream)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            evs.append(e0.elapsed_time(e1) * 1e3)
        w, ev = statistics.median(walls), statistics.median(evs)
        print(json.dumps({"probe": "graph", "K": K, "wait": tag, "wall_us": round(w, 2), "event_us": round(ev, 2),
                          "wall_per_step_us": round(w / K, 3), "event_per_step_us": round(ev / K, 3)}), flush=True)
        del g
    dev.close()


if __name__ == "__main__":
    main()
