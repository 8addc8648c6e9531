#!/usr/bin/env python3
"""Where does bench.py's wall time go beyond the GPU span? (round 3)

Interleaves enqueue variants of the headline bench's timed region (K launches
of the cfg2 VALIDATE kernel over rotated copies) and reports, per variant, the
median / min wall time (sync; t0; enqueue; sync; t1), HIP-event span, and the
host time of the enqueue itself:
  py     Python loop, one wgcs_checksum_batch per step, torch events (round-2 bench)
  pyb    Python loop, one wgcs_checksum_batches call per step
  c      one wgcs_checksum_batches call for all K steps, events recorded in C
  cne    same, no events
  pyne   Python loop, no events
for S launch streams.  usage: probe_bracket.py [K] [trials] [S...]
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("ROC_ACTIVE_WAIT_TIMEOUT", "100000")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from wireguard_amd import synth  # noqa: E402
from wireguard_amd.tun import Device, MODE_VALIDATE  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    S_list = [int(x) for x in sys.argv[3:]] or [2]
    torch.cuda.set_device(0)
    dev = Device(0)
    arena_np, pkts_np, _ = synth.make_batch(65536, 1500, kinds="tcp4")
    n = len(pkts_np)
    nbytes = int(pkts_np["len"].astype(np.int64).sum())
    R = 4
    arenas = [torch.from_numpy(arena_np).to("cuda") for _ in range(R)]
    pkts = torch.from_numpy(pkts_np.view(np.uint8)).to("cuda")
    outs = [torch.empty(n * 2, dtype=torch.uint8, device="cuda") for _ in range(R)]
    Smax = max(S_list)
    streams = [torch.cuda.Stream() for _ in range(Smax)]
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    e1.record(streams[0])
    joins = [torch.cuda.Event() for _ in streams]
    one = [dev.batch_list([(arenas[i], pkts, n, outs[i])]) for i in range(R)]

    def bl(k0):
        return dev.batch_list([(arenas[(k0 + k) % R], pkts, n, outs[(k0 + k) % R]) for k in range(K)])

    def run(var, S, k0):
        ss = streams[:S]
        b = bl(k0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev = var not in ("cne", "pyne")
        if var in ("c", "cne"):
            dev.checksum_batches(MODE_VALIDATE, b, ss, e0 if ev else None, e1 if ev else None)
        else:
            if ev:
                e0.record(ss[0])
                for st in ss[1:]:
                    st.wait_event(e0)
            for k in range(K):
                i = (k0 + k) % R
                if var == "pyb":
                    dev.checksum_batches(MODE_VALIDATE, one[i], ss[k % S:k % S + 1])
                else:
                    dev.checksum_batch(MODE_VALIDATE, arenas[i], pkts, n, outs[i], stream=ss[k % S])
            if ev:
                for j, st in zip(joins, ss[1:]):
                    j.record(st)
                    ss[0].wait_event(j)
                e1.record(ss[0])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        span = e0.elapsed_time(e1) * 1e3 if ev else float("nan")
        return (t2 - t0) * 1e6, span, (t1 - t0) * 1e6

    variants = ["py", "pyb", "c", "cne", "pyne"]
    for S in S_list:
        for v in variants:  # warm
            run(v, S, 0)
        res = {v: [] for v in variants}
        for t in range(trials):
            for v in (variants if t % 2 == 0 else variants[::-1]):
                res[v].append(run(v, S, t * K))
        for v in variants:
            w = [r[0] for r in res[v]]
            sp = [r[1] for r in res[v]]
            enq = [r[2] for r in res[v]]
            wm = statistics.median(w)
            out = {"probe": "bracket", "variant": v, "S": S, "K": K, "trials": trials,
                   "wall_us_med": round(wm, 1), "wall_us_min": round(min(w), 1),
                   "span_us_med": round(statistics.median(sp), 1), "enqueue_us_med": round(statistics.median(enq), 1),
                   "wall_minus_span_med": round(statistics.median([a - b for a, b in zip(w, sp)]), 1),
                   "GiB_s_med": round(nbytes * K / (wm * 1e-6) / 2**30, 1)}
            print(json.dumps(out), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
