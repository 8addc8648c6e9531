#!/usr/bin/env python3
"""Per-launch GPU time of one kernel from a rocprofv3 --kernel-trace CSV, for
runs whose launches overlap (consecutive independent batches on 2 streams).

With overlapping launches each dispatch's own duration (what --stats
averages) includes the time it shares the GPU with its neighbour, so the
stats average exceeds the per-launch throughput time.  This script splits the
trace into bursts (launches of the kernel separated by < GAP_US of idle time),
and for every burst of at least MIN_N launches prints
  n, span = last end - first start, span/n (per-launch GPU time, the quantity
  bench.py's HIP events measure over the timed region), the union of busy
  intervals / n, the mean dispatch duration and the mean overlap.
usage: python scripts/trace_span.py TRACE_CSV [KERNEL_SUBSTR] [MIN_N] [GAP_US] [> out.json]
"""
import csv
import json
import sys


def bursts(rows, gap_ns):
    out, cur, end = [], [], None
    for s, e in rows:
        if cur and s - end > gap_ns:
            out.append(cur)
            cur, end = [], None
        cur.append((s, e))
        end = e if end is None else max(end, e)
    if cur:
        out.append(cur)
    return out


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "checksum_batch_kernel"
    min_n = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    gap_ns = float(sys.argv[4]) * 1e3 if len(sys.argv) > 4 else 20e3
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                  for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"])
    for b in bursts(rows, gap_ns):
        if len(b) < min_n:
            continue
        n = len(b)
        span = max(e for _, e in b) - b[0][0]
        busy, cs, ce = 0, None, None  # union of busy intervals
        for s, e in b:
            if ce is None or s > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        dur = sum(e - s for s, e in b) / n
        print(json.dumps({"kernel": sub, "n": n, "span_us": round(span / 1e3, 2),
                          "span_per_launch_us": round(span / n / 1e3, 3),
                          "busy_per_launch_us": round(busy / n / 1e3, 3),
                          "mean_dispatch_us": round(dur / 1e3, 3),
                          "mean_concurrency": round(dur * n / busy, 3)}))


if __name__ == "__main__":
    main()
