#!/bin/bash
# Round 5: the headline kernel on one stream under rocprofv3 (the judge's
# fraction is its kernel-stats average): the one-pass grid against round 4's
# 16 blocks per CU, twice each, with per-launch durations from the trace.
# Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_cfg2_1s_prof}; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for v in base BLOCKS_PER_CU=16; do
    envs=(); [ $v != base ] && envs=("WGCS_$v")
    name=${v//=/}_$r
    (cd /tmp && env "${envs[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run --output-format csv -- python3 $ROOT/bench.py --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e --no-strong > $OUT/$name.log 2>&1) || { echo "FAIL $name"; tail -5 $OUT/$name.log; exit 1; }
    python3 - $OUT/$name <<'PY'
import csv, statistics, sys
d = sys.argv[1]
for r in csv.DictReader(open(d + "/run_kernel_stats.csv")):
    if "checksum_batch" in r["Name"]:
        avg = float(r["AverageNs"]) / 1e3
tr = [r for r in csv.DictReader(open(d + "/run_kernel_trace.csv")) if "checksum_batch" in r["Kernel_Name"]]
dur = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tr)
print(d.split("/")[-1], "launches", len(dur), "avg", round(avg, 2), "median", round(statistics.median(dur), 2), "min", round(dur[0], 2), "frac(avg)", round(98304000 / avg / 1e3 / 8000, 4))
PY
    grep '^{"metric"' $OUT/$name.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.readline()); r=d['roofline']; print('   events 1s', r['kernel_ms']*1e3, r['frac'])"
  done
done
