#!/bin/bash
# Round 5: rocprofv3 kernel trace of the configs[4] launches on one stream
# with the --warm-ms prewarm: every launch's own duration in issue order, so
# the ramp (cold launches) and the warm steady state are read off the trace,
# not off HIP events.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_cfg5_trace}; mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --config cfg5 --streams 1 --steps 20 --warmup 5 --warm-ms ${WARM:-40} --cpu-seconds 0 --no-e2e > $OUT/bench.log 2>&1) || { echo "rc=$?"; tail -5 $OUT/bench.log; exit 1; }
grep '^{"metric"' $OUT/bench.log > $OUT/line.jsonl
python3 - $OUT <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
f = glob.glob(out + "/prof/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "checksum_batch_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
t0 = int(rows[0]["Start_Timestamp"])
print("launches", len(d))
for i in range(0, len(d), max(1, len(d) // 24)):
    print(i, round((int(rows[i]["Start_Timestamp"]) - t0) / 1e6, 2), "ms", round(d[i], 1), "us")
last = d[-20:]
print("last 20 mean", round(sum(last) / len(last), 2), "us ->", round(1572864000 / (sum(last) / len(last)) / 1e3 / 8000, 4))
json.dump({"durations_us": d, "starts_ms": [(int(r["Start_Timestamp"]) - t0) / 1e6 for r in rows]}, open(out + "/durations.json", "w"))
PY
