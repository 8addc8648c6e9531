#!/bin/bash
# Round 5: does the chip need a time-based warmup?  The same K-step region
# timed 6 times per process (bench.py --repeat), by warmup depth, for the
# headline (cfg2) and configs[4] (cfg5).  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_warm_regions}; mkdir -p $OUT
for v in ${VARIANTS:-"cfg2 5" "cfg2 2000" "cfg2 5" "cfg2 2000"}; do
  set -- $v
  timeout -k 10 200 python bench.py --config $1 --steps 20 --warmup $2 --repeat 6 --cpu-seconds 0 --no-e2e --no-strong > $OUT/$1_w$2.log 2>&1 || { echo "rc=$? $v"; tail -5 $OUT/$1_w$2.log; exit 1; }
  grep '^{"metric"' $OUT/$1_w$2.log | sed "s/^{/{\"tag\": \"$1_w$2\", /" >> $OUT/lines.jsonl
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); t = d["timing"]; K = d["steps"]
    reps = [round(r["event_span_us"] / K, 2) for r in t.get("repeats", [])]
    print(d["tag"], round(d["roofline"]["kernel_ms"] * 1e3, 2), d["roofline"]["frac"], d["value"], "repeats us/launch:", reps,
          "ungated:", round(t.get("ungated", {}).get("event_span_us", 0) / K, 2))
PY
