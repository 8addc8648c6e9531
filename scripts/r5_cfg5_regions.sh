#!/bin/bash
# Round 5: region-to-region spread of the 1 M-frame launches (cfg5) -- the
# same K steps timed 4 times per process, by warmup depth and stream count.
# Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_cfg5_regions}; mkdir -p $OUT
for v in "2 5" "2 40" "1 5" "2 5"; do
  set -- $v
  timeout -k 10 200 python bench.py --config cfg5 --steps 20 --warmup $2 --streams $1 --repeat 4 --cpu-seconds 0 --no-e2e > $OUT/s$1_w$2.log 2>&1 || { echo "rc=$? $v"; tail -5 $OUT/s$1_w$2.log; exit 1; }
  grep '^{"metric"' $OUT/s$1_w$2.log | sed "s/^{/{\"tag\": \"s$1_w$2\", /" >> $OUT/lines.jsonl
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); t = d["timing"]
    reps = [r for r in t.get("repeats", [])]
    print(d["tag"], d["roofline"]["kernel_ms"], d["roofline"]["frac"], "repeats:", reps, "ungated:", t.get("ungated", {}).get("event_span_us"))
PY
