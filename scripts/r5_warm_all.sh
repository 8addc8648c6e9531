#!/bin/bash
# Round 5: what a time-based warmup does to each bench kernel -- the flat read
# of cfg5's bytes, cfg4 (GSO) and GRO shapes with a short vs a ~50-ms warmup.
# Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_warm_all}; mkdir -p $OUT
BIG_ONLY=1 NSHAPES=2 WARM_MS=0 timeout -k 10 200 python -u scripts/probe_stream3.py > $OUT/flat.jsonl 2> $OUT/flat.err || { echo flat0; tail -3 $OUT/flat.err; exit 1; }
BIG_ONLY=1 NSHAPES=2 WARM_MS=60 timeout -k 10 200 python -u scripts/probe_stream3.py >> $OUT/flat.jsonl 2>> $OUT/flat.err || { echo flat60; tail -3 $OUT/flat.err; exit 1; }
cat $OUT/flat.jsonl
for v in "cfg4 - 20" "cfg4 - 6000" "gro_device shuffled 4" "gro_device shuffled 200" "gro_device 4x32 4" "gro_device 4x32 200"; do
  set -- $v
  extra=""; [ $1 = gro_device ] && extra="--gro-shape $2"
  timeout -k 10 200 python bench.py --config $1 $extra --steps 40 --warmup $3 --cpu-seconds 0 --no-e2e > $OUT/run.log 2>&1 || { echo "rc=$? $v"; tail -5 $OUT/run.log; exit 1; }
  grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"tag\": \"$1_$2_w$3\", /" >> $OUT/lines.jsonl
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:28s} value {d['value']:12.1f} kern {r['kernel_ms']*1e3:8.2f} us frac {r['frac']:.4f}")
PY
