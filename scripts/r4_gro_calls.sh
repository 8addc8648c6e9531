#!/bin/bash
# Round 4 probe: gro_device with 1x / 2x / 3x the resident calls per launch
# (7 per CU = 1,792), 4x32 and shuffled shapes, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_gro_calls}; mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2; do
  for shape in 4x32 shuffled; do
    for c in 1792 3584 5376; do
      WGCS_GRO_CALLS=$c timeout -k 10 150 python bench.py --config gro_device --gro-shape $shape --steps 20 --warmup 3 --cpu-seconds 0 --no-e2e > $OUT/run.log 2>&1 || { echo "rc=$? $shape $c"; tail -5 $OUT/run.log; exit 1; }
      grep '^{' $OUT/run.log | sed "s/^{/{\"calls\": $c, \"shape\": \"$shape\", \"round\": $r, /" >> $OUT/ab.jsonl
    done
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['shape'], d['calls'], d['round'], round(d['value']/1e6), r['kernel_ms'], r['frac'])"
