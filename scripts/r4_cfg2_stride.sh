#!/bin/bash
# Round 4 probe: cfg2 with frames back to back (1500 B apart, the headline) vs
# frames in 1504- / 1536- / 2048-B slots, interleaved on one box.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_cfg2_stride}; mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2 3; do
  for st in 0 1504 1536 2048; do
    timeout -k 10 120 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e --no-strong --frame-stride $st > $OUT/run.log 2>&1 || { echo "rc=$? on $st"; tail -5 $OUT/run.log; exit 1; }
    grep '^{' $OUT/run.log | sed "s/^{/{\"stride\": $st, \"round\": $r, /" >> $OUT/ab.jsonl
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['stride'], d['round'], d['value'], r['kernel_ms'], r.get('kernel_ms_one_stream'), r['frac'])"
