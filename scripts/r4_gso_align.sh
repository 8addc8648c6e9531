#!/bin/bash
# Round 4: cfg4 with the output slots placed so that bufs[i][offset] starts on a
# 128-B line (and the jobs at 128-B multiples), interleaved A/B on one box.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_gso_align}; mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2 3; do
  for v in "0 0" "128 0" "128 128" "0 128" "64 0"; do
    set -- $v
    timeout -k 10 120 python bench.py --config cfg4 --steps 50 --warmup 10 --cpu-seconds 0 --no-e2e \
      --gso-out-align $1 --gso-in-align $2 > $OUT/run.log 2>&1 || { echo "rc=$? on $v"; tail -5 $OUT/run.log; exit 1; }
    grep '^{' $OUT/run.log | sed "s/^{/{\"out_align\": $1, \"in_align\": $2, \"round\": $r, /" >> $OUT/ab.jsonl
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['out_align'], d['in_align'], d['round'], r['kernel_ms'], r.get('kernel_ms_one_stream'), r['frac'])"
