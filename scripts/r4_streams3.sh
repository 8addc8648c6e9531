#!/bin/bash
# Round 4 probe: three launch streams (with GPU_MAX_HW_QUEUES=8 so each gets a
# hardware queue) against the bench's two, cfg4 and cfg2, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_streams3}; mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2; do
  for cfg in cfg4 cfg2; do
    for v in "2 4" "2 8" "3 8" "4 8"; do
      set -- $v
      GPU_MAX_HW_QUEUES=$2 timeout -k 10 150 python bench.py --config $cfg --streams $1 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e --no-strong > $OUT/run.log 2>&1 || { echo "rc=$? $cfg $v"; tail -5 $OUT/run.log; exit 1; }
      grep '^{' $OUT/run.log | sed "s/^{/{\"S\": $1, \"hwq\": $2, \"cfg\": \"$cfg\", \"round\": $r, /" >> $OUT/ab.jsonl
    done
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['cfg'], 'S', d['S'], 'hwq', d['hwq'], d['round'], r['kernel_ms'], r['frac'], r.get('kernel_ms_one_stream'))"
