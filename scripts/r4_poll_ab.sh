#!/bin/bash
# Round 4 probe: the driver's bench command with and without polling the
# closing event before torch.cuda.synchronize(), interleaved, 4 each.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_poll}; mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2 3 4; do
  for v in poll nopoll; do
    fl=""; [ $v = poll ] && fl="--poll"
    timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 $fl > $OUT/run.log 2>&1 || { echo "rc=$? $v"; tail -5 $OUT/run.log; exit 1; }
    grep '^{' $OUT/run.log | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $OUT/ab.jsonl
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l)
    print(d['variant'], d['round'], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['timing']['wall_minus_span_us'])"
