#!/bin/bash
# Round 4 probe: 2 / 3 / 4 launch streams (8 hardware queues) for gro_device,
# udp_split and udp_coalesce, interleaved, 2 rounds.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_streams_other}; mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2; do
  for cfg in gro_device udp_split udp_coalesce; do
    for S in 2 3 4; do
      GPU_MAX_HW_QUEUES=8 timeout -k 10 150 python bench.py --config $cfg --streams $S --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e > $OUT/run.log 2>&1 || { echo "rc=$? $cfg $S"; tail -5 $OUT/run.log; exit 1; }
      grep '^{' $OUT/run.log | sed "s/^{/{\"S\": $S, \"cfg\": \"$cfg\", \"round\": $r, /" >> $OUT/ab.jsonl
    done
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['cfg'], 'S', d['S'], d['round'], r['kernel_ms'], r['frac'])"
