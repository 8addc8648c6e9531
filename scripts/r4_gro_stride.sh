#!/bin/bash
# Round 4 probe: gro_device with the Write buffers 65,552 B apart (packed
# Go-sized slices), 65,664 (128-B multiple) and 69,632 (page multiple, where
# Go's allocator puts a 65,551-B slice), 4x32 and shuffled, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_gro_stride}; mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2; do
  for shape in 4x32 shuffled; do
    for st in 65552 65664 69632; do
      WGCS_GRO_STRIDE=$st timeout -k 10 150 python bench.py --config gro_device --gro-shape $shape --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e > $OUT/run.log 2>&1 || { echo "rc=$? $shape $st"; tail -5 $OUT/run.log; exit 1; }
      grep '^{' $OUT/run.log | sed "s/^{/{\"stride\": $st, \"shape\": \"$shape\", \"round\": $r, /" >> $OUT/ab.jsonl
    done
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['shape'], d['stride'], d['round'], round(d['value']/1e6), r['kernel_ms'], r['frac'])"
