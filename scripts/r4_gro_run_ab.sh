#!/bin/bash
# Round 4 probe: GRO in-order runs decided 64 packets at a time by a wave
# (tcp_append_run) against the one-lane walker (exp/libwgcsum_base.so, the
# previous build), same box, interleaved, after the GRO parity tests.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_gro_run}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gro_batch.py tests/test_gpu_gro.py tests/test_gpu_wstager.py > $OUT/tests.txt 2>&1 \
  || { echo "tests rc=$?"; tail -20 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
: > $OUT/ab.jsonl
for r in 1 2; do
  for shape in ${SHAPES:-4x32 1x128 shuffled 4x32rev}; do
    for lib in ${LIBS:-base new}; do
      if [ $lib = new ]; then unset WGCS_LIB; else export WGCS_LIB=$PWD/exp/libwgcsum_$lib.so; fi
      steps=40; [ $shape = 4x32rev ] && steps=8
      timeout -k 10 150 python bench.py --config gro_device --gro-shape $shape --steps $steps --warmup 3 --cpu-seconds 0 --no-e2e > $OUT/run.log 2>&1 || { echo "rc=$? $shape $lib"; tail -5 $OUT/run.log; exit 1; }
      grep '^{' $OUT/run.log | sed "s/^{/{\"lib\": \"$lib\", \"shape\": \"$shape\", \"round\": $r, /" >> $OUT/ab.jsonl
    done
  done
done
unset WGCS_LIB
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['shape'], d['lib'], d['round'], round(d['value']/1e6), r['kernel_ms'], r['frac'])"
