#!/bin/bash
# rocprofv3 kernel-trace summaries of gro_device (1 stream) for the 4x32 and
# 1x128 call shapes, after the in-order run change.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_gro_prof}; mkdir -p $OUT
for shape in ${SHAPES:-4x32 1x128}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$shape -o run --output-format csv -- python3 bench.py --config gro_device --gro-shape $shape --streams 1 --steps 20 --warmup 3 --cpu-seconds 0 --no-e2e > $OUT/$shape.log 2>&1 || { echo "rc=$? $shape"; tail -5 $OUT/$shape.log; exit 1; }
  grep '^{' $OUT/$shape.log > $OUT/${shape}_line.jsonl
  f=$(find $OUT/$shape -name "*kernel_stats.csv"); [ -n "$f" ] && cp "$f" $OUT/${shape}_kernel_stats.csv
  grep -i gro_batch $OUT/${shape}_kernel_stats.csv | cut -c1-200
done
