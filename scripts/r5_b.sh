#!/bin/bash
# Round 5: GRO parity after the wave-scope LDS ordering, GSO store-policy A/B,
# the counters this rocprofv3 offers (measurement script, NOT product code).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5_b; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gro_batch.py tests/test_gpu_wstager.py tests/test_gpu_gro.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/gro_tests.log 2>&1 || { tail -20 $OUT/gro_tests.log; exit 1; }
tail -1 $OUT/gro_tests.log
for shape in 4x32 shuffled; do
  timeout -k 10 200 python bench.py --config gro_device --gro-shape $shape --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e > $OUT/gro_$shape.log 2>&1 || exit 1
  grep '^{"metric"' $OUT/gro_$shape.log | sed "s/^{/{\"tag\": \"gro_$shape\", /" >> $OUT/lines.jsonl
done
TAG=r5_wt LIBS="libwgcsum.so scripts/probe_so/libwgcsum_wt0.so scripts/probe_so/libwgcsum_aux0.so scripts/probe_so/libwgcsum_aux2.so scripts/probe_so/libwgcsum_aux17.so" bash scripts/r5_gso_ab.sh 2 || exit 1
timeout -k 5 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
true
