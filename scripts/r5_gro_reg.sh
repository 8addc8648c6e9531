#!/bin/bash
# Round 5: GRO wave item loop over register-held items (tcp_gro_reg) -- GRO
# parity, then interleaved A/B against the previous build, then the flat-read
# ceiling at cfg5's size (scripts/probe_stream3.py).  Measurement script.
# usage: TAG=... LIBS="scripts/probe_so/a.so libwgcsum.so" bash scripts/r5_gro_reg.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_gro_reg}; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${NOTESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_gro_batch.py tests/test_gpu_gro.py tests/test_gpu_wstager.py > $OUT/tests.txt 2>&1 \
    || { echo "tests rc=$?"; tail -20 $OUT/tests.txt; exit 1; }
  tail -1 $OUT/tests.txt
fi
for r in 1 2; do
  for shape in ${SHAPES:-shuffled 4x32 1x128}; do
    for lib in ${LIBS:-scripts/probe_so/libwgcsum_gro_base.so libwgcsum.so}; do
      p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
      name=$(basename $lib .so)
      WGCS_LIB=$p timeout -k 10 150 python bench.py --config gro_device --gro-shape $shape --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e > $OUT/run.log 2>&1 || { echo "rc=$? $shape $lib"; tail -5 $OUT/run.log; exit 1; }
      grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"lib\": \"$name\", \"shape\": \"$shape\", \"round\": $r, /" >> $OUT/ab.jsonl
    done
  done
done
python3 - $OUT/ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d['roofline']
    print(f"{d['shape']:10s} {d['lib']:24s} {d['round']} {d['value']/1e6:8.1f} M/s kern {r['kernel_ms']*1e3:7.1f} us frac {r['frac']:.4f}")
PY
if [ "${STREAM:-1}" = 1 ]; then
  timeout -k 10 300 python -u scripts/probe_stream3.py > $OUT/stream3.jsonl 2> $OUT/stream3.err || { echo "stream3 rc=$?"; tail -5 $OUT/stream3.err; exit 1; }
  cat $OUT/stream3.jsonl
fi
