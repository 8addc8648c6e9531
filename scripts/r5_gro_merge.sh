#!/bin/bash
# Round 5: GRO header checks and checksumValid in one pass over each packet
# (gro_batch_kernel step 1) -- GRO parity, interleaved A/B against the
# previous build, and the L2's sized read requests + WRITE_SIZE per launch
# for both.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_gro_merge}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_gro_batch.py tests/test_gpu_gro.py tests/test_gpu_wstager.py > $OUT/tests.txt 2>&1 \
  || { echo "tests rc=$?"; tail -20 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
LIBS=${LIBS:-"scripts/probe_so/libwgcsum_gro_base.so libwgcsum.so"}
for r in 1 2; do
  for shape in ${SHAPES:-shuffled 4x32 1x128}; do
    for lib in $LIBS; do
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
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
for shape in ${PMC_SHAPES-4x32 shuffled}; do
  for lib in $LIBS; do
    p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
    name=$(basename $lib .so)
    for c in sized WRITE_SIZE; do
      ctr=$c; [ $c = sized ] && ctr=$SIZED
      (cd /tmp && WGCS_LIB=$p timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/pmc_${shape}_${name}_$c -o run --output-format csv -- python3 $ROOT/bench.py --config gro_device --gro-shape $shape --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/pmc_${shape}_${name}_$c.log 2>&1) || { echo "FAIL pmc $shape $name $c"; exit 1; }
    done
    echo "== $shape $name: $(python3 scripts/pmc_sized.py $OUT/pmc_${shape}_${name}_sized gro_batch | cut -c80-400)"
  done
done
