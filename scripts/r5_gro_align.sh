#!/bin/bash
# Round 5: GRO with packets on 128-byte lines (gro_device --gro-buf-align,
# the write stager's slices): parity, A/B against the round-4 layout, and the
# L2's sized read requests + WRITE_SIZE per launch (measurement script).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_gro_align}; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${NOTESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_gro_batch.py tests/test_gpu_wstager.py tests/test_gpu_gro.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for rep in 1 2; do
  for shape in ${SHAPES:-4x32 shuffled}; do
    for al in 128 0; do
      timeout -k 10 200 python bench.py --config gro_device --gro-shape $shape --gro-buf-align $al --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e > $OUT/${shape}_a${al}_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $OUT/${shape}_a${al}_$rep.log | sed "s/^{/{\"tag\": \"${shape}_a${al}_$rep\", /" >> $OUT/lines.jsonl
    done
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:20s} {d['value']/1e6:8.1f} Mpkt/s kern {r['kernel_ms']*1e3:7.1f} us frac {r['frac']:.4f}")
PY
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
for shape in ${SHAPES:-4x32 shuffled}; do
  for al in 128 0; do
    for c in sized WRITE_SIZE; do
      ctr=$c; [ $c = sized ] && ctr=$SIZED
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/pmc_${shape}_a${al}_$c -o run --output-format csv -- python3 $ROOT/bench.py --config gro_device --gro-shape $shape --gro-buf-align $al --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/pmc_${shape}_a${al}_$c.log 2>&1) || { echo "FAIL pmc $shape $al $c"; exit 1; }
    done
    echo "== $shape align $al: $(python3 scripts/pmc_sized.py $OUT/pmc_${shape}_a${al}_sized gro_batch | cut -c80-400)"
  done
done
