#!/bin/bash
# Round 5: GRO with checksumValid's first-line partial taken in step 1: parity,
# A/B against the previous build, sized reads (measurement script).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_gro_fuse}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gro_batch.py tests/test_gpu_wstager.py tests/test_gpu_gro.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for shape in 4x32 shuffled 1x128; do
    for lib in gro_fuse gro_base; do
      WGCS_LIB=$ROOT/scripts/probe_so/libwgcsum_$lib.so timeout -k 10 200 python bench.py --config gro_device --gro-shape $shape --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e > $OUT/${shape}_${lib}_$rep.log 2>&1 || exit 1
      grep '^{"metric"' $OUT/${shape}_${lib}_$rep.log | sed "s/^{/{\"tag\": \"${shape}_${lib}_$rep\", /" >> $OUT/lines.jsonl
    done
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:24s} {d['value']/1e6:8.1f} Mpkt/s kern {r['kernel_ms']*1e3:7.1f} us frac {r['frac']:.4f}")
PY
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
for shape in 4x32 shuffled; do
  (cd /tmp && WGCS_LIB=$ROOT/scripts/probe_so/libwgcsum_gro_fuse.so timeout -s KILL 120 rocprofv3 --pmc $SIZED --kernel-trace -d $OUT/pmc_$shape -o run --output-format csv -- python3 $ROOT/bench.py --config gro_device --gro-shape $shape --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/pmc_$shape.log 2>&1) || { echo "FAIL pmc"; exit 1; }
  echo "== $shape: $(python3 scripts/pmc_sized.py $OUT/pmc_$shape gro_batch | cut -c80-400)"
done
