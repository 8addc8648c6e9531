#!/bin/bash
# gro_device: parity tests, one line per call shape, rocprofv3 stats + FETCH/WRITE passes.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_gro}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc"; tail -n 1 $OUT/$n.log | cut -c1-200; case $rc in 124|134|137|139) exit $rc;; esac; }
summ() { grep '^{' $OUT/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['config']['call_shape'], 'Mpps', round(d['value']/1e6,1), 'kern_us', round(r['kernel_ms']*1e3,1), 'frac', r['frac'], 'writes', d['config']['writes_per_call'])"; }
if [ "${TESTS:-1}" = 1 ]; then
step tests 400 python -u -m pytest tests/test_gpu_gro_batch.py tests/test_gpu_wstager.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
fi
for sh in ${SHAPES:-4x32 1x128 4x32rev 1x128rev shuffled}; do
  step gro_$sh 200 python bench.py --config gro_device --gro-shape $sh --steps 40 --warmup 4 --cpu-seconds 0; summ gro_$sh
done
if [ "${PROF:-1}" = 1 ]; then
  for sh in ${PSHAPES:-4x32 1x128}; do
    (cd /tmp && step prof_$sh 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$sh -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config gro_device --gro-shape $sh --steps 20 --warmup 2 --cpu-seconds 0 --streams 1)
    (cd /tmp && step pmcf_$sh 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmcf_$sh -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config gro_device --gro-shape $sh --steps 8 --warmup 2 --cpu-seconds 0 --streams 1)
    (cd /tmp && step pmcw_$sh 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmcw_$sh -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config gro_device --gro-shape $sh --steps 8 --warmup 2 --cpu-seconds 0 --streams 1)
  done
fi
