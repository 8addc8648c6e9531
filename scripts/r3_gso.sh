#!/bin/bash
# GSO check: parity tests, then cfg4 lines at 128 and 64 output slots (2 streams and 1 stream).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_gso}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc"; tail -n 2 $OUT/$n.log | cut -c1-300; case $rc in 124|134|137|139) exit $rc;; esac; }
summ() { grep '^{' $OUT/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['config'].get('max_segs'), 'value', d['value'], 'kern_us', round(r['kernel_ms']*1e3,2), 'frac', r['frac'], '1s_us', round(r.get('kernel_ms_one_stream',0)*1e3,2), 'frac1', r.get('frac_one_stream'))"; }
if [ "${TESTS:-1}" = 1 ]; then
step tests 500 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_stager.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
fi
for ms in 128 64; do
  for rep in 1 2; do step cfg4_${ms}_$rep 200 python bench.py --config cfg4 --max-segs $ms --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e; summ cfg4_${ms}_$rep; done
done
if [ "${SQ:-0}" = 1 ]; then
  (cd /tmp && step sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d $OUT/sq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 20 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1)
  python3 scripts/pmc_summary.py $OUT/sq 2>/dev/null | tail -20 || true
fi
