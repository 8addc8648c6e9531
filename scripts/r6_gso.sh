#!/bin/bash
# Round 6: staged GSO image -- parity, then an interleaved A/B against the
# round-5 kernel (WGCS_GSO_STAGED=0) and stage sizes, four streams and one,
# and a rocprofv3 one-stream summary.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
T=${TAG:-r6_gso}
OUT=$ROOT/gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_stager.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS=${LIBS:-"libwgcsum.so scripts/probe_so/libwgcsum_r5gso.so scripts/probe_so/libwgcsum_stg1.so scripts/probe_so/libwgcsum_stg4.so"}
TAG=${T}_ab LIBS="$LIBS" bash scripts/r5_gso_ab.sh 2 || exit 1
TAG=${T}_ab1 LIBS="$LIBS" BENCH_ARGS="--streams 1" bash scripts/r5_gso_ab.sh 2 || exit 1
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof1s -o run --output-format csv -- python3 $ROOT/bench.py --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/prof1s.log 2>&1) || exit 1
echo done
