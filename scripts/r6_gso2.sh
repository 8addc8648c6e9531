#!/bin/bash
# Round 6: staged GSO (head published by an LDS word, no barrier) -- parity,
# stamps, interleaved A/B against round 5's kernel.  NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
T=${TAG:-r6_gso2}
OUT=$ROOT/gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_stager.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
NWAVES=12 timeout -k 10 120 python scripts/probe_gso_stamps.py run > $OUT/stamps.jsonl 2>&1 || exit 1
LIBS=${LIBS:-"libwgcsum.so scripts/probe_so/libwgcsum_r5gso.so"}
TAG=${T}_ab LIBS="$LIBS" bash scripts/r5_gso_ab.sh 2 || exit 1
TAG=${T}_ab1 LIBS="$LIBS" BENCH_ARGS="--streams 1" bash scripts/r5_gso_ab.sh 2 || exit 1
echo done
