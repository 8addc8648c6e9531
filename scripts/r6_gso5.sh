#!/bin/bash
# Round 6: staged GSO -- parity, per-role stamps, A/B vs round 5 (NOT product code).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
T=${TAG:-r6_gso5}
OUT=$ROOT/gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_stager.py tests/test_gpu_fullsize.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
STAMPS_SO=scripts/probe_so/libwgcsum_gso_roles.so timeout -k 10 120 python scripts/probe_gso_roles.py > $OUT/roles.jsonl 2>&1 || exit 1
LIBS=${LIBS:-"libwgcsum.so scripts/probe_so/libwgcsum_r5gso.so"}
TAG=${T}_ab LIBS="$LIBS" bash scripts/r5_gso_ab.sh 2 || exit 1
TAG=${T}_ab1 LIBS="$LIBS" BENCH_ARGS="--streams 1" bash scripts/r5_gso_ab.sh 2 || exit 1
echo done
