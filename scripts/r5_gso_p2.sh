#!/bin/bash
# Round 5: more GSO launch shapes with the scalar head -- P = 2 x 8 waves,
# P = 3 x 8, P = 2 x 4 -- against the default P = 3 x 4: GSO parity per build,
# then interleaved cfg4 lines on four streams and one.  Measurement script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_gso_p2}; mkdir -p $OUT
LIBS=${LIBS:-"libwgcsum.so scripts/probe_so/libwgcsum_gso_p2w8s.so scripts/probe_so/libwgcsum_gso_p3w8s.so scripts/probe_so/libwgcsum_gso_p2w4s.so"}
for lib in $LIBS; do
  p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
  name=$(basename $lib .so)
  WGCS_LIB=$p timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gso.py tests/test_gpu_fullsize.py > $OUT/tests_$name.txt 2>&1 || { echo "tests $name rc=$?"; tail -5 $OUT/tests_$name.txt; exit 1; }
  echo "$name $(tail -1 $OUT/tests_$name.txt)"
done
TAG=${TAG:-r5_gso_p2}_ab LIBS="$LIBS" bash scripts/r5_gso_ab.sh 2 || exit 1
TAG=${TAG:-r5_gso_p2}_ab1 LIBS="$LIBS" BENCH_ARGS="--streams 1" bash scripts/r5_gso_ab.sh 2 || exit 1
