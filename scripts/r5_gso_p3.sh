#!/bin/bash
# Round 5: GSO P = 3 x 4 waves (scalar head) against P = 1 x 8 waves --
# three interleaved reps on four streams and one, and the L2's sized reads +
# WRITE_SIZE for both.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_gso_p3}; mkdir -p $OUT
export TMPDIR=/tmp
LIBS=${LIBS:-"libwgcsum.so scripts/probe_so/libwgcsum_gso_p3w4s.so"}
TAG=${TAG:-r5_gso_p3}_ab LIBS="$LIBS" bash scripts/r5_gso_ab.sh 3 || exit 1
TAG=${TAG:-r5_gso_p3}_ab1 LIBS="$LIBS" BENCH_ARGS="--streams 1" bash scripts/r5_gso_ab.sh 2 || exit 1
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
for lib in $LIBS; do
  p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
  name=$(basename $lib .so)
  for c in sized WRITE_SIZE; do
    ctr=$c; [ $c = sized ] && ctr=$SIZED
    (cd /tmp && WGCS_LIB=$p timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/pmc_${name}_$c -o run --output-format csv -- python3 $ROOT/bench.py --config cfg4 --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1 > $OUT/pmc_${name}_$c.log 2>&1) || { echo "FAIL pmc $name $c"; exit 1; }
  done
  echo "== $name $(python3 scripts/pmc_sized.py $OUT/pmc_${name}_sized gso_lds | cut -c150-400)"
done
