#!/bin/bash
# Round 5: HBM traffic per launch (measurement script, NOT product code).
# For each config, three rocprofv3 passes of the same one-stream bench command:
# FETCH_SIZE, WRITE_SIZE, and the L2's sized read requests
# (TCC_EA0_RDREQ{,_128B,_64B,_32B}_sum, scripts/pmc_sized.py); first the
# calibration probe under the sized counters.
# usage: TAG=r5_pmc bash scripts/r5_pmc.sh [cal] [cfg2] [cfg3] [cfg5] [cfg4] [gro4x32] [groshuf]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r5_pmc}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
pass() {  # name counters... -- bench args
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" --kernel-trace -d $OUT/$name -o run --output-format csv -- python3 "$@" > $OUT/$name.log 2>&1) || { echo "FAIL $name"; tail -5 $OUT/$name.log; exit 1; }
  echo "== $name ok"
}
cfg() {  # tag bench-args...
  local t=$1; shift
  pass ${t}_fetch FETCH_SIZE -- $ROOT/bench.py "$@" --cpu-seconds 0 --no-e2e --no-event-timing --streams 1
  pass ${t}_write WRITE_SIZE -- $ROOT/bench.py "$@" --cpu-seconds 0 --no-e2e --no-event-timing --streams 1
  pass ${t}_sized $SIZED -- $ROOT/bench.py "$@" --cpu-seconds 0 --no-e2e --no-event-timing --streams 1
}
want() { [ $# -eq 0 ] && return 0; for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(cal cfg2 cfg3 cfg5 cfg4 gro4x32 groshuf)
if want cal; then
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $SIZED --kernel-trace -d $OUT/cal -o run --output-format csv -- python3 $ROOT/scripts/probe_fetch_cal.py > $OUT/cal.log 2>&1) || { echo "FAIL cal"; tail -5 $OUT/cal.log; exit 1; }
  python3 scripts/pmc_sized.py cal $OUT/cal $OUT/cal.log | tee $OUT/cal_summary.json
fi
want cfg2 && cfg cfg2 --steps 30 --warmup 3 --no-strong
want cfg3 && cfg cfg3 --config cfg3 --steps 20 --warmup 2
want cfg5 && cfg cfg5 --config cfg5 --steps 10 --warmup 2
want cfg4 && cfg cfg4 --config cfg4 --steps 30 --warmup 3
want gro4x32 && cfg gro4x32 --config gro_device --gro-shape 4x32 --steps 10 --warmup 2
want groshuf && cfg groshuf --config gro_device --gro-shape shuffled --steps 10 --warmup 2
want udpsplit && cfg udpsplit --config udp_split --steps 10 --warmup 2
for d in $OUT/*_sized; do echo "== $(basename $d)"; python3 scripts/pmc_sized.py $d | cut -c1-400; done
echo "== done"
