#!/bin/bash
# Round 5: GSO parity with the LDS-staged kernel (gso_lds_kernel), then an
# interleaved A/B of cfg4 against the round-4 grid (WGCS_GSO_KERNEL=rows) on
# the bench default (4 streams) and one stream, and rocprofv3 one-stream stats
# of both.  usage: TAG=r5_gso bash scripts/r5_gso.sh [notests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r5_gso}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== [$name] $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(tail -n 1 "$OUT/$name.log" | cut -c1-200)"
  case $rc in 124|134|137|139) echo "FATAL in $name (rc=$rc): stopping"; exit $rc;; esac
  [ "$name" = tests ] && [ $rc -ne 0 ] && { echo "tests failed: stopping"; exit 1; }
  return 0
}
line() {  # name limit bench-args...
  local name=$1 lim=$2; shift 2
  step "$name" "$lim" python bench.py "$@"
  grep '^{"metric"' "$OUT/$name.log" | tail -n 1 | sed "s/^{/{\"tag\": \"$name\", /" >> "$OUT/lines.jsonl"
}
if [ "${1:-}" != notests ]; then
  step tests 600 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_fullsize.py tests/test_gpu_stager.py tests/test_gpu_c_harness.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
fi
for rep in 1 2; do
  line cfg4_lds_$rep 240 --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e
  export WGCS_GSO_KERNEL=rows
  line cfg4_rows_$rep 240 --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e
  unset WGCS_GSO_KERNEL
done
(cd /tmp && step prof_lds_1s 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_lds_1s" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e --streams 1)
export WGCS_GSO_KERNEL=rows
(cd /tmp && step prof_rows_1s 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rows_1s" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e --streams 1)
echo "== done"
