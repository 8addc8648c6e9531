#!/bin/bash
# Round 5, first box: the GPU suite on the tree with the round's first fixes,
# smoke, the driver's cfg2 line (doorbell on every stream, ungated wall time
# beside it) and the same line with --no-event-timing on two streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r5_a}
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
  return 0
}
line() {  # name limit bench-args...
  local name=$1 lim=$2; shift 2
  step "$name" "$lim" python bench.py "$@"
  grep '^{"metric"' "$OUT/$name.log" | tail -n 1 | sed "s/^{/{\"tag\": \"$name\", /" >> "$OUT/lines.jsonl"
}
step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
line cfg2_driver 300 --gpus 1 --steps 20 --warmup 5
line cfg2_noev 300 --gpus 1 --steps 20 --warmup 5 --no-event-timing --cpu-seconds 0 --no-e2e --no-strong
line cfg4 300 --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e
echo "== done"
