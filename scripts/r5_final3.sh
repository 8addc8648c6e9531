#!/bin/bash
# Round-5 close-out on the final tree: the whole GPU suite + smoke, the
# driver's command twice, the cfg4 line, and one-stream rocprofv3 summaries of
# cfg2 and cfg4 at the driver's step count (20 + 5: inside the first ~2 ms of
# load, before the shader clock's dip) and at 200 + 20 (across it).
# Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r5_final3}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  echo "== [$name] $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(tail -n 1 "$OUT/$name.log" | cut -c1-200)"
  case $rc in 0|1) ;; *) echo "FATAL in $name (rc=$rc): stopping"; exit $rc;; esac
}
line() {
  local name=$1 lim=$2; shift 2
  step "$name" "$lim" python bench.py "$@"
  grep '^{"metric"' "$OUT/$name.log" | tail -n 1 | sed "s/^{/{\"tag\": \"$name\", /" >> "$OUT/lines.jsonl"
}
prof() {
  local name=$1; shift
  (cd /tmp && step "$name" 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/bench.py" "$@" --cpu-seconds 0 --no-e2e)
}
step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
line cfg2_driver_a 300 --gpus 1 --steps 20 --warmup 5
line cfg2_driver_b 300 --gpus 1 --steps 20 --warmup 5
line cfg4 300 --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e
prof prof_cfg2_1s_20a --steps 20 --warmup 5 --streams 1 --no-strong
prof prof_cfg2_1s_20b --steps 20 --warmup 5 --streams 1 --no-strong
prof prof_cfg2_1s_200 --steps 200 --warmup 20 --streams 1 --no-strong
prof prof_cfg4_1s_20 --config cfg4 --steps 20 --warmup 5 --streams 1
prof prof_cfg4_1s_200 --config cfg4 --steps 200 --warmup 20 --streams 1
echo "== done"
