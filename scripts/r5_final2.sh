#!/bin/bash
# Round-5 end, after the GSO launch-shape change: the whole GPU suite + smoke
# on the final tree, the cfg4 lines (four streams, one), rocprofv3 summaries of
# cfg4, and the driver's command once more.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r5_final2}
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
step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
line cfg4 300 --config cfg4 --steps 200 --warmup 20 --cpu-seconds 4
line cfg4_b 300 --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e
line cfg4_1stream 300 --config cfg4 --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e
line cfg2_driver 300 --gpus 1 --steps 20 --warmup 5
(cd /tmp && step prof_cfg4 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg4" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e)
(cd /tmp && step prof_cfg4_1s 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg4_1s" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e)
python3 scripts/trace_span.py "$OUT/prof_cfg4/run_kernel_trace.csv" gso_lds 50 20 | sed "s/^{/{\"run\": \"prof_cfg4\", /" >> "$OUT/trace_span.jsonl"
echo "== done"
