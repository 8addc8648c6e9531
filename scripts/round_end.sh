#!/bin/bash
# Round-end measurement set on a 1-GPU box: GPU tests, smoke, one bench line
# per config (JSON lines appended to gpurun_out/$TAG/lines.jsonl) and
# rocprofv3 kernel-trace/stats + FETCH_SIZE/WRITE_SIZE passes for the
# headline and GSO kernels.  Every GPU step has its own time limit; a timeout,
# abort or fault stops the script (no further GPU work after it).
# usage: TAG=r2_end scripts/round_end.sh [tests] [lines] [prof] [pmc]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r2_end}
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
want() { for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests lines prof pmc)

if want tests; then
  step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if want lines; then
  line cfg2_driver 300 --gpus 1 --steps 20 --warmup 5
  line cfg2 300 --steps 200 --warmup 20 --cpu-seconds 4 --no-strong
  line cfg2_fill 300 --steps 200 --warmup 20 --mode fill --cpu-seconds 0 --no-e2e --no-strong
  line cfg2_1stream 300 --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e --no-strong
  line cfg3 300 --config cfg3 --steps 100 --warmup 10 --cpu-seconds 4
  line cfg5 300 --config cfg5 --steps 50 --warmup 5 --cpu-seconds 4
  line cfg4 300 --config cfg4 --steps 100 --warmup 10 --cpu-seconds 4
  line cfg4_64slots 300 --config cfg4 --max-segs 64 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e
  line cfg1 300 --config cfg1 --steps 200 --warmup 20 --cpu-seconds 4
  line gro 300 --config gro --steps 200 --warmup 20 --cpu-seconds 3
  line gro_staged 300 --config gro_staged --steps 30 --warmup 5 --cpu-seconds 3
  line gro_device 300 --config gro_device --steps 40 --warmup 4 --cpu-seconds 3
  line gro_device_1x128 300 --config gro_device --gro-shape 1x128 --steps 40 --warmup 4 --cpu-seconds 0
  line gro_device_4x32rev 300 --config gro_device --gro-shape 4x32rev --steps 20 --warmup 2 --cpu-seconds 0
  line gro_device_shuffled 300 --config gro_device --gro-shape shuffled --steps 40 --warmup 4 --cpu-seconds 0
  line udp_split 300 --config udp_split --steps 50 --warmup 5 --cpu-seconds 3
  line udp_coalesce 300 --config udp_coalesce --steps 50 --warmup 5 --cpu-seconds 3
fi
if want prof; then
  (cd /tmp && step prof_driver 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_driver" -o run --output-format csv -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e --no-strong)
  python3 scripts/trace_span.py "$OUT/prof_driver/run_kernel_trace.csv" checksum_batch 20 20 | sed "s/^{/{\"run\": \"prof_driver\", /" >> "$OUT/trace_span.jsonl"
  (cd /tmp && step prof_cfg2 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg2" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e --no-strong)
  (cd /tmp && step prof_cfg2_1s 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg2_1s" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e --streams 1 --no-strong)
  (cd /tmp && step prof_cfg4 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg4" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e)
  (cd /tmp && step prof_gro_shuffled 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_gro_shuffled" -o run --output-format csv -- python3 "$ROOT/bench.py" --config gro_device --gro-shape shuffled --steps 20 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1)
  (cd /tmp && step prof_cfg4_1s 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_cfg4_1s" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e --streams 1)
  for d in prof_cfg2 prof_cfg2_1s prof_cfg4 prof_cfg4_1s; do
    k=checksum_batch; case $d in prof_cfg4*) k=gso_rows;; esac
    python3 scripts/trace_span.py "$OUT/$d/run_kernel_trace.csv" $k 50 20 | sed "s/^{/{\"run\": \"$d\", /" >> "$OUT/trace_span.jsonl"
  done
fi
if want pmc; then
  (cd /tmp && step pmcf_cfg2 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmcf_cfg2" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1 --no-strong)
  (cd /tmp && step pmcw_cfg2 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_cfg2" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1 --no-strong)
  (cd /tmp && step pmcf_cfg4 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmcf_cfg4" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1)
  (cd /tmp && step pmcw_cfg4 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_cfg4" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1)
  (cd /tmp && step pmcf_gro_shuffled 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmcf_gro_shuffled" -o run --output-format csv -- python3 "$ROOT/bench.py" --config gro_device --gro-shape shuffled --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1)
  (cd /tmp && step pmcw_gro_shuffled 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_gro_shuffled" -o run --output-format csv -- python3 "$ROOT/bench.py" --config gro_device --gro-shape shuffled --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1)
fi
echo "== done"
