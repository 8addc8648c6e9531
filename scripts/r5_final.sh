#!/bin/bash
# Round-5 end measurement set on a 1-GPU box (measurement script, NOT product
# code): GPU tests + smoke, the driver's command twice, one bench line per
# config, rocprofv3 kernel-trace/stats summaries, and (pmc) three PMC passes
# per config -- FETCH_SIZE, WRITE_SIZE, the L2's sized read requests
# (scripts/pmc_sized.py) -- for profiles/traffic.json.  Every GPU step has its
# own time limit; a timeout, abort or fault stops the script.
# usage: TAG=r5_final bash scripts/r5_final.sh [tests] [lines] [prof] [pmc]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r5_final}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== [$name] $(date +%T)"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(tail -n 1 "$OUT/$name.log" | cut -c1-200)"
  case $rc in 0|1) ;; *) echo "FATAL in $name (rc=$rc): stopping"; exit $rc;; esac
  return 0
}
line() {  # name limit bench-args...
  local name=$1 lim=$2; shift 2
  step "$name" "$lim" python bench.py "$@"
  grep '^{"metric"' "$OUT/$name.log" | tail -n 1 | sed "s/^{/{\"tag\": \"$name\", /" >> "$OUT/lines.jsonl"
}
prof() {  # name bench-args...
  local name=$1; shift
  (cd /tmp && step "$name" 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/bench.py" "$@" --cpu-seconds 0 --no-e2e)
}
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
pass() {  # name counters... -- bench args
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" --kernel-trace -d $OUT/$name -o run --output-format csv -- python3 $ROOT/bench.py "$@" --cpu-seconds 0 --no-e2e --no-event-timing --streams 1 > $OUT/$name.log 2>&1) || { echo "FAIL $name"; tail -5 $OUT/$name.log; exit 1; }
  echo "== $name ok"
}
cfg() {  # tag bench-args...
  local t=$1; shift
  pass pmcf_$t FETCH_SIZE -- "$@"
  pass pmcw_$t WRITE_SIZE -- "$@"
  pass pmcs_$t $SIZED -- "$@"
}
want() { for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests lines prof)

if want tests; then
  step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if want lines; then
  line cfg2_driver_a 300 --gpus 1 --steps 20 --warmup 5
  line cfg2_driver_b 300 --gpus 1 --steps 20 --warmup 5
  line cfg2 300 --steps 200 --warmup 20 --cpu-seconds 4 --no-strong
  line cfg2_fill 300 --steps 200 --warmup 20 --mode fill --cpu-seconds 0 --no-e2e --no-strong
  line cfg3 300 --config cfg3 --steps 100 --warmup 10 --cpu-seconds 4
  line cfg5 300 --config cfg5 --steps 50 --warmup 5 --cpu-seconds 4
  line cfg4 300 --config cfg4 --steps 200 --warmup 20 --cpu-seconds 4
  line cfg4_1stream 300 --config cfg4 --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e
  line cfg1 300 --config cfg1 --steps 200 --warmup 20 --cpu-seconds 4
  line gro 300 --config gro --steps 200 --warmup 20 --cpu-seconds 3
  line gro_staged 300 --config gro_staged --steps 30 --warmup 5 --cpu-seconds 3
  line gro_device 300 --config gro_device --steps 40 --warmup 4 --cpu-seconds 3
  line gro_device_1x128 300 --config gro_device --gro-shape 1x128 --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e
  line gro_device_shuffled 300 --config gro_device --gro-shape shuffled --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e
  line gro_device_4x32rev 300 --config gro_device --gro-shape 4x32rev --steps 20 --warmup 2 --cpu-seconds 0 --no-e2e
  line gro_device_16x8 300 --config gro_device --gro-shape 16x8 --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e
  line gro_device_1x128udp 300 --config gro_device --gro-shape 1x128udp --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e
  line udp_split 300 --config udp_split --steps 50 --warmup 5 --cpu-seconds 3
  line udp_coalesce 300 --config udp_coalesce --steps 50 --warmup 5 --cpu-seconds 3
fi
if want prof; then
  prof prof_driver --gpus 1 --steps 20 --warmup 5 --no-strong
  prof prof_cfg2_1s --steps 200 --warmup 20 --streams 1 --no-strong
  prof prof_cfg5_1s --config cfg5 --steps 20 --warmup 5 --streams 1
  prof prof_cfg4 --config cfg4 --steps 200 --warmup 20
  prof prof_cfg4_1s --config cfg4 --steps 200 --warmup 20 --streams 1
  prof prof_gro_4x32_1s --config gro_device --gro-shape 4x32 --steps 20 --warmup 2 --streams 1
  prof prof_gro_shuffled_1s --config gro_device --gro-shape shuffled --steps 20 --warmup 2 --streams 1
  python3 scripts/trace_span.py "$OUT/prof_driver/run_kernel_trace.csv" checksum_batch 20 20 | sed "s/^{/{\"run\": \"prof_driver\", /" >> "$OUT/trace_span.jsonl"
  python3 scripts/trace_span.py "$OUT/prof_cfg4/run_kernel_trace.csv" gso_lds 50 20 | sed "s/^{/{\"run\": \"prof_cfg4\", /" >> "$OUT/trace_span.jsonl"
fi
if want pmc; then
  cfg cfg2 --steps 30 --warmup 3 --no-strong
  cfg cfg2fill --steps 30 --warmup 3 --no-strong --mode fill
  cfg cfg3 --config cfg3 --steps 20 --warmup 2
  cfg cfg5 --config cfg5 --steps 10 --warmup 2 --warm-ms 0
  cfg cfg4 --config cfg4 --steps 30 --warmup 3
  cfg gro4x32 --config gro_device --gro-shape 4x32 --steps 10 --warmup 2
  cfg gro1x128 --config gro_device --gro-shape 1x128 --steps 10 --warmup 2
  cfg groshuf --config gro_device --gro-shape shuffled --steps 10 --warmup 2
  cfg udpsplit --config udp_split --steps 10 --warmup 2
  cfg udpcoal --config udp_coalesce --steps 10 --warmup 2
fi
echo "== done"
