#!/bin/bash
# Round-6 measurement set on a 1-GPU box (measurement script, NOT product
# code).  Parts (each fits one gpurun call):
#   tests  : the whole GPU suite + smoke
#   lines  : the driver's command (twice, plus no flags), one bench line per config
#   prof   : one-stream rocprofv3 --kernel-trace --stats of cfg2 at the driver's
#            count (20 + 5, twice) and at 200 + 20, cfg4, GRO, udp_split
#   sq     : SQ instruction counters of the checksum kernel and of a flat read of
#            the same bytes (scripts/probe_stream2.py)
#   pmc    : FETCH / WRITE / sized-read passes for udp_split (traffic.json)
#   gloo8  : the 8-rank line rehearsed as 8 gloo ranks sharing the GPU
# Every GPU step has its own time limit; a timeout, abort or fault stops the script.
# usage: TAG=r6_final bash scripts/r6_final.sh tests lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r6_final}
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
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
pmcrun() {  # name counters... -- python-args
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" --kernel-trace -d $OUT/$name -o run --output-format csv -- python3 "$@" > $OUT/$name.log 2>&1) || { echo "FAIL $name"; tail -5 $OUT/$name.log; exit 1; }
  echo "== $name ok"
}
want() { for a in "${ARGS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests lines)

if want tests; then
  step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if want lines; then
  line cfg2_noflags 300
  line cfg2_driver_a 300 --gpus 1 --steps 20 --warmup 5
  line cfg2_driver_b 300 --gpus 1 --steps 20 --warmup 5
  line cfg2 300 --steps 200 --warmup 20 --cpu-seconds 4 --no-strong
  line cfg3 300 --config cfg3 --steps 100 --warmup 10 --cpu-seconds 4
  line cfg5 300 --config cfg5 --steps 50 --warmup 5 --cpu-seconds 4
  line cfg4 300 --config cfg4 --steps 200 --warmup 20 --cpu-seconds 4
  line cfg4_1stream 300 --config cfg4 --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e
  line cfg1 300 --config cfg1 --steps 200 --warmup 20 --cpu-seconds 4
  line gro_device 300 --config gro_device --steps 40 --warmup 4 --cpu-seconds 3
  line gro_device_shuffled 300 --config gro_device --gro-shape shuffled --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e
  line gro_device_1x128 300 --config gro_device --gro-shape 1x128 --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e
  line gro_device_16x8 300 --config gro_device --gro-shape 16x8 --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e
  line udp_split 300 --config udp_split --steps 50 --warmup 5 --cpu-seconds 3
  line udp_coalesce 300 --config udp_coalesce --steps 50 --warmup 5 --cpu-seconds 3
fi
if want prof; then
  prof prof_cfg2_1s_20a --steps 20 --warmup 5 --streams 1 --no-strong
  prof prof_cfg2_1s_20b --steps 20 --warmup 5 --streams 1 --no-strong
  prof prof_cfg2_1s_200 --steps 200 --warmup 20 --streams 1 --no-strong
  prof prof_driver --gpus 1 --steps 20 --warmup 5 --no-strong
  prof prof_cfg4_1s_20 --config cfg4 --steps 20 --warmup 5 --streams 1
  prof prof_cfg4_1s_200 --config cfg4 --steps 200 --warmup 20 --streams 1
  prof prof_udp_split_1s --config udp_split --steps 50 --warmup 5 --streams 1
  prof prof_gro_shuffled_1s --config gro_device --gro-shape shuffled --steps 20 --warmup 2 --streams 1
fi
if want sq; then
  pmcrun sq_cfg2 $SQ -- $ROOT/bench.py --steps 45 --warmup 5 --streams 1 --no-strong --cpu-seconds 0 --no-e2e --no-event-timing
  pmcrun sq_flat $SQ -- $ROOT/scripts/probe_stream2.py
fi
if want pmc; then
  for p in "f:FETCH_SIZE" "w:WRITE_SIZE" "s:$SIZED"; do
    pmcrun pmc${p%%:*}_udpsplit ${p#*:} -- $ROOT/bench.py --config udp_split --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1
  done
fi
if want pmccs; then
  for p in "f:FETCH_SIZE" "w:WRITE_SIZE" "s:$SIZED"; do
    pmcrun pmc${p%%:*}_cfg2 ${p#*:} -- $ROOT/bench.py --steps 30 --warmup 3 --no-strong --cpu-seconds 0 --no-e2e --no-event-timing --streams 1
  done
fi
if want gloo8; then
  export WGCS_DIST_BACKEND=gloo
  step gloo8 600 python bench.py --gpus 8 --steps 20 --warmup 5
  unset WGCS_DIST_BACKEND
  grep '^{"metric"' "$OUT/gloo8.log" | tail -n 1 > "$OUT/rehearse_gpus8_gloo.jsonl"
fi
echo "== done"
