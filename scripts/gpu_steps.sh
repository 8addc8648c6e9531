#!/bin/bash
# Run GPU steps on the gpurun box.  Each step has its own time limit; a test
# failure does not stop the chain, but a timeout / abort / segfault does (no
# further GPU work after a fault).  Logs go under gpurun_out/.
# usage: scripts/gpu_steps.sh STEP...   STEP = tests | bench | prof | pmc | smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-r2}
step() {
  local name=$1 lim=$2; shift 2
  echo "== [$name] $(date +%T) $*"
  timeout -k 10 "$lim" "$@" > "$OUT/$TAG.$name.log" 2>&1
  local rc=$?
  echo "== [$name] rc=$rc"
  tail -n 5 "$OUT/$TAG.$name.log"
  case $rc in 124|134|137|139) echo "FATAL in $name (rc=$rc): stopping"; exit $rc;; esac
  return 0
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    tests-all) step tests 1100 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    tests-gso) step tests_gso 600 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_stager.py tests/test_gpu_fullsize.py tests/test_golden.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    tests-conn) step tests_conn 400 python -u -m pytest tests/test_gpu_conn.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    bench-usplit) step bench_usplit 300 python bench.py --config udp_split --steps 100 --warmup 10 --cpu-seconds 5 ;;
    bench-ucoal) step bench_ucoal 300 python bench.py --config udp_coalesce --steps 100 --warmup 10 --cpu-seconds 5 ;;
    prof-udp) (cd /tmp && step prof_usplit 300 rocprofv3 --kernel-trace --stats -d "$OUT/profusplit_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config udp_split --steps 50 --warmup 5 --cpu-seconds 0 --no-e2e) && (cd /tmp && step prof_ucoal 300 rocprofv3 --kernel-trace --stats -d "$OUT/profucoal_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config udp_coalesce --steps 50 --warmup 5 --cpu-seconds 0 --no-e2e) ;;
    sweep) step sweep 400 python scripts/sweep_checksum.py ;;
    probe-glds) step probe_glds 300 python scripts/probe_glds.py ;;
    probe-rows) step probe_rows 300 python scripts/probe_rows.py ;;
    sweep-align) step sweep_align 400 python scripts/sweep_checksum.py --variants 16:6:8:1:16,16:6:8:1:64,16:6:8:1:128,16:8:8:1:16,16:8:8:1:64,16:8:8:1:128 ;;
    sweep-cfg3) step sweep_cfg3 400 python scripts/sweep_checksum.py --config cfg3 ;;
    probe) step probe 400 python scripts/probe_stream.py ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 400 python bench.py --steps 200 --warmup 20 ;;
    bench-noevt) step bench_noevt 300 python bench.py --steps 200 --warmup 20 --no-event-timing --cpu-seconds 0 ;;
    bench-fill) step bench_fill 300 python bench.py --steps 200 --warmup 20 --mode fill --cpu-seconds 0 ;;
    bench-cfg3) step bench_cfg3 300 python bench.py --config cfg3 --steps 100 --warmup 10 --cpu-seconds 4 ;;
    bench-cfg4) step bench_cfg4 300 python bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 4 ;;
    bench-cfg4-1s) step bench_cfg4_1s 300 python bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --streams 1 ;;
    bench-gro) step bench_gro 300 python bench.py --config gro --steps 200 --warmup 20 --cpu-seconds 3 ;;
    bench-gro-staged) step bench_gros 300 python bench.py --config gro_staged --steps 30 --warmup 5 --cpu-seconds 3 ;;
    bench-cfg1) step bench_cfg1 300 python bench.py --config cfg1 --steps 200 --warmup 20 --cpu-seconds 5 ;;
    bench-driver) step bench_drv 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench-cfg5) step bench_cfg5 300 python bench.py --config cfg5 --steps 100 --warmup 10 --cpu-seconds 4 ;;
    prof) (cd /tmp && step prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e) ;;
    pmc) (cd /tmp && step pmc 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --cpu-seconds 0 --no-e2e --no-event-timing) ;;
    pmc-w) (cd /tmp && step pmcw 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --cpu-seconds 0 --no-e2e --no-event-timing) ;;
    prof-cfg4) (cd /tmp && step prof_cfg4 400 rocprofv3 --kernel-trace --stats -d "$OUT/profcfg4_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 50 --warmup 5 --cpu-seconds 0 --no-e2e) ;;
    pmc-gso) (cd /tmp && step pmcf_cfg4 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmcf_cfg4_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e) && (cd /tmp && step pmcw_cfg4 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_cfg4_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e) ;;
    pmc-cs) for c in "cfg2 --mode fill" "cfg3" "cfg5"; do t=$(echo $c | tr -d ' -'); (cd /tmp && step pmcf_$t 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmcf_${t}_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e --no-event-timing) && (cd /tmp && step pmcw_$t 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_${t}_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 30 --warmup 3 --cpu-seconds 0 --no-e2e --no-event-timing) || exit 1; done ;;
    pmc-udp) for c in udp_split udp_coalesce; do (cd /tmp && step pmcf_$c 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmcf_${c}_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 20 --warmup 3 --cpu-seconds 0 --no-e2e) && (cd /tmp && step pmcw_$c 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmcw_${c}_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 20 --warmup 3 --cpu-seconds 0 --no-e2e) || exit 1; done ;;
    pmc-sq-cfg4) (cd /tmp && step pmcsq_cfg4 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -d "$OUT/pmcsqcfg4_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 20 --warmup 2 --cpu-seconds 0) ;;
    pmc-sq2-cfg4) (cd /tmp && step pmcsq2_cfg4 400 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmcsq2cfg4_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --config cfg4 --steps 20 --warmup 2 --cpu-seconds 0) ;;
    pmc-sq) (cd /tmp && step pmcsq 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-trace -d "$OUT/pmcsq_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --cpu-seconds 0) ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done"
