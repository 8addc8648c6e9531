#!/bin/bash
# Round 6: checksum kernel instruction cuts, A/B (NOT product code): the whole
# GPU suite on the product build, interleaved one-stream 200-step and
# driver-shaped lines per library, then per library rocprofv3 one-stream
# summaries at 45 and 420 launches and one SQ counter pass.
# usage: LIBS="libwgcsum.so scripts/probe_so/x.so" TAG=... bash scripts/r6_cs_ab2.sh [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
T=${TAG:-r6_cs_ab2}
OUT=$ROOT/gpurun_out/$T; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
REPS=${1:-3}
for rep in $(seq 1 $REPS); do
  for lib in ${LIBS}; do
    p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
    name=$(basename $lib .so)_$rep
    WGCS_LIB=$p timeout -k 10 120 python bench.py --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e --no-strong > $OUT/${name}_1s.log 2>&1 || { tail -5 $OUT/${name}_1s.log; exit 1; }
    grep '^{"metric"' $OUT/${name}_1s.log | sed "s/^{/{\"tag\": \"${name}_1s\", /" >> $OUT/lines.jsonl
    WGCS_LIB=$p timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e > $OUT/${name}_drv.log 2>&1 || { tail -5 $OUT/${name}_drv.log; exit 1; }
    grep '^{"metric"' $OUT/${name}_drv.log | sed "s/^{/{\"tag\": \"${name}_drv\", /" >> $OUT/lines.jsonl
  done
done
python3 - "$OUT/lines.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    one = r.get("kernel_ms_one_stream")
    print(f"{d['tag']:28s} value {d['value']:8.1f}  kernel {r['kernel_ms']*1e3:6.2f} us frac {r['frac']:.4f}" +
          (f"  1s {one*1e3:6.2f} us {r['frac_one_stream']:.4f}" if one else ""))
PY
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for lib in ${LIBS}; do
  p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
  name=$(basename $lib .so)
  for k in "45:--steps 20 --warmup 5" "420:--steps 200 --warmup 20"; do
    (cd /tmp && WGCS_LIB=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_${name}_${k%%:*} -o run --output-format csv -- python3 $ROOT/bench.py ${k#*:} --streams 1 --no-strong --cpu-seconds 0 --no-e2e > $OUT/prof_${name}_${k%%:*}.log 2>&1) || { echo "FAIL prof $name"; exit 1; }
    echo "prof $name ${k%%:*}: $(grep checksum_batch_kernel $OUT/prof_${name}_${k%%:*}/run_kernel_stats.csv | cut -d, -f2-6)"
  done
  (cd /tmp && WGCS_LIB=$p timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace -d $OUT/sq_$name -o run --output-format csv -- python3 $ROOT/bench.py --steps 45 --warmup 5 --streams 1 --no-strong --cpu-seconds 0 --no-e2e --no-event-timing > $OUT/sq_$name.log 2>&1) || { echo "FAIL sq $name"; exit 1; }
  python3 scripts/pmc_summary.py $OUT/sq_$name | grep -A9 checksum_batch
done
echo done
