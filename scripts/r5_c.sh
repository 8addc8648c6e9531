#!/bin/bash
# Round 5: cfg4 launch-stream count A/B for gso_lds_kernel, and its SQ
# instruction counters on one stream (measurement script, NOT product code).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/r5_c; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for s in 2 3 4 6; do
    timeout -k 10 120 python bench.py --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e --streams $s > $OUT/s${s}_$rep.log 2>&1 || exit 1
    grep '^{"metric"' $OUT/s${s}_$rep.log | sed "s/^{/{\"tag\": \"s${s}_$rep\", /" >> $OUT/lines.jsonl
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:8s} {r['kernel_ms']*1e3:7.2f} us frac {r['frac']:.4f} value {d['value']}")
PY
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --kernel-trace -d $OUT/sq1 -o run --output-format csv -- python3 $ROOT/bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/sq1.log 2>&1) || { echo "FAIL sq1"; tail -5 $OUT/sq1.log; exit 1; }
python3 scripts/pmc_summary.py $OUT/sq1 | grep -A10 gso_
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM --kernel-trace -d $OUT/sq2 -o run --output-format csv -- python3 $ROOT/bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/sq2.log 2>&1) || { echo "FAIL sq2"; tail -5 $OUT/sq2.log; exit 1; }
python3 scripts/pmc_summary.py $OUT/sq2 | grep -A10 gso_
