#!/bin/bash
# Round 5: SQ counters of gro_batch_kernel per call shape (measurement
# script, NOT product code): instruction mix and LDS waits, one stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_gro_sq}; mkdir -p $OUT
export TMPDIR=/tmp
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH"
C2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_ANY"
for shape in 4x32 shuffled; do
  for set in 1 2; do
    ctr=$C1; [ $set = 2 ] && ctr=$C2
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/${shape}_$set -o run --output-format csv -- python3 $ROOT/bench.py --config gro_device --gro-shape $shape --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/${shape}_$set.log 2>&1) || { echo "FAIL $shape $set"; tail -5 $OUT/${shape}_$set.log; exit 1; }
  done
done
python3 - $OUT <<'PY'
import csv, glob, sys, statistics
out = sys.argv[1]
for shape in ("4x32", "shuffled"):
    vals = {}
    for s in (1, 2):
        for f in glob.glob(f"{out}/{shape}_{s}/**/run_counter_collection.csv", recursive=True):
            per = {}
            for r in csv.DictReader(open(f)):
                if "gro_batch" not in r["Kernel_Name"]:
                    continue
                per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            for k, d in per.items():
                vals[k] = statistics.median(d.values())
    print(shape, {k: round(v) for k, v in sorted(vals.items())})
PY
