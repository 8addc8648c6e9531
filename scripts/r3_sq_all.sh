#!/bin/bash
# SQ instruction counts per kernel for the other bench lines (NOT product code).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_sq_all}; mkdir -p $OUT
for c in ${CFGS:-udp_coalesce udp_split gro_device cfg2}; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $OUT/$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/$c.log 2>&1) || { echo "FAIL $c"; tail -5 $OUT/$c.log; exit 1; }
  echo "== $c"; python3 scripts/pmc_summary.py $OUT/$c | grep -v -i "elementwise\|vectorized\|fill" | head -24
done
