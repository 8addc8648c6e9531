#!/bin/bash
# SQ instruction counts of gso_rows_kernel per library build (NOT product code):
# whole kernel vs a head-only timing build, one stream, cfg4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_gso_sq}; mkdir -p $OUT
for lib in ${LIBS:-libwgcsum_base.so libwgcsum_headonly.so}; do
  (cd /tmp && WGCS_LIB=$GRAFT_REPO_ROOT/scripts/probe_so/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $OUT/$lib -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/$lib.log 2>&1) || { echo "FAIL $lib"; tail -5 $OUT/$lib.log; exit 1; }
  echo "== $lib"; python3 scripts/pmc_summary.py $OUT/$lib | grep -A9 gso_rows
done
