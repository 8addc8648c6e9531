#!/bin/bash
# Where the GSO waves' cycles go (NOT product code): issue-stall vs wait vs active
# quad-cycles, whole kernel and head-only timing build, one stream, cfg4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_gso_sq_wait}; mkdir -p $OUT
for lib in ${LIBS:-libwgcsum_s3.so libwgcsum_s3_headonly.so}; do
  (cd /tmp && WGCS_LIB=$GRAFT_REPO_ROOT/scripts/probe_so/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU --kernel-trace -d $OUT/$lib -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/$lib.log 2>&1) || { echo "FAIL $lib"; tail -5 $OUT/$lib.log; exit 1; }
  echo "== $lib"; python3 scripts/pmc_summary.py $OUT/$lib | grep -A9 gso_rows
done
