#!/bin/bash
# cfg2 launch knobs incl. 16 lanes per frame (NOT product code): two interleaved rounds,
# two-stream HIP-event time per launch and the one-stream reference; then SQ counts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_sweep_g16}; mkdir -p $OUT
for rep in 1 2; do
for v in ${VARIANTS:-"16 4 32" "8 6 16" "16 6 16" "8 8 16" "16 4 16" "24 6 16" "12 6 16"}; do
  set -- $v
  WGCS_BLOCKS_PER_CU=$1 WGCS_UNROLL=$2 WGCS_LANES_PER_PKT=$3 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e > $OUT/sw.log 2>&1 || exit 1
  line="bpc=$1 U=$2 G=$3 $(grep -o '"kernel_ms": [0-9.]*' $OUT/sw.log) $(grep -o '"frac": [0-9.]*' $OUT/sw.log | head -1) $(grep -o '"kernel_ms_one_stream": [0-9.]*' $OUT/sw.log)"
  echo "$line"; echo "$line" >> $OUT/sweep.txt
done; done
for v in "16 4 32" "8 6 16"; do
  set -- $v
  (cd /tmp && WGCS_BLOCKS_PER_CU=$1 WGCS_UNROLL=$2 WGCS_LANES_PER_PKT=$3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $OUT/sq_$1_$2_$3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/sq_$1_$2_$3.log 2>&1) || exit 1
  echo "== sq $v"; python3 scripts/pmc_summary.py $OUT/sq_$1_$2_$3 | grep -A7 "wgcs::" | grep -E "wgcs|SALU|VALU|WAVES"
done
