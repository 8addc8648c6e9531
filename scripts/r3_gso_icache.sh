#!/bin/bash
# Instruction-fetch counters of gso_rows_kernel (NOT product code): is the head
# waiting on the instruction cache at launch start? cfg4, one stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_gso_icache}; mkdir -p $OUT
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1); grep -o -E "SQC?_[A-Z_]*(IFETCH|ICACHE|INST_FETCH|_IC_)[A-Z_]*" $OUT/avail.txt | sort -u | head -20
for set in "${SETS[@]:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH}"; do :; done
C=$(grep -o -E "SQC?_[A-Z_]*(IFETCH|ICACHE)[A-Z_]*" $OUT/avail.txt | sort -u | head -4 | tr '\n' ' ')
echo "counters: $C"
[ -n "$C" ] || exit 0
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $C SQ_WAVES --kernel-trace -d $OUT/ic -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > $OUT/ic.log 2>&1) || { echo FAIL; tail -5 $OUT/ic.log; exit 1; }
python3 scripts/pmc_summary.py $OUT/ic | grep -A8 "wgcs::"
