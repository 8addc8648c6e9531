#!/bin/bash
# Round 4: FETCH_SIZE / WRITE_SIZE passes for cfg5 (BASELINE configs[4], the
# 1M mixed batch; the strong block's kernel), one stream.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_pmc_cfg5}; mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $OUT/$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1 > $OUT/$c.log 2>&1) || { tail -5 $OUT/$c.log; exit 1; }
done
echo done
