#!/bin/bash
# Round 4 (late): FETCH_SIZE / WRITE_SIZE passes (separate runs) of
# gro_device, one stream, for the 4x32 and shuffled call shapes with the
# final GRO kernel.  scripts/pmc_traffic.py turns them into traffic.json records.
set -u
cd "$GRAFT_REPO_ROOT"
ROOT=$PWD
OUT=$PWD/gpurun_out/${TAG:-r4_gro_pmc}; mkdir -p $OUT
export TMPDIR=/tmp
for shape in ${SHAPES:-4x32 shuffled}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d "$OUT/${c}_$shape" -o run --output-format csv -- python3 "$ROOT/bench.py" --config gro_device --gro-shape $shape --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --streams 1 > "$OUT/${c}_$shape.log" 2>&1) || { echo "rc=$? $c $shape"; tail -5 "$OUT/${c}_$shape.log"; exit 1; }
    grep '^{' "$OUT/${c}_$shape.log" > "$OUT/${c}_${shape}_line.jsonl"
  done
done
echo done
