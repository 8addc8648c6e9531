#!/bin/bash
# Round 4: gro_batch_kernel phase timeline per call shape (timing-only build), and the
# gro_device bench line for every shape.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_gro}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc $(tail -n 1 $OUT/$n.log | cut -c1-200)"; case $rc in 124|134|137|139) exit $rc;; esac; return $rc; }
WGCS_LIB_PARTIAL=1 step phases 300 python scripts/probe_gro_phases.py || exit 1
cat $OUT/phases.log
for s in ${SHAPES:-4x32 shuffled 1x128}; do
  step line_$s 200 python bench.py --config gro_device --gro-shape $s --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e || exit 1
  grep '^{' $OUT/line_$s.log | cut -c1-400
done
