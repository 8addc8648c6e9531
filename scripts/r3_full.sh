#!/bin/bash
# Full GPU suite + smoke + the driver's bench line + a 2-rank gloo rehearsal of --gpus 2.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_full}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc"; tail -n 2 $OUT/$n.log | cut -c1-400; case $rc in 124|134|137|139) exit $rc;; esac; }
step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step drv 200 python bench.py --gpus 1 --steps 20 --warmup 5
step gpus2 300 env WGCS_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 0
