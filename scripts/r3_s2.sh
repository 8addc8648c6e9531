#!/bin/bash
# Round-3 session 2: where the driver invocation's wall time goes.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r3_s2; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
for i in 1 2 3; do step rep$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e --repeat 6; done
(cd /tmp && step trace 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e)
for i in 1 2 3; do grep '^{' $OUT/rep$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['timing'])"; done
ls -R $OUT/trace | head
