#!/bin/bash
# Round-3 session 1: Go probe, targeted GPU tests, the driver's bench line x3.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r3_s1; mkdir -p $OUT
bash scripts/r3_probe_go.sh gpurun_out/r3_go_probe.txt
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc"; tail -n 3 $OUT/$n.log | cut -c1-400; case $rc in 124|134|137|139) exit $rc;; esac; }
step tests 600 python -u -m pytest tests/test_gpu_wstager.py tests/test_bench_launcher.py tests/test_gpu_checksum.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for i in 1 2 3; do step drv$i 120 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e; done
step drvfull 200 python bench.py --gpus 1 --steps 20 --warmup 5
