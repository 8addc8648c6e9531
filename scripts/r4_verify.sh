#!/bin/bash
# Round 4: parity of the changed paths first, the whole GPU suite, smoke, then
# the cfg2 frame-stride probe and the flat-stream probe (one and two streams).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_verify}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc $(tail -n 1 $OUT/$n.log | cut -c1-200)"; [ $rc -ne 0 ] && exit $rc; return 0; }
step changed 400 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_checksum.py tests/test_gpu_stager.py tests/test_gpu_gro_batch.py tests/test_gpu_gro.py tests/test_gpu_wstager.py -x -q --timeout 120 --timeout-method thread
step suite 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step stride 600 bash scripts/r4_cfg2_stride.sh
step stream2 300 python scripts/probe_stream2.py
