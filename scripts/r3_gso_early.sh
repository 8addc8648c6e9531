#!/bin/bash
# GSO early payload loads: parity tests, phase stamps, A/B against the previous kernel (NOT product code).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r3_gso_early}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_stager.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 3 $OUT/tests.log; [ $rc = 0 ] || exit $rc
for v in gso_stamps2_e4:2 gso_stamps_e4:1; do
  lib=${v%%:*}; m=${v##*:}
  WGCS_LIB=scripts/probe_so/libwgcsum_$lib.so STAMPS=$m timeout -k 10 120 python scripts/probe_gso_stamps.py run > $OUT/st_$lib.jsonl 2>&1 || exit 1
  echo "== $lib"; grep probe $OUT/st_$lib.jsonl
done
TAG=${TAG:-r3_gso_early} ROUNDS=${ROUNDS:-3} CFGS=cfg4 LIBS="${LIBS:-libwgcsum_base.so libwgcsum_early4.so libwgcsum_early4_pre.so libwgcsum_early5.so}" bash scripts/r3_wt_ab.sh
