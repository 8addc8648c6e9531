#!/bin/bash
# Round 5: checksum waves on contiguous frame runs -- parity at the default
# one-pass grid and at a 1-block-per-CU grid (every wave walks a long run),
# then grid A/B per config with the L2's sized read requests (r5_cfg5_traffic.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_cs_contig}; mkdir -p $OUT
export TMPDIR=/tmp
T="tests/test_gpu_checksum.py tests/test_gpu_batches.py tests/test_gpu_fullsize.py"
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu $T > $OUT/tests_default.txt 2>&1 \
  || { echo "tests rc=$?"; tail -20 $OUT/tests_default.txt; exit 1; }
tail -1 $OUT/tests_default.txt
WGCS_BLOCKS_PER_CU=1 timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu $T > $OUT/tests_bpc1.txt 2>&1 \
  || { echo "tests bpc1 rc=$?"; tail -20 $OUT/tests_bpc1.txt; exit 1; }
tail -1 $OUT/tests_bpc1.txt
TAG=${TAG:-r5_cs_contig} bash scripts/r5_cfg5_traffic.sh
