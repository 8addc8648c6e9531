#!/bin/bash
# Round 6: ring parity + per-call latency, product vs a no-fence timing build (NOT product code)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_ring3}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/ring_tests.log 2>&1; rc=$?
tail -3 $OUT/ring_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/calls.jsonl 2>&1 || { tail -20 $OUT/calls.jsonl; exit 1; }
WGCS_LIB=$PWD/scripts/probe_so/libwgcsum_ringnofence.so timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/calls_nofence.jsonl 2>&1 || { tail -20 $OUT/calls_nofence.jsonl; exit 1; }
cat $OUT/calls.jsonl $OUT/calls_nofence.jsonl
echo done
