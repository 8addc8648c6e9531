#!/bin/bash
# Round 6: the resident per-call ring -- parity first (alone, bounded), then
# GSO / checksum parity and the per-call latencies.  NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_ring}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/ring_tests.log 2>&1; rc=$?
tail -15 $OUT/ring_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/calls.jsonl 2>&1 || { tail -20 $OUT/calls.jsonl; exit 1; }
cat $OUT/calls.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_stager.py tests/test_gpu_checksum.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
echo done
