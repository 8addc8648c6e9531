#!/bin/bash
# Round 6: ring parity + per-call latency with inline checksumValid requests,
# A/B against pointer requests (WGCS_RING_INLINE=0), and phase stamps.  NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_ring4}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/ring_tests.log 2>&1; rc=$?
tail -3 $OUT/ring_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/calls_inline_$r.jsonl 2>&1 || { tail -20 $OUT/calls_inline_$r.jsonl; exit 1; }
  WGCS_RING_INLINE=0 timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/calls_ptr_$r.jsonl 2>&1 || { tail -20 $OUT/calls_ptr_$r.jsonl; exit 1; }
done
WGCS_LIB=$PWD/scripts/probe_so/libwgcsum_ringstamps.so timeout -k 10 120 python scripts/probe_ring_stamps.py > $OUT/stamps.jsonl 2>&1 || { tail -20 $OUT/stamps.jsonl; exit 1; }
for f in $OUT/calls_*.jsonl $OUT/stamps.jsonl; do echo "$(basename $f) $(tail -1 $f | cut -c1-600)"; done
echo done
