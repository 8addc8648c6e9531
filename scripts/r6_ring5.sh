#!/bin/bash
# Round 6: why virtio reads run ~1 us slower after inline checksum requests:
# virtio-only runs, and inline requests whose payload lines the host flushes
# after each call (WGCS_RING_FLUSH=1).  NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_ring5}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/ring_tests.log 2>&1; rc=$?
tail -1 $OUT/ring_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "inline:" "ptr:WGCS_RING_INLINE=0" "skip:PROBE_SKIP_CS=1" "flush:WGCS_RING_FLUSH=1"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/calls_${name}_$r.jsonl 2>&1 || { tail -20 $OUT/calls_${name}_$r.jsonl; exit 1; }
  done
done
for f in $OUT/calls_*.jsonl; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
h=d['handle_virtio_read']; c=d['checksum_valid']
print('$(basename $f)', {k:v['median_us'] for k,v in c.items()}, {k:v['median_us'] for k,v in h.items() if isinstance(v,dict)})
"; done
echo done
