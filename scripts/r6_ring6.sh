#!/bin/bash
# Round 6: virtio reads whose header bytes travel inline with the request:
# ring + GSO parity, per-call latency inline vs pointer requests, stamps.  NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_ring6}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_gso.py tests/test_gpu_stager.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { tail -30 $OUT/tests.log; exit $rc; }
for r in 1 2; do
  for v in "inline:" "ptr:WGCS_RING_INLINE=0"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/calls_${name}_$r.jsonl 2>&1 || { tail -20 $OUT/calls_${name}_$r.jsonl; exit 1; }
  done
done
WGCS_LIB=$PWD/scripts/probe_so/libwgcsum_ringstamps.so timeout -k 10 120 python scripts/probe_ring_stamps.py > $OUT/stamps.jsonl 2>&1 || { tail -20 $OUT/stamps.jsonl; exit 1; }
for f in $OUT/calls_*.jsonl; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
h=d['handle_virtio_read']; c=d['checksum_valid']
print('$(basename $f)', {k:v['median_us'] for k,v in c.items()}, {k:v['median_us'] for k,v in h.items() if isinstance(v,dict)})
"; done
cat $OUT/stamps.jsonl
echo done
