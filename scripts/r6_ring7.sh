#!/bin/bash
# Round 6: ring A/B (four staggered polls in LDS-DMA slots, then 2-wave workgroups) against
# registers: ring + GSO parity, per-call latency A/B (interleaved), stamps.  NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_ring7}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_gso.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { tail -30 $OUT/tests.log; exit $rc; }
for r in 1 2; do
  for lib in libwgcsum.so ${ABLIB:-scripts/probe_so/libwgcsum_ring4w.so}; do
    p=$PWD/$lib; [ "$lib" = libwgcsum.so ] && p=$PWD/wireguard_amd/libwgcsum.so
    name=$(basename $lib .so)_$r
    WGCS_LIB=$p timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/calls_$name.jsonl 2>&1 || { tail -20 $OUT/calls_$name.jsonl; exit 1; }
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
