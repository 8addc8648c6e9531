#!/bin/bash
# Ring round-trip probe variants (NOT product code): scripts/probe_ring.hip
# args: blocks, variant (0 host-memory record, 1 device-memory record), loads (0 sc0sc1, 1 inv sc0, 2 inv sc1, 3 plain)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_ring_probe3}; mkdir -p $OUT
for a in "1 0 0" "3 0 0" "8 0 0"; do
  timeout -k 5 60 ./scripts/probe_so/probe_ring $a > $OUT/p.txt 2>&1; rc=$?; grep '"ring"' $OUT/p.txt >> $OUT/all.jsonl; [ $rc -eq 0 ] || { cat $OUT/p.txt; exit $rc; }
done
cat $OUT/all.jsonl
echo done
