#!/bin/bash
# Ring round-trip probe (NOT product code): scripts/probe_ring.hip
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_ring_probe}; mkdir -p $OUT
for nb in 1 4; do
  timeout -k 5 60 ./scripts/probe_so/probe_ring $nb 1 >> $OUT/ring.jsonl 2>&1 || exit 1
done
timeout -k 5 60 ./scripts/probe_so/probe_ring 4 0 >> $OUT/ring.jsonl 2>&1 || exit 1
echo done
