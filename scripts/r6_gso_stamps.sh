#!/bin/bash
# Round 6: phase stamps of the staged GSO kernel against round 5's (NOT product code).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_gso_stamps}; mkdir -p $OUT
for v in "" _r5; do
  NWAVES=12 STAMPS_SO=scripts/probe_so/libwgcsum_gso_stamps$v.so timeout -k 10 120 python scripts/probe_gso_stamps.py run > $OUT/stamps$v.jsonl 2>&1 || exit 1
done
echo done
