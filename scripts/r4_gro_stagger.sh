#!/bin/bash
# Round 4 probe: gro_batch_kernel with its odd calls started 20 / 40 / 80 us
# late (timing-only -DWGCS_GRO_STAGGER builds), so the calls' memory and LDS
# phases do not line up, against the kept kernel; 4x32 and shuffled.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_gro_stagger}; mkdir -p $OUT
L="scripts/probe_so/libwgcsum_base.so scripts/probe_so/libwgcsum_stag20.so scripts/probe_so/libwgcsum_stag40.so scripts/probe_so/libwgcsum_stag80.so"
CFG=gro_device ROUNDS=2 EXTRA="--gro-shape 4x32" timeout -k 10 400 bash scripts/probe_lib_bench.sh $L > $OUT/4x32.jsonl || exit 1
CFG=gro_device ROUNDS=2 EXTRA="--gro-shape shuffled" timeout -k 10 400 bash scripts/probe_lib_bench.sh $L > $OUT/shuffled.jsonl || exit 1
python3 - $OUT <<'PY'
import json, sys
for f in ("4x32", "shuffled"):
    for l in open(f"{sys.argv[1]}/{f}.jsonl"):
        j = json.loads(l); r = j["line"]["roofline"]
        print(f, j["lib"], j["round"], r["kernel_ms"], r["frac"])
PY
