#!/bin/bash
# Round 4: non-temporal full-chunk stores (WGCS_STORE_NT probe build) with and
# without 128-B aligned output slots, cfg4, interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_gso_nt}; mkdir -p $OUT
L="scripts/probe_so/libwgcsum_base.so scripts/probe_so/libwgcsum_nt.so"
CFG=cfg4 ROUNDS=3 EXTRA="--gso-out-align 128 --gso-in-align 128" timeout -k 10 400 bash scripts/probe_lib_bench.sh $L > $OUT/aligned.jsonl || exit 1
CFG=cfg4 ROUNDS=3 timeout -k 10 400 bash scripts/probe_lib_bench.sh $L > $OUT/packed.jsonl || exit 1
python3 - $OUT <<'PY'
import json, sys, collections
for f in ("aligned", "packed"):
    d = collections.defaultdict(list)
    for l in open(f"{sys.argv[1]}/{f}.jsonl"):
        j = json.loads(l); r = j["line"]["roofline"]
        d[j["lib"]].append((round(r["kernel_ms"] * 1e3, 2), round(r.get("kernel_ms_one_stream", 0) * 1e3, 2)))
    for k, v in d.items():
        print(f, k, v)
PY
