#!/bin/bash
# Round 4 probe: the first group's first 2 / 3 / 4 / 6 payload windows issued
# before the job sums (-DWGCS_GSO_EARLY), on the final cfg4 setup (four
# streams, slots on lines) and one stream; parity of each variant first.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_gso_early}; mkdir -p $OUT
L="scripts/probe_so/libwgcsum_base.so scripts/probe_so/libwgcsum_e2.so scripts/probe_so/libwgcsum_e3.so scripts/probe_so/libwgcsum_e4.so scripts/probe_so/libwgcsum_e6.so"
for v in e2 e3 e4 e6; do
  WGCS_LIB=scripts/probe_so/libwgcsum_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_fullsize.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/par_$v.log 2>&1 || { tail -3 $OUT/par_$v.log; exit 1; }
  tail -1 $OUT/par_$v.log
done
CFG=cfg4 ROUNDS=3 timeout -k 10 600 bash scripts/probe_lib_bench.sh $L > $OUT/ab.jsonl || exit 1
python3 - $OUT/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); r = j["line"]["roofline"]
    d[j["lib"]].append((round(r["kernel_ms"] * 1e3, 2), round(r.get("kernel_ms_one_stream", 0) * 1e3, 2)))
for k, v in d.items():
    print(k, v)
PY
