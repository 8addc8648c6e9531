#!/bin/bash
# Round 5: cfg4 (GSO, gso_lds_kernel) by stream count -- is the 4-stream rate
# bound by the 2 blocks per CU that 73.7 KB of LDS per block allows?
# Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_gso_streams}; mkdir -p $OUT
for r in 1 2; do
  for ns in 1 2 3 4 6 8; do
    timeout -k 10 120 python bench.py --config cfg4 --streams $ns --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e > $OUT/s$ns.log 2>&1 || { echo "rc=$? $ns"; tail -5 $OUT/s$ns.log; exit 1; }
    grep '^{"metric"' $OUT/s$ns.log | sed "s/^{/{\"tag\": \"s${ns}_$r\", /" >> $OUT/lines.jsonl
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:8s} kern {r['kernel_ms']*1e3:7.2f} us frac {r['frac']:.4f} value {d['value']}")
PY
