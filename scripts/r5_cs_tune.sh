#!/bin/bash
# Round 5: checksum launch tuning (api.cpp's WGCS_* overrides) on the headline
# config, two streams and one, interleaved.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_cs_tune}; mkdir -p $OUT
for r in 1 2; do
  for v in ${VARIANTS:-base UNROLL=6 UNROLL=3 LANES_PER_PKT=16 LANES_PER_PKT=64 LANES_PER_PKT=16,UNROLL=8}; do
    envs=()
    if [ "$v" != base ]; then IFS=',' read -ra kv <<< "$v"; for x in "${kv[@]}"; do envs+=("WGCS_$x"); done; fi
    env "${envs[@]}" timeout -k 10 120 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e --no-strong > $OUT/run.log 2>&1 || { echo "rc=$? $v"; tail -5 $OUT/run.log; exit 1; }
    grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"tag\": \"${v//[=,]/}_$r\", /" >> $OUT/lines.jsonl
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:28s} 2s {r['kernel_ms']*1e3:6.2f} us {r['frac']:.4f}  1s {r['kernel_ms_one_stream']*1e3:6.2f} us {r['frac_one_stream']:.4f}  {r['kernel']}")
PY
