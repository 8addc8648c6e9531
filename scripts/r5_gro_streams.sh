#!/bin/bash
# Round 5: gro_device by stream count (consecutive launches on S streams:
# calls of the next launch start as the previous launch's calls retire).
# Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_gro_streams}; mkdir -p $OUT
for r in 1 2; do
  for shape in shuffled 4x32; do
    for ns in 1 2 3 4; do
      timeout -k 10 150 python bench.py --config gro_device --gro-shape $shape --streams $ns --steps 40 --warmup 4 --cpu-seconds 0 --no-e2e > $OUT/run.log 2>&1 || { echo "rc=$? $shape $ns"; tail -5 $OUT/run.log; exit 1; }
      grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"tag\": \"${shape}_s${ns}_$r\", /" >> $OUT/lines.jsonl
    done
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:16s} {d['value']/1e6:8.1f} M/s kern {r['kernel_ms']*1e3:7.1f} us frac {r['frac']:.4f}")
PY
