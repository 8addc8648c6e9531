#!/bin/bash
# Round 5: the driver's command with and without the configs[4] prewarm
# (--warm-ms), alternated.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_strong_prewarm}; mkdir -p $OUT
for r in 1 2; do
  for w in 40 0; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --warm-ms $w > $OUT/w${w}_$r.log 2>&1 || { echo "rc=$? $w"; tail -5 $OUT/w${w}_$r.log; exit 1; }
    grep '^{"metric"' $OUT/w${w}_$r.log | sed "s/^{/{\"tag\": \"warm${w}_$r\", /" >> $OUT/lines.jsonl
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
sys.path.insert(0, ".")
import bench
for l in open(sys.argv[1]):
    d = json.loads(l); s = d["cfg5_strong"]
    print(d["tag"], "value", d["value"], "frac", d["roofline"]["frac"], "| strong", s["value"], s["roofline"]["frac"],
          round(s["roofline"]["kernel_ms"] * 1e3, 1), "us prewarm", s.get("prewarm", {}).get("launches"),
          "problems", bench.line_problems({k: v for k, v in d.items() if k != "tag"}))
PY
