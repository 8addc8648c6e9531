#!/bin/bash
# Round 5: the GPU suite on the new checksum defaults (one-pass grid, 128-B
# aligned iterations) and the GSO LDS kernel, smoke, the driver's line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_d}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $OUT/tests.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_$k.log 2>&1 || exit 1
  grep '^{"metric"' $OUT/driver_$k.log | sed "s/^{/{\"tag\": \"driver_$k\", /" >> $OUT/lines.jsonl
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]; s = d.get("cfg5_strong", {})
    print(d["tag"], d["value"], r["kernel_ms"], r["frac"], r.get("frac_one_stream"), "strong", s.get("value"), s.get("roofline", {}).get("frac"),
          "ungated", d.get("timing", {}).get("ungated", {}).get("GiB_per_s"), "cpu", d["cpu_baseline"]["value"])
PY
