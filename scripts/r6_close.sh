#!/bin/bash
# Round-6 close-out on the last tree (measurement script, NOT product code):
# the whole GPU suite, smoke, the driver's command twice, per-call ring latency.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6_close}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -1 $OUT/tests.log; [ $rc -eq 0 ] || { tail -30 $OUT/tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for r in a b; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_$r.log 2>&1 || { tail -5 $OUT/driver_$r.log; exit 1; }
  grep '^{"metric"' $OUT/driver_$r.log | tail -1 | sed "s/^{/{\"tag\": \"driver_$r\", /" >> $OUT/lines.jsonl
done
timeout -k 10 200 python scripts/probe_ring_calls.py > $OUT/ring_calls.jsonl 2>&1 || { tail -20 $OUT/ring_calls.jsonl; exit 1; }
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
for l in open(o + "/lines.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(d["tag"], d["value"], "frac", r["frac"], "1s", r.get("frac_one_stream"), "cfg5_strong", d["cfg5_strong"]["roofline"]["frac"] if "cfg5_strong" in d else None)
d = json.loads(open(o + "/ring_calls.jsonl").read().strip().splitlines()[-1])
print({k: v["median_us"] for k, v in d["checksum_valid"].items()}, {k: v["median_us"] for k, v in d["handle_virtio_read"].items() if isinstance(v, dict)})
PY
echo done
