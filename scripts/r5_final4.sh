#!/bin/bash
# Round-5 last check on the committed tree: the whole GPU suite, smoke and the
# driver's command once.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_final4}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/driver.log; exit 1; }
grep '^{"metric"' $OUT/driver.log > $OUT/driver_line.jsonl
python3 -c "
import json; d=json.loads(open('$OUT/driver_line.jsonl').readline()); r=d['roofline']
print('driver', d['value'], d['unit'], 'frac', r['frac'], 'one stream', r.get('frac_one_stream'), 'cfg5_strong', d.get('cfg5_strong',{}).get('roofline',{}).get('frac'))"
