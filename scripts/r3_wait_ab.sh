#!/bin/bash
# A/B (NOT product code): completion-wait mode of the HIP runtime in the driver's
# invocation: wall - event span of each timed region with the default wait
# (active for ROC_ACTIVE_WAIT_TIMEOUT us, then blocked on an interrupt) vs a longer spin.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r3_wait_ab}; mkdir -p $OUT
for r in 1 2; do
  for w in default 0 50 2000; do
    if [ $w = default ]; then E=""; else E="ROC_ACTIVE_WAIT_TIMEOUT=$w"; fi
    line=$(env $E timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e --repeat 4 2>>$OUT/err.log | grep '^{') || { echo "FAIL $w"; exit 1; }
    echo "{\"wait\": \"$w\", \"round\": $r, \"line\": $line}" >> $OUT/wait.jsonl
    echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['timing']; print('$w', d['value'], t['wall_minus_span_us'], [round(x['wall_us']-x['event_span_us'],1) for x in t.get('repeats',[])])"
  done
done
