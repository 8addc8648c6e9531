#!/bin/bash
# Round 4: the cfg4 line with its defaults (4 streams, slots on lines), twice,
# and its rocprofv3 kernel trace (span per launch over the four streams).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_cfg4_final}; mkdir -p $OUT
: > $OUT/lines.jsonl
for r in 1 2; do
  timeout -k 10 200 python bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 2 > $OUT/l$r.log 2>&1 || { tail -5 $OUT/l$r.log; exit 1; }
  grep '^{' $OUT/l$r.log >> $OUT/lines.jsonl
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e > $OUT/prof.log 2>&1) || exit 1
python3 scripts/trace_span.py $OUT/prof/run_kernel_trace.csv gso_rows 100 20 | tee $OUT/trace_span.jsonl
python3 -c "
import json
for l in open('$OUT/lines.jsonl'):
    d = json.loads(l); r = d['roofline']
    print(d['value'], r['kernel_ms'], r['frac'], r.get('kernel_ms_one_stream'), d['config']['streams'], d['config']['hw_queues'])"
