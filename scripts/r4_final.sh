#!/bin/bash
# Final check of the committed tree: GPU suite, smoke, the driver's bench command three times.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_final}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc $(tail -n 1 $OUT/$n.log | cut -c1-160)"; case $rc in 124|134|137|139) exit $rc;; esac; }
step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do step drv$i 200 python bench.py --gpus 1 --steps 20 --warmup 5; grep '^{' $OUT/drv$i.log >> $OUT/driver_lines.jsonl; done
python3 -c "
import json
for l in open('$OUT/driver_lines.jsonl'):
    d=json.loads(l); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['roofline'].get('frac_one_stream'), d['timing']['wall_minus_span_us'])"
