#!/bin/bash
# Round 4, late: FETCH_SIZE calibration (GRO and udp_coalesce patterns) and the
# N = 2 line rehearsed as two gloo ranks on the box's one GPU (two-stream
# strong block).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_late}; mkdir -p $OUT
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fcal -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/probe_fetch_cal.py > $OUT/fcal.log 2>&1) || exit 1
python3 scripts/fetch_cal_summary.py $OUT/fcal $OUT/fcal.log | tee $OUT/fcal_summary.json
WGCS_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/g2.log 2>&1 || { tail -5 $OUT/g2.log; exit 1; }
grep '^{' $OUT/g2.log > $OUT/g2.jsonl
python3 -c "
import json, sys
sys.path.insert(0, '.')
import bench
d = json.loads(open('$OUT/g2.jsonl').readline())
s = d['cfg5_strong']
print(d['n_gpus'], d['value'], d['roofline']['frac'], 'strong', s['value'], s['streams'], s['roofline']['frac'], 'problems', bench.line_problems(d))"
