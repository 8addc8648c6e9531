#!/bin/bash
# Round 4 probe: GRO wave-walk variants -- v1: try the append run again right
# after an insert; v2: walk only flows of 16+ packets by a wave; v3: both --
# phase timelines (timing-only builds) and interleaved gro_device lines.
set -u
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r4_gro_walk}; mkdir -p $OUT
: > $OUT/phases.jsonl
for v in cur v1 v2 v3; do
  so=scripts/probe_so/libwgcsum_grostamps.so; [ $v != cur ] && so=scripts/probe_so/libwgcsum_grostamps_$v.so
  WGCS_STAMPS_SO=$PWD/$so WGCS_LIB_PARTIAL=1 timeout -k 10 200 python scripts/probe_gro_phases.py > $OUT/ph.log 2>&1 || { echo "phases rc=$? $v"; tail -5 $OUT/ph.log; exit 1; }
  grep '^{' $OUT/ph.log | sed "s/^{/{\"variant\": \"$v\", /" >> $OUT/phases.jsonl
done
python3 -c "
import json
for l in open('$OUT/phases.jsonl'):
    d = json.loads(l)
    if d['shape'] in ('4x32','1x128','shuffled','16x8','32x4','1x128udp'):
        print(d['variant'], d['shape'], d['median_us']['walk'], d['call_us'], d['launch_span_us'])"
TAG=${TAG:-r4_gro_walk}_ab SHAPES="shuffled 16x8 4x32 1x128" LIBS="new v1 v2 v3" bash scripts/r4_gro_run_ab.sh
