#!/bin/bash
# Round 5: where cfg5's (and cfg3's) reads beyond the algorithmic bytes come
# from (measurement script, NOT product code).  Per launch
# tuning variant (api.cpp's WGCS_* overrides): the L2's sized read requests
# (scripts/pmc_sized.py) and a timing line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_cfg5_traffic}; mkdir -p $OUT
export TMPDIR=/tmp
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
for cfg in ${CONFIGS:-cfg5 cfg3}; do
  for v in ${VARIANTS:-base NT=0 ALIGN=128 BLOCKS_PER_CU=512 UNROLL=6}; do
    envs=()
    if [ "$v" != base ]; then IFS=',' read -ra kv <<< "$v"; for x in "${kv[@]}"; do envs+=("WGCS_$x"); done; fi
    name=${cfg}_${v//[=,]/}
    (cd /tmp && env "${envs[@]}" timeout -s KILL 120 rocprofv3 --pmc $SIZED --kernel-trace -d $OUT/$name -o run --output-format csv -- python3 $ROOT/bench.py --config $cfg --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1 > $OUT/$name.log 2>&1) || { echo "FAIL $name"; tail -5 $OUT/$name.log; exit 1; }
    echo "== $name $(python3 scripts/pmc_sized.py $OUT/$name checksum_batch | cut -c1-60,150-400)"
    extra=""; [ $cfg = cfg2 ] && extra="--no-strong"
    env "${envs[@]}" timeout -k 10 120 python3 bench.py --config $cfg --steps ${STEPS:-30} --warmup 3 --cpu-seconds 0 --no-e2e $extra > $OUT/${name}_line.log 2>&1 || exit 1
    grep '^{"metric"' $OUT/${name}_line.log | sed "s/^{/{\"tag\": \"$name\", /" >> $OUT/lines.jsonl
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    one = r.get("kernel_ms_one_stream")
    print(f"{d['tag']:36s} {r['kernel_ms']*1e3:8.2f} us frac {r['frac']:.4f} value {d['value']}"
          + (f"  1s {one*1e3:8.2f} us {r['frac_one_stream']:.4f}" if one else ""))
PY
