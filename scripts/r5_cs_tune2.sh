#!/bin/bash
# Round 5: 16-lane rows with 6 / 8 loads in flight against the default
# (32 lanes, 4) on cfg2 / cfg2 fill / cfg3 / cfg5, parity with the candidate
# as default via env, and sized reads.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_cs_tune2}; mkdir -p $OUT
export TMPDIR=/tmp
T="tests/test_gpu_checksum.py tests/test_gpu_batches.py tests/test_gpu_fullsize.py"
WGCS_LANES_PER_PKT=16 WGCS_UNROLL=8 timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu $T > $OUT/tests_g16u8.txt 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests_g16u8.txt; exit 1; }
tail -1 $OUT/tests_g16u8.txt
for r in 1 2; do
  for v in base LANES_PER_PKT=16,UNROLL=8 LANES_PER_PKT=16,UNROLL=6; do
    envs=()
    if [ "$v" != base ]; then IFS=',' read -ra kv <<< "$v"; for x in "${kv[@]}"; do envs+=("WGCS_$x"); done; fi
    for c in "cfg2" "cfg2 --mode fill" "cfg3" "cfg5"; do
      set -- $c
      name=${v//[=,]/}_$1${2:+fill}_$r
      extra="--no-strong"; [ $1 != cfg2 ] && extra=""
      env "${envs[@]}" timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e $extra > $OUT/run.log 2>&1 || { echo "rc=$? $name"; tail -5 $OUT/run.log; exit 1; }
      grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"tag\": \"$name\", /" >> $OUT/lines.jsonl
    done
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    one = r.get("kernel_ms_one_stream")
    print(f"{d['tag']:36s} {r['kernel_ms']*1e3:7.2f} us {r['frac']:.4f}" + (f"  1s {one*1e3:7.2f} us {r['frac_one_stream']:.4f}" if one else ""))
PY
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
for c in cfg2 cfg5; do
  extra="--no-strong"; [ $c != cfg2 ] && extra="--warm-ms 0"
  (cd /tmp && WGCS_LANES_PER_PKT=16 WGCS_UNROLL=8 timeout -s KILL 120 rocprofv3 --pmc $SIZED --kernel-trace -d $OUT/sized_$c -o run --output-format csv -- python3 $ROOT/bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1 $extra > $OUT/sized_$c.log 2>&1) || { echo "FAIL sized $c"; exit 1; }
  echo "== $c g16u8 $(python3 scripts/pmc_sized.py $OUT/sized_$c checksum_batch | cut -c150-400)"
done
