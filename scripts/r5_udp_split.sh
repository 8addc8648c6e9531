#!/bin/bash
# Round 5: udp_split with regular instead of non-temporal source loads (the
# lines two neighbouring packets share can then be served by the L2 the
# second time): interleaved A/B + the L2's sized reads.  Measurement script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_udp_split}; mkdir -p $OUT
export TMPDIR=/tmp
LIBS=${LIBS:-"libwgcsum.so scripts/probe_so/libwgcsum_udp_split_rt.so"}
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conn.py > $OUT/tests.txt 2>&1 || { echo "tests rc=$?"; tail -5 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
for r in 1 2 3; do
  for lib in $LIBS; do
    p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
    name=$(basename $lib .so)
    WGCS_LIB=$p timeout -k 10 150 python bench.py --config udp_split --steps 50 --warmup 5 --cpu-seconds 0 --no-e2e > $OUT/run.log 2>&1 || { echo "rc=$? $name"; tail -5 $OUT/run.log; exit 1; }
    grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"tag\": \"${name}_$r\", /" >> $OUT/lines.jsonl
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:34s} {r['kernel_ms']*1e3:7.2f} us frac {r['frac']:.4f}  1s {r['kernel_ms_one_stream']*1e3:7.2f} us {r['frac_one_stream']:.4f}")
PY
SIZED="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
for lib in $LIBS; do
  p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
  name=$(basename $lib .so)
  (cd /tmp && WGCS_LIB=$p timeout -s KILL 120 rocprofv3 --pmc $SIZED --kernel-trace -d $OUT/sized_$name -o run --output-format csv -- python3 $ROOT/bench.py --config udp_split --steps 10 --warmup 2 --cpu-seconds 0 --no-e2e --no-event-timing --streams 1 > $OUT/sized_$name.log 2>&1) || { echo "FAIL sized $name"; exit 1; }
  echo "== $name $(python3 scripts/pmc_sized.py $OUT/sized_$name udp_split | cut -c100-400)"
done
