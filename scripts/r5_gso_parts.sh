#!/bin/bash
# Round 5: GSO jobs split over P workgroups (gso_lds_kernel<NW, U, NT, P>) --
# parity of every variant build, then interleaved cfg4 A/B (default streams
# and one stream).  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_gso_parts}; mkdir -p $OUT
export TMPDIR=/tmp
LIBS=${LIBS:-"libwgcsum.so scripts/probe_so/libwgcsum_gso_p1w8.so scripts/probe_so/libwgcsum_gso_p2w6.so scripts/probe_so/libwgcsum_gso_p3w4.so scripts/probe_so/libwgcsum_gso_p4w4.so scripts/probe_so/libwgcsum_gso_p3w6.so"}
for lib in $LIBS; do
  p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
  name=$(basename $lib .so)
  WGCS_LIB=$p timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gso.py tests/test_gpu_stager.py > $OUT/tests_$name.txt 2>&1 || { echo "tests $name rc=$?"; tail -20 $OUT/tests_$name.txt; exit 1; }
  echo "$name $(tail -1 $OUT/tests_$name.txt)"
done
WGCS_LIB=$ROOT/wireguard_amd/libwgcsum.so timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k gso > $OUT/tests_fullsize.txt 2>&1 || { echo "fullsize rc=$?"; tail -20 $OUT/tests_fullsize.txt; exit 1; }
tail -1 $OUT/tests_fullsize.txt
for rep in 1 2; do
  for lib in $LIBS; do
    p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
    name=$(basename $lib .so)
    for ns in 0 1; do
      extra=""; [ $ns = 1 ] && extra="--streams 1"
      WGCS_LIB=$p timeout -k 10 120 python bench.py --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e $extra > $OUT/run.log 2>&1 || { echo "rc=$? $name"; tail -5 $OUT/run.log; exit 1; }
      grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"tag\": \"${name}_s${ns}_$rep\", /" >> $OUT/lines.jsonl
    done
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:36s} kern {r['kernel_ms']*1e3:7.2f} us frac {r['frac']:.4f} streams {d['config'].get('streams')}")
PY
