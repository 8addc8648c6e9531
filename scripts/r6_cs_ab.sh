#!/bin/bash
# Round 6: checksum kernel A/B (NOT product code): checksum parity, then
# interleaved one-stream 200-step and driver-shaped lines per library.
# usage: LIBS="libwgcsum.so scripts/probe_so/x.so" TAG=... bash scripts/r6_cs_ab.sh [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
T=${TAG:-r6_cs_ab}
OUT=$ROOT/gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_checksum.py tests/test_gpu_batches.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
REPS=${1:-3}
for rep in $(seq 1 $REPS); do
  for lib in ${LIBS}; do
    p=$ROOT/$lib; [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
    name=$(basename $lib .so)_$rep
    WGCS_LIB=$p timeout -k 10 120 python bench.py --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e --no-strong > $OUT/${name}_1s.log 2>&1 || { tail -5 $OUT/${name}_1s.log; exit 1; }
    grep '^{"metric"' $OUT/${name}_1s.log | sed "s/^{/{\"tag\": \"${name}_1s\", /" >> $OUT/lines.jsonl
    WGCS_LIB=$p timeout -k 10 120 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e > $OUT/${name}_drv.log 2>&1 || { tail -5 $OUT/${name}_drv.log; exit 1; }
    grep '^{"metric"' $OUT/${name}_drv.log | sed "s/^{/{\"tag\": \"${name}_drv\", /" >> $OUT/lines.jsonl
  done
done
python3 - "$OUT/lines.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    one = r.get("kernel_ms_one_stream")
    print(f"{d['tag']:28s} value {d['value']:8.1f}  kernel {r['kernel_ms']*1e3:6.2f} us frac {r['frac']:.4f}" +
          (f"  1s {one*1e3:6.2f} us {r['frac_one_stream']:.4f}" if one else ""))
PY
