#!/bin/bash
# Round 5: checksum blocks of 256 / 512 / 1,024 threads (WGCS_CS_BLOCK builds):
# checksum parity per build, then cfg2 lines (the driver's command and a
# 200-step one-stream region) interleaved over 3 rounds.  Measurement script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_cs_block}; mkdir -p $OUT
LIBS=${LIBS:-"wireguard_amd/libwgcsum.so scripts/probe_so/libwgcsum_csblk512.so scripts/probe_so/libwgcsum_csblk1024.so"}
T="tests/test_gpu_checksum.py tests/test_gpu_batches.py tests/test_gpu_fullsize.py"
for lib in $LIBS; do
  name=$(basename $lib .so)
  WGCS_LIB=$ROOT/$lib timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu $T > $OUT/tests_$name.txt 2>&1 || { echo "tests $name rc=$?"; tail -5 $OUT/tests_$name.txt; exit 1; }
  echo "$name $(tail -1 $OUT/tests_$name.txt)"
done
for r in 1 2 3; do
  for lib in $LIBS; do
    name=$(basename $lib .so)
    WGCS_LIB=$ROOT/$lib timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e --no-strong > $OUT/run.log 2>&1 || { echo "rc=$? $name"; tail -5 $OUT/run.log; exit 1; }
    grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"tag\": \"drv_${name}_$r\", /" >> $OUT/lines.jsonl
    WGCS_LIB=$ROOT/$lib timeout -k 10 150 python bench.py --steps 200 --warmup 20 --streams 1 --cpu-seconds 0 --no-e2e --no-strong > $OUT/run.log 2>&1 || { echo "rc=$? $name"; tail -5 $OUT/run.log; exit 1; }
    grep '^{"metric"' $OUT/run.log | sed "s/^{/{\"tag\": \"one_${name}_$r\", /" >> $OUT/lines.jsonl
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:30s} {r['kernel_ms']*1e3:7.2f} us frac {r['frac']:.4f}  1s {r.get('kernel_ms_one_stream', 0)*1e3:7.2f}")
PY
