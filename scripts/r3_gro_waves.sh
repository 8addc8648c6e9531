#!/bin/bash
# gro_batch_kernel compiled for 7 vs 8 waves per SIMD (NOT product code): parity of the
# 8-wave build, then gro_device lines at 1,792 and 2,048 calls per launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r3_gro_waves}; mkdir -p $OUT
WGCS_LIB=scripts/probe_so/libwgcsum_gw8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gro_batch.py tests/test_gpu_wstager.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do for lib in gw7 gw8; do for calls in 1792 2048; do for shape in 4x32 1x128; do
  line=$(WGCS_GRO_CALLS=$calls WGCS_LIB=scripts/probe_so/libwgcsum_$lib.so timeout -k 10 120 python bench.py --config gro_device --gro-shape $shape --steps 40 --warmup 4 --cpu-seconds 0 2>>$OUT/err.log | grep '^{') || exit 1
  echo "{\"lib\": \"$lib\", \"calls\": $calls, \"shape\": \"$shape\", \"line\": $line}" >> $OUT/ab.jsonl
  echo "$lib calls=$calls $shape $(echo $line | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e6,1), 'Mpkt/s', round(r['kernel_ms']*1e3,1), 'us', r['frac'])")"
done; done; done; done
