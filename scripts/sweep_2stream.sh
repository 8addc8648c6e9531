set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in "16 4 32" "8 4 32" "12 4 32" "24 4 32" "32 4 32" "16 3 32" "16 6 32" "16 4 64" "8 6 32"; do
  set -- $v
  WGCS_BLOCKS_PER_CU=$1 WGCS_UNROLL=$2 WGCS_LANES_PER_PKT=$3 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e > gpurun_out/sw.log 2>&1 || exit 1
  echo "bpc=$1 U=$2 G=$3 $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/sw.log) $(grep -o '"frac": [0-9.]*' gpurun_out/sw.log | head -1) $(grep -o '"kernel_ms_one_stream": [0-9.]*' gpurun_out/sw.log)"
done; done
