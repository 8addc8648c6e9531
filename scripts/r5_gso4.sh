#!/bin/bash
# Round 5: GSO parity on the wave-0-head LDS kernel, A/B against the round-4
# grid, phase stamps (NOT product code: a measurement script).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_gso4}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_fullsize.py tests/test_gpu_stager.py tests/test_gpu_c_harness.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
NWAVES=8 timeout -k 10 120 python scripts/probe_gso_stamps.py run > $OUT/stamps_lds.jsonl 2>&1 || exit 1
cat $OUT/stamps_lds.jsonl | grep streams
export WGCS_GSO_KERNEL_AB=1
for rep in 1 2; do
  timeout -k 10 120 python bench.py --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e > $OUT/lds_$rep.log 2>&1 || exit 1
  grep '^{"metric"' $OUT/lds_$rep.log | sed "s/^{/{\"tag\": \"lds_$rep\", /" >> $OUT/lines.jsonl
  WGCS_GSO_KERNEL=rows timeout -k 10 120 python bench.py --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e > $OUT/rows_$rep.log 2>&1 || exit 1
  grep '^{"metric"' $OUT/rows_$rep.log | sed "s/^{/{\"tag\": \"rows_$rep\", /" >> $OUT/lines.jsonl
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    print(f"{d['tag']:12s} {r['kernel_ms']*1e3:7.2f} us  frac {r['frac']:.4f}  1s {r['kernel_ms_one_stream']*1e3:7.2f} us {r['frac_one_stream']:.4f}")
PY
