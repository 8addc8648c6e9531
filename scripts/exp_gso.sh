#!/bin/bash
# A/B timing of kernel variants built into exp/*.so (timing only, not product).
# CFG selects the bench config (default cfg4, the GSO split).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for so in "" exp/*.so; do
  echo "== variant ${so:-product}"
  WGCS_LIB=${so:+$PWD/$so} timeout -k 10 120 python bench.py --config ${CFG:-cfg4} --no-e2e --steps 200 --warmup 20 --cpu-seconds 0 2>&1 \
    | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], d['roofline']['d2d_copy_same_bytes_ms'])" || exit 1
done
