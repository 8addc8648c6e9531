#!/bin/bash
# A/B timing of GSO kernel variants built into exp/*.so (timing only, not product).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for so in "" exp/*.so; do
  echo "== variant ${so:-product}"
  WGCS_LIB=${so:+$PWD/$so} timeout -k 10 120 python bench.py --config cfg4 --steps 200 --warmup 20 --cpu-seconds 0 2>&1 \
    | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], d['roofline']['d2d_copy_same_bytes_ms'])" || exit 1
done
