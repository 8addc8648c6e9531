#!/bin/bash
# Round 4: wave-cooperative walk of long TCP flows in gro_batch_kernel -- parity
# (every GRO GPU test through the batched kernel), phase timeline, then an
# interleaved A/B of the gro_device lines per call shape (base vs coop library).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_gro_coop}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc $(tail -n 1 $OUT/$n.log | cut -c1-200)"; case $rc in 124|134|137|139) exit $rc;; esac; return $rc; }
step parity 400 python -u -m pytest tests/test_gpu_gro_batch.py tests/test_gpu_wstager.py tests/test_gpu_gro.py tests/test_gpu_abi_safety.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread || { grep -E "Error|assert|FAIL" $OUT/parity.log | head -20; exit 1; }
WGCS_LIB_PARTIAL=1 step phases 300 python scripts/probe_gro_phases.py || exit 1
grep '^{' $OUT/phases.log
for r in 1 2; do
  for s in ${SHAPES:-shuffled 4x32 1x128 4x32rev}; do
    for lib in base coop; do
      WGCS_LIB=scripts/probe_so/libwgcsum_$lib.so WGCS_LIB_PARTIAL=1 step l_${s}_${lib}_$r 200 python bench.py --config gro_device --gro-shape $s --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e || exit 1
      grep '^{' $OUT/l_${s}_${lib}_$r.log | sed "s/^{/{\"lib\": \"$lib\", \"shape\": \"$s\", /" >> $OUT/ab.jsonl
    done
  done
done
python3 - $OUT/ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); r = j.get("roofline", {})
    d[(j["shape"], j["lib"])].append((round(j["value"] / 1e6, 1), r.get("frac"), r.get("kernel_ms")))
for k in sorted(d): print(k, d[k])
PY
