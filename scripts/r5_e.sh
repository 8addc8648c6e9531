#!/bin/bash
# Round 5: the driver's command, interleaved: checksum grid one pass (default)
# vs the round-4 16 blocks per CU, 3 rounds (measurement script).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5_e}; mkdir -p $OUT
for k in 1 2 3; do
  for v in base BLOCKS_PER_CU=16 ALIGN=16; do
    envs=(); [ $v != base ] && envs=("WGCS_$v")
    env "${envs[@]}" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e > $OUT/${v}_$k.log 2>&1 || exit 1
    grep '^{"metric"' $OUT/${v}_$k.log | sed "s/^{/{\"tag\": \"${v}_$k\", /" >> $OUT/lines.jsonl
  done
done
python3 - $OUT/lines.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]; t = d["timing"]; s = d["cfg5_strong"]
    print(f"{d['tag']:22s} {d['value']:8.1f} kern {r['kernel_ms']*1e3:6.2f} frac {r['frac']:.4f} 1s {r['frac_one_stream']:.4f} wall-span {t['wall_minus_span_us']:6.2f} ungated {t['ungated']['GiB_per_s']:8.1f} strong {s['value']:8.1f} {s['roofline']['frac']:.4f}")
PY
