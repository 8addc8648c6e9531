#!/bin/bash
# Round 4: the driver's bench line at N=1 (now with cfg5_strong), and the N>1
# line rehearsed as gloo ranks sharing the box's one GPU (--gpus 2 and 4).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_multi}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc $(tail -n 1 $OUT/$n.log | cut -c1-200)"; case $rc in 124|134|137|139) exit $rc;; esac; }
python3 - > $OUT/pci_probe.txt 2>&1 <<'EOF'
import os, torch
p = torch.cuda.get_device_properties(0)
print({k: getattr(p, k, None) for k in ("name", "pci_domain_id", "pci_bus_id", "pci_device_id", "gcnArchName")})
print("affinity", sorted(os.sched_getaffinity(0)))
from wireguard_amd import shard
print(shard.gpu_local_cpus(p))
print(shard.bind_numa_local(torch, 0, apply=False))
EOF
cat $OUT/pci_probe.txt
step drv1 300 python bench.py --gpus 1 --steps 20 --warmup 5
grep '^{' $OUT/drv1.log > $OUT/drv1.jsonl
# doorbell A/B on the driver's command shape (cfg2 only, interleaved)
for r in 1 2 3; do
  for g in gate nogate; do
    extra=""; [ $g = nogate ] && extra="--no-gate"
    step ab_${g}_$r 120 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-e2e --no-strong $extra && grep '^{' $OUT/ab_${g}_$r.log | sed "s/^{/{\"ab\": \"$g\", /" >> $OUT/gate_ab.jsonl
  done
done
python3 -c "
import json
for l in open('$OUT/gate_ab.jsonl'):
    d = json.loads(l); print(d['ab'], d['value'], d['timing']['wall_minus_span_us'], d['roofline']['kernel_ms'])"
export WGCS_DIST_BACKEND=gloo
step g2 300 python bench.py --gpus 2 --steps 20 --warmup 5
grep '^{' $OUT/g2.log > $OUT/r4_rehearse_gpus2_gloo.jsonl
step g4 300 python bench.py --gpus 4 --steps 20 --warmup 5
grep '^{' $OUT/g4.log > $OUT/r4_rehearse_gpus4_gloo.jsonl
unset WGCS_DIST_BACKEND
python3 -c "
import json, sys
sys.path.insert(0, '.')
import bench
for fn in ('drv1.jsonl', 'r4_rehearse_gpus2_gloo.jsonl', 'r4_rehearse_gpus4_gloo.jsonl'):
    for l in open('$OUT/' + fn):
        d = json.loads(l)
        s = d.get('cfg5_strong', {})
        print(fn, d['n_gpus'], d['value'], d['roofline']['frac'], d['roofline'].get('kernel_ms_per_rank'), 'strong', s.get('value'), s.get('roofline', {}).get('frac'), 'cpu', d.get('cpu_baseline', {}).get('value'), 'problems', bench.line_problems(d))
"
