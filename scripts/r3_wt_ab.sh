#!/bin/bash
# A/B (NOT product code): plain vs write-through (sc1) 16-B output stores, on the
# output-heavy lines: cfg4 (GSO) one and two streams, udp_split, udp_coalesce, gro_device.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=$PWD/gpurun_out/${TAG:-r3_wt_ab}; mkdir -p $OUT
ROUNDS=${ROUNDS:-2}
run() {  # lib cfg extra...
  local lib=$1 cfg=$2; shift 2
  local line
  line=$(WGCS_LIB=scripts/probe_so/$lib timeout -k 10 120 python bench.py --config $cfg --steps 100 --warmup 10 --cpu-seconds 0 --no-e2e "$@" 2>>$OUT/err.log | grep '^{') || { echo "FAIL $lib $cfg rc=$?"; exit 1; }
  echo "{\"lib\": \"$lib\", \"cfg\": \"$cfg\", \"extra\": \"$*\", \"line\": $line}" >> $OUT/ab.jsonl
  echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$lib $cfg $*', d['value'], r.get('kernel_ms'), r.get('frac'), r.get('kernel_ms_one_stream'), r.get('frac_one_stream'))"
}
for r in $(seq 1 $ROUNDS); do
  for lib in ${LIBS:-libwgcsum_base.so libwgcsum_wt.so}; do
    for c in ${CFGS:-cfg4 udp_split udp_coalesce gro_device}; do run $lib $c || exit 1; done
  done
done
