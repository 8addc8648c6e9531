#!/bin/bash
# Round 5: interleaved cfg4 A/B of library builds (NOT product code).
# usage: TAG=... LIBS="libwgcsum.so scripts/probe_so/x.so ..." bash scripts/r5_gso_ab.sh [reps]
# (BENCH_ARGS: extra bench.py arguments; CONFIG: bench config, default cfg4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r5_gso_ab}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
REPS=${1:-2}
for rep in $(seq 1 $REPS); do
  for lib in ${LIBS}; do
    name=$(basename $lib .so)_$rep
    p=$ROOT/$lib
    [ "$lib" = libwgcsum.so ] && p=$ROOT/wireguard_amd/libwgcsum.so
    echo "== [$name] $(date +%T)"
    WGCS_LIB=$p timeout -k 10 120 python bench.py --config ${CONFIG:-cfg4} --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e ${BENCH_ARGS:-} > "$OUT/$name.log" 2>&1
    rc=$?
    echo "== [$name] rc=$rc"
    case $rc in 0) ;; *) echo "FATAL rc=$rc"; tail -5 "$OUT/$name.log"; exit $rc;; esac
    grep '^{"metric"' "$OUT/$name.log" | tail -n 1 | sed "s/^{/{\"tag\": \"$name\", /" >> "$OUT/lines.jsonl"
  done
done
python3 - "$OUT/lines.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["roofline"]
    one = r.get("kernel_ms_one_stream")
    print(f"{d['tag']:32s} {r['kernel_ms']*1e3:7.2f} us  frac {r['frac']:.4f}" +
          (f"  1s {one*1e3:7.2f} us {r['frac_one_stream']:.4f}" if one else ""))
PY
