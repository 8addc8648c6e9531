#!/bin/bash
# Round 4: GSO rows-per-segment variants (WGCS_GSO_PARTS / WAVES) -- parity of the
# variant libraries on the GSO tests, then an interleaved cfg4 A/B.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_gso_ab}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc $(tail -n 1 $OUT/$n.log | cut -c1-200)"; case $rc in 124|134|137|139) exit $rc;; esac; return $rc; }
LIBS=${LIBS:-"p1 p2 p4 p2w6 p2w8 p4w8"}
for v in $LIBS; do
  [ "$v" = p1 ] && continue
  WGCS_LIB=scripts/probe_so/libwgcsum_$v.so step par_$v 300 python -u -m pytest tests/test_gpu_gso.py tests/test_gpu_fullsize.py tests/test_gpu_stager.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread || exit 1
done
args=""; for v in $LIBS; do args="$args scripts/probe_so/libwgcsum_$v.so"; done
CFG=cfg4 ROUNDS=${ROUNDS:-3} step ab 900 bash scripts/probe_lib_bench.sh $args || exit 1
python3 - $OUT/ab.log <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith("{"):
        j = json.loads(l); r = j["line"]["roofline"]
        d[j["lib"]].append((r["kernel_ms"] * 1e3, r.get("kernel_ms_one_stream", 0) * 1e3))
for k, v in d.items():
    print(k, "two-stream us", [round(a, 2) for a, _ in v], "one-stream us", [round(b, 2) for _, b in v])
PY
