#!/bin/bash
# Round 4, first box: the whole GPU suite (new ABI-safety and GSO tests), smoke, then the N>1 line rehearsal.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/${TAG:-r4_a}; mkdir -p $OUT
step() { local n=$1 l=$2; shift 2; echo "== [$n] $(date +%T)"; timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "== [$n] rc=$rc $(tail -n 1 $OUT/$n.log | cut -c1-200)"; case $rc in 124|134|137|139) exit $rc;; esac; return $rc; }
step tests 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -rs || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit 1; }
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
TAG=r4_multi bash scripts/r4_multi.sh
