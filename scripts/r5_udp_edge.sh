#!/bin/bash
# Round 5: udp_split with the packet's first and last 128-B lines (shared with
# the neighbouring packets) loaded temporal and the rest non-temporal
# (WGCS_UDP_SPLIT_EDGE_T): conn parity on that build, then the interleaved
# A/B + sized reads of r5_udp_split.sh.  Measurement script, NOT product code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-r5_udp_edge}; mkdir -p $OUT
WGCS_LIB=$ROOT/scripts/probe_so/libwgcsum_udp_edge_t.so timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conn.py > $OUT/tests_edge.txt 2>&1 || { echo "edge tests rc=$?"; tail -5 $OUT/tests_edge.txt; exit 1; }
tail -1 $OUT/tests_edge.txt
TAG=${TAG:-r5_udp_edge} LIBS="libwgcsum.so scripts/probe_so/libwgcsum_udp_edge_t.so" bash scripts/r5_udp_split.sh
