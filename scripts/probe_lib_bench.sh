#!/bin/bash
# A/B of library builds on one bench config (NOT product code): interleaves
# `python bench.py --config $CFG` over the libraries named on the command line
# (WGCS_LIB), ROUNDS rounds, one JSON line each, tagged with the library.
# usage: CFG=udp_coalesce ROUNDS=3 bash scripts/probe_lib_bench.sh scripts/probe_so/libwgcsum_a.so ...
set -o pipefail
CFG=${CFG:-cfg2}; ROUNDS=${ROUNDS:-3}; EXTRA=${EXTRA:-}
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    line=$(WGCS_LIB="$lib" WGCS_LIB_PARTIAL=1 timeout -k 10 120 python bench.py --config "$CFG" --steps 200 --warmup 20 --cpu-seconds 0 --no-e2e $EXTRA 2>/dev/null | grep '^{') || exit 1
    echo "{\"lib\": \"$(basename "$lib")\", \"round\": $r, \"line\": $line}"
  done
done
