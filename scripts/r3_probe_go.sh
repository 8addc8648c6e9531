#!/bin/bash
# Records whether a Go toolchain exists on the GPU box (north_star asks for a
# pure-Go CPU baseline).  Host-only, no GPU use.
OUT=${1:-gpurun_out/r3_go_probe.txt}
{
  echo "date: $(date -u +%FT%TZ)"
  echo "host nproc: $(nproc)"
  for t in go gccgo tinygo gofmt; do
    p=$(command -v $t 2>/dev/null)
    if [ -n "$p" ]; then echo "$t: $p ($($t version 2>&1 | head -n 1))"; else echo "$t: not found"; fi
  done
  ls -d /usr/local/go /usr/lib/go* /opt/go 2>/dev/null || echo "no Go installation directory (/usr/local/go, /usr/lib/go*, /opt/go)"
} > "$OUT" 2>&1
cat "$OUT"
