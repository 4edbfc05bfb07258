#!/bin/bash
# Per-call tier A/B with the parity download beside the chains (now default): early per-caller
# uploads on / off.
set -euo pipefail
OUT=${1:-gpurun_out/r2_early_both}
mkdir -p "$OUT"
for r in 1 2; do
  for e in 0 1; do
    echo "== early_h2d=$e run $r" >> "$OUT/percall.log"
    CEC_COALESCE_EARLY_H2D=$e timeout -k 10 200 ./tools/percall_bench 10 32 64 100 256 >> "$OUT/percall.log" 2>&1
  done
done
echo "early both done"
