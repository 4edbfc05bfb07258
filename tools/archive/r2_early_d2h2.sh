#!/bin/bash
# Per-call tier, parity download beside the chains (host-side hand-over): repeated runs at high
# caller counts (a device-side cross-stream form hung once at 256 pageable callers), early
# per-caller uploads on / off, and a 10-caller coalescing trace.
set -euo pipefail
OUT=${1:-gpurun_out/r2_early_d2h2}
mkdir -p "$OUT"
for r in 1 2 3; do
  for e in 0 1; do
    echo "== early_h2d=$e run $r" >> "$OUT/percall.log"
    CEC_COALESCE_EARLY_H2D=$e timeout -k 10 150 ./tools/percall_bench 10 32 64 100 256 >> "$OUT/percall.log" 2>&1
  done
done
CEC_COALESCE_EARLY_D2H=0 timeout -k 10 150 ./tools/percall_bench 64 100 256 > "$OUT/percall_d2h0.log" 2>&1
CEC_COALESCE_TRACE=1 timeout -k 10 120 ./tools/percall_bench 10 > "$OUT/trace10.log" 2>&1
echo "early d2h2 done"
