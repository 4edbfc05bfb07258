#!/bin/bash
# Per-call tier A/B: early per-caller uploads (CEC_COALESCE_EARLY_H2D=1) vs one upload by the
# leader after every caller's copy-in; per-call GPU tests with the knob on first.
set -euo pipefail
OUT=${1:-gpurun_out/r2_early_h2d}
mkdir -p "$OUT"
CEC_COALESCE_EARLY_H2D=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "per_call or part_encode or coalesc or threads or percall" > "$OUT/pytest_early.log" 2>&1
for r in 1 2; do
  for e in 0 1; do
    echo "== early=$e run $r" >> "$OUT/percall.log"
    CEC_COALESCE_EARLY_H2D=$e timeout -k 10 200 ./tools/percall_bench 10 16 32 64 100 256 >> "$OUT/percall.log" 2>&1
  done
done
echo "early done"
