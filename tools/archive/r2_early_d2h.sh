#!/bin/bash
# Per-call tier A/B: the parity downloaded on a side stream right after the encode, beside the
# SHA-256 chains (CEC_COALESCE_EARLY_D2H=1), vs after the chains; per-call GPU tests with it on.
set -euo pipefail
OUT=${1:-gpurun_out/r2_early_d2h}
mkdir -p "$OUT"
CEC_COALESCE_EARLY_D2H=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "per_call or part_encode or coalesc or threads or percall" > "$OUT/pytest_early.log" 2>&1
for r in 1 2; do
  for e in 0 1; do
    echo "== early_d2h=$e run $r" >> "$OUT/percall.log"
    CEC_COALESCE_EARLY_D2H=$e timeout -k 10 200 ./tools/percall_bench 10 32 64 100 256 >> "$OUT/percall.log" 2>&1
  done
done
echo "early d2h done"
