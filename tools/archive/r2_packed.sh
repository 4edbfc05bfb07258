#!/bin/bash
# Packed read upload: GPU tests + c5r A/B (CEC_C5R_PACKED=1: submit_packed; 0: per-run copies).
#   bash tools/r2_packed.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/r2_packed}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread -k "read or resilver or verify or pipeline or multi or retry" > "$OUT/pytest.log" 2>&1
for i in 1 2; do
  for k in 1 0; do
    CEC_C5R_PACKED=$k timeout -k 10 300 python -u bench.py --config c5r --stream-gib 64 --check > "$OUT/c5r_packed${k}_$i.log" 2>&1
  done
done
echo "packed done"
