#!/bin/bash
set -euo pipefail
OUT=${1:-gpurun_out/r2_d2hspan}
mkdir -p "$OUT"
for i in 1 2; do
  for sp in 1 0; do
    CEC_READ_D2H_SPAN=$sp CEC_C5R_PACKED=1 timeout -k 10 300 python -u bench.py --config c5r --stream-gib 64 --check > "$OUT/c5r_span${sp}_$i.log" 2>&1
  done
done
echo done
