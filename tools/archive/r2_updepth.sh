#!/bin/bash
# c5r (packed uploads): one shared upload stream (CEC_READ_UPSTREAM=1) with 4 / 6 / 8 slots vs
# the default per-slot uploads, interleaved.
set -euo pipefail
OUT=${1:-gpurun_out/r2_updepth}
mkdir -p "$OUT"
for i in 1 2; do
  for cfg in "0 4" "1 4" "1 6" "1 8"; do
    set -- $cfg
    CEC_READ_UPSTREAM=$1 CEC_STREAM_DEPTH=$2 CEC_C5R_PACKED=1 timeout -k 10 300 \
      python -u bench.py --config c5r --stream-gib 64 --check > "$OUT/c5r_up$1_d$2_$i.log" 2>&1
  done
done
echo "updepth done"
