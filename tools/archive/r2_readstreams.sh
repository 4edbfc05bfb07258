#!/bin/bash
# Read-stream A/B: decode on a side stream beside the verification (CEC_READ_SIDE) and one
# shared upload stream for all slots (CEC_READ_UPSTREAM).  Read-path GPU tests with both knobs
# on, then c5r (per-run and packed uploads) interleaved over the four combinations.
#   bash tools/r2_readstreams.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/r2_readstreams}
mkdir -p "$OUT"
CEC_READ_SIDE=1 CEC_READ_UPSTREAM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_stress.py -x -q --timeout 300 --timeout-method thread -k "read or resilver or verify or pipeline or multi or retry" > "$OUT/pytest_knobs.log" 2>&1
for i in 1 2; do
  for side in 0 1; do
    for up in 0 1; do
      for packed in 0 1; do
        CEC_READ_SIDE=$side CEC_READ_UPSTREAM=$up CEC_C5R_PACKED=$packed \
          timeout -k 10 300 python -u bench.py --config c5r --stream-gib 64 --check \
          > "$OUT/c5r_side${side}_up${up}_packed${packed}_$i.log" 2>&1
      done
    done
  done
done
echo "readstreams done"
