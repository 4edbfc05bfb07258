#!/bin/bash
# Hardware-queue A/B for the host-staged streams: HIP maps streams onto GPU_MAX_HW_QUEUES
# compute queues (4 by default), so a pipeline with more streams than queues shares queues
# between slots.  c5r (packed and per-run uploads) with side-stream decode on/off and
# 4 / 8 slots, at 4, 8 and 16 queues; c5 at 4 / 8 slots.
#   bash tools/r2_hwq.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/r2_hwq}
mkdir -p "$OUT"
for q in 4 8 16; do
  for side in 0 1; do
    for dep in 4 8; do
      GPU_MAX_HW_QUEUES=$q CEC_READ_SIDE=$side CEC_STREAM_DEPTH=$dep CEC_C5R_PACKED=1 \
        timeout -k 10 300 python -u bench.py --config c5r --stream-gib 64 --check \
        > "$OUT/c5r_q${q}_side${side}_d${dep}.log" 2>&1
    done
  done
  for dep in 4 8; do
    GPU_MAX_HW_QUEUES=$q CEC_STREAM_DEPTH=$dep timeout -k 10 300 python -u bench.py --config c5 --stream-gib 64 \
      > "$OUT/c5_q${q}_d${dep}.log" 2>&1
  done
done
echo "hwq done"
