#!/bin/bash
# Residency caps for rs_apply_kernel (the v_perm encode of shapes without a bit-sliced build) at
# 1-3 parity rows, interleaved, each checked against the oracle: RS(2,1) (tests/cluster.rs),
# RS(4,2), RS(8,2), RS(6,3); 8 192 parts x 1 MiB (RS(8,2): 4 096).
set -o pipefail
T=gpurun_out/${1:-r3_vperm_shapes_ab}
mkdir -p $T
for rep in 1 2; do
  for shape in 2,1 4,2 8,2 6,3; do
    parts=8192; [ $shape = 8,2 ] && parts=4096
    for cap in 0 2 3 4; do
      tag="s${shape/,/_}_cap${cap}_$rep"
      timeout -k 10 120 env CEC_APPLY_BLOCKS_PER_CU=$cap python -u bench.py --config c1enc --shape $shape --parts $parts --check --no-cpu-baseline > $T/bench_$tag.log 2>&1 || exit 1
      echo "RS($shape) cap=$cap rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"check_vs_oracle": [a-z]*' $T/bench_$tag.log | tr '\n' ' ')"
    done
  done
done
