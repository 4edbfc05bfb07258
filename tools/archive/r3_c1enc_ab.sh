#!/bin/bash
# Residency caps for the RS(3,2) bit-sliced encode (the reference's example clusters' shape),
# interleaved, each checked against the oracle.
set -o pipefail
T=gpurun_out/${1:-r3_c1enc_ab}
mkdir -p $T
for rep in 1 2 3; do
  for cap in 0 1 2 3 4; do
    timeout -k 10 120 env CEC_APPLY_BLOCKS_PER_CU=$cap python -u bench.py --config c1enc --check --no-cpu-baseline > $T/bench_c1enc_cap${cap}_$rep.log 2>&1 || exit 1
    echo "c1enc cap=$cap rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"check_vs_oracle": [a-z]*' $T/bench_c1enc_cap${cap}_$rep.log | tr '\n' ' ')"
  done
done
