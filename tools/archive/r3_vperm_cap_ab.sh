#!/bin/bash
# Residency caps for rs_apply_kernel (the v_perm encode of shapes without a bit-sliced build;
# here RS(10,4) / RS(20,8) forced onto it with CEC_APPLY_BS=0), interleaved; then c3r and c3e2
# on the current defaults.
set -o pipefail
T=gpurun_out/${1:-r3_vperm_cap_ab}
mkdir -p $T
run() {  # tag config env...
  local tag=$1 c=$2; shift 2
  env "$@" timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline > $T/bench_${c}_$tag.log 2>&1 || exit 1
  echo "$c $tag $(grep -o '"ms_per_step": [0-9.]*' $T/bench_${c}_$tag.log | head -1)"
}
for rep in 1 2 3; do
  for cap in 0 2 3 4; do
    for c in c2enc c4enc; do
      run "vperm_cap${cap}_$rep" $c CEC_APPLY_BS=0 CEC_APPLY_BLOCKS_PER_CU=$cap
    done
  done
  run "default_$rep" c3r
  run "default_$rep" c3e2
done
