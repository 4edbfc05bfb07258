#!/bin/bash
# Occupancy sweep of the HBM-bound GF kernels, interleaved on one box: CEC_APPLY_BLOCKS_PER_CU caps
# residency at n 256-thread blocks (= waves per SIMD) per CU through an unused LDS reservation
# (0 = the kernel's register-bound occupancy).  Reconstruct also A/Bs the row classes
# (CEC_APPLY_RGCLS=0: kernel compiled for 8 rows, 135 VGPRs).
set -o pipefail
T=gpurun_out/${1:-r3_occ_ab}
mkdir -p $T
CEC_APPLY_BLOCKS_PER_CU=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "reconstruct or encode or split" > $T/pytest_occ2.log 2>&1 || { tail -30 $T/pytest_occ2.log; exit 1; }
tail -1 $T/pytest_occ2.log
run() {  # tag config env...
  local tag=$1 c=$2; shift 2
  env "$@" timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline > $T/bench_${c}_$tag.log 2>&1 || exit 1
  echo "$c $tag $(grep -o '"ms_per_step": [0-9.]*' $T/bench_${c}_$tag.log | head -1)"
}
for rep in 1 2 3; do
  for occ in 0 1 2 3 4; do
    for c in c3e2 c3; do
      run "cls1_occ${occ}_$rep" $c CEC_APPLY_RGCLS=1 CEC_APPLY_BLOCKS_PER_CU=$occ
      run "cls0_occ${occ}_$rep" $c CEC_APPLY_RGCLS=0 CEC_APPLY_BLOCKS_PER_CU=$occ
    done
    for c in c2enc c4enc; do
      run "occ${occ}_$rep" $c CEC_APPLY_BLOCKS_PER_CU=$occ
    done
  done
done
