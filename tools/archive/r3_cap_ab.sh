#!/bin/bash
# The per-kernel residency caps as defaults (rs_kernels.hip apply_lds) against no cap
# (CEC_APPLY_BLOCKS_PER_CU=0) and the compile-time-d reconstruct (CEC_APPLY_CD=5), interleaved.
set -o pipefail
T=gpurun_out/${1:-r3_cap_ab}
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "reconstruct or encode or split or read" > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
run() {  # tag config env...
  local tag=$1 c=$2; shift 2
  env "$@" timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline --check > $T/bench_${c}_$tag.log 2>&1 || exit 1
  echo "$c $tag $(grep -o '"ms_per_step": [0-9.]*\|"check_vs_oracle": [a-z]*' $T/bench_${c}_$tag.log | tr '\n' ' ')"
}
for rep in 1 2 3; do
  for c in c3e2 c3 c2enc c4enc; do
    run "cap_$rep" $c
    run "nocap_$rep" $c CEC_APPLY_BLOCKS_PER_CU=0
    case $c in c3e2|c3) run "cap_cd5_$rep" $c CEC_APPLY_CD=5 ;; esac
  done
done
