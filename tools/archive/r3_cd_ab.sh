#!/bin/bash
# A/B of the reconstruct kernel's row classes (CEC_APPLY_RGCLS=0: compiled for 8 rows, 'old') and
# of the compile-time-d form (CEC_APPLY_CD = loads G inputs ahead; 0 = run-time
# d), interleaved on one box: c3e2 (north_star's 2-erasure reconstruct_data) and C3 (1-4 erasures,
# data + parity), each checked against the oracle; then the reconstruct GPU tests under each G.
set -o pipefail
T=gpurun_out/${1:-r3_cd_ab}
mkdir -p $T
for cd in 0 5; do
  CEC_APPLY_CD=$cd timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 150 --timeout-method thread -k "reconstruct or read or resilver or split" > $T/pytest_cd$cd.log 2>&1 || { tail -30 $T/pytest_cd$cd.log; exit 1; }
  tail -1 $T/pytest_cd$cd.log
done
for rep in 1 2; do
  for cd in old 0 2 5 10; do
    for c in c3e2 c3; do
      if [ $cd = old ]; then export CEC_APPLY_RGCLS=0 CEC_APPLY_CD=0; else export CEC_APPLY_RGCLS=1 CEC_APPLY_CD=$cd; fi
      ck=""; [ $rep = 1 ] && ck="--check"
      timeout -k 10 300 python -u bench.py --config $c $ck --no-cpu-baseline > $T/bench_${c}_cd${cd}_$rep.log 2>&1 || exit 1
      echo "$c cd=$cd rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"check_vs_oracle": [a-z]*' $T/bench_${c}_cd${cd}_$rep.log | tr '\n' ' ')"
    done
  done
done
