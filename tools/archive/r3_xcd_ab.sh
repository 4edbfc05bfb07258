#!/bin/bash
# XCD-aware block order in rs_apply / rs_apply_var: GPU parity tests, then an interleaved A/B
# (CEC_APPLY_XCD=0/1) on the HBM-bound configs.
set -o pipefail
T=gpurun_out/r3_xcd_ab
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { tail -30 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
for r in 1 2; do
  for x in 1 0; do
    for c in c2enc c3e2 c3; do
      CEC_APPLY_XCD=$x timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $T/bench_${c}_xcd${x}_$r.log 2>&1 || exit 1
      echo "xcd=$x run $r $c: $(grep -o '"kernels": {"[^"]*": {"ms": [0-9.]*' $T/bench_${c}_xcd${x}_$r.log | grep -o '[0-9.]*$') ms, $(grep -o '"frac": [0-9.]*' $T/bench_${c}_xcd${x}_$r.log | head -1)"
    done
  done
done
CEC_APPLY_XCD=1 timeout -k 10 200 python -u bench.py --config c3r --no-cpu-baseline --check > $T/bench_c3r_xcd1.log 2>&1 || exit 1
CEC_APPLY_XCD=0 timeout -k 10 200 python -u bench.py --config c3r --no-cpu-baseline > $T/bench_c3r_xcd0.log 2>&1 || exit 1
for x in 1 0; do echo "c3r xcd=$x: $(grep -o '"value": [0-9.]*' $T/bench_c3r_xcd$x.log | head -1)"; done
