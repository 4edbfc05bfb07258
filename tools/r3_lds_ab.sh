#!/bin/bash
# LDS product-table apply path: GPU parity suite, then an interleaved A/B (CEC_APPLY_LDS=1/0,
# XCD order on) on the HBM-bound configs and the read batch.
set -o pipefail
T=gpurun_out/r3_lds_ab
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { tail -30 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
for r in 1 2; do
  for x in 1 0; do
    for c in c2enc c3e2 c3; do
      CEC_APPLY_LDS=$x timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --check > $T/bench_${c}_lds${x}_$r.log 2>&1 || exit 1
      echo "lds=$x run $r $c: $(grep -o '"kernels": {"[^"]*": {"ms": [0-9.]*' $T/bench_${c}_lds${x}_$r.log | grep -o '[0-9.]*$') ms, $(grep -o '"frac": [0-9.]*' $T/bench_${c}_lds${x}_$r.log | head -1) $(grep -o '"check_vs_oracle": [a-z]*' $T/bench_${c}_lds${x}_$r.log)"
    done
  done
done
for x in 1 0; do
  CEC_APPLY_LDS=$x timeout -k 10 200 python -u bench.py --config c3r --no-cpu-baseline --check > $T/bench_c3r_lds$x.log 2>&1 || exit 1
  echo "c3r lds=$x: $(grep -o '"value": [0-9.]*' $T/bench_c3r_lds$x.log | head -1) $(grep -o '"check_vs_oracle": [a-z]*' $T/bench_c3r_lds$x.log)"
done
