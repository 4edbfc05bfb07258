#!/bin/bash
# Bit-sliced encode kernel (rs_encode_bs_kernel): the -m gpu suite with it on (default), then an
# interleaved A/B against the v_perm kernel (CEC_APPLY_BS=0) on the RS(10,4) and RS(20,8)
# encodes, a tile-size sweep of the bit-sliced kernel, and the default bench line.
set -o pipefail
T=gpurun_out/r3_bs_ab
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { tail -30 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
for r in 1 2; do
  for bs in 1 0; do
    for c in c2enc c4enc; do
      CEC_APPLY_BS=$bs timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --check > $T/bench_${c}_bs${bs}_$r.log 2>&1 || exit 1
      echo "bs=$bs run $r $c: $(grep -o '"kernels": {"[^"]*": {"ms": [0-9.]*' $T/bench_${c}_bs${bs}_$r.log | grep -o '[0-9.]*$') ms, $(grep -o '"frac": [0-9.]*' $T/bench_${c}_bs${bs}_$r.log | head -1) $(grep -o '"check[a-z_]*": [a-z]*' $T/bench_${c}_bs${bs}_$r.log | head -1)"
    done
  done
done
for tb in 8192 32768 65536 16384; do
  CEC_APPLY_TILE=$tb timeout -k 10 200 python -u bench.py --config c2enc --no-cpu-baseline > $T/bench_c2enc_t$tb.log 2>&1 || exit 1
  echo "tile=$tb c2enc: $(grep -o '"kernels": {"[^"]*": {"ms": [0-9.]*' $T/bench_c2enc_t$tb.log | grep -o '[0-9.]*$') ms"
done
timeout -k 10 300 python -u bench.py > $T/bench_c2.log 2>&1 || exit 1
grep -o '"north_star": {.*' $T/bench_c2.log | head -c 1500; echo
