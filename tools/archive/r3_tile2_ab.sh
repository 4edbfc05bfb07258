#!/bin/bash
# Column tile per block (CEC_APPLY_TILE) 8 KiB vs the 16 KiB default, interleaved, on every
# HBM-bound config: the bit-sliced encodes (c2enc, c4enc) and the v_perm reconstructs (c3e2, c3).
set -o pipefail
T=gpurun_out/r3_tile2_ab
mkdir -p $T
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "bitsliced or encode" > $T/pytest_bs.log 2>&1 || { tail -30 $T/pytest_bs.log; exit 1; }
tail -1 $T/pytest_bs.log
for r in 1 2; do
  for tb in 8192 16384; do
    for c in c2enc c4enc c3e2 c3; do
      CEC_APPLY_TILE=$tb timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $T/bench_${c}_t${tb}_$r.log 2>&1 || exit 1
      echo "tile=$tb run $r $c: $(grep -o '"kernels": {"[^"]*": {"ms": [0-9.]*' $T/bench_${c}_t${tb}_$r.log | grep -o '[0-9.]*$') ms"
    done
  done
done
