#!/bin/bash
# rs_apply tile size per block (CEC_APPLY_TILE) with the XCD order: parity at 8 KiB and 64 KiB
# tiles, then an interleaved A/B on C2 encode and the 2-erasure reconstruct.
set -o pipefail
T=gpurun_out/r3_tile_ab
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { tail -30 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
for tb in 8192 65536; do
  CEC_APPLY_TILE=$tb timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 150 --timeout-method thread -k "encode or reconstruct or apply or read or fuzz" > $T/pytest_tile$tb.log 2>&1 || { tail -30 $T/pytest_tile$tb.log; exit 1; }
  echo "tile $tb: $(tail -1 $T/pytest_tile$tb.log)"
done
for r in 1 2; do
  for tb in 16384 8192 32768 65536; do
    for c in c2enc c3e2; do
      CEC_APPLY_TILE=$tb timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $T/bench_${c}_t${tb}_$r.log 2>&1 || exit 1
      echo "tile=$tb run $r $c: $(grep -o '"kernels": {"[^"]*": {"ms": [0-9.]*' $T/bench_${c}_t${tb}_$r.log | grep -o '[0-9.]*$') ms"
    done
  done
done
