set -euo pipefail
OUT=gpurun_out/r2c; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread > $OUT/t_multi.log 2>&1
for dv in 0 0,0 0,0,0,0; do
  timeout -k 10 300 python -u bench.py --config c5 --stream-gib 128 --devices $dv > $OUT/bench_c5_dev$dv.log 2>&1
  timeout -k 10 300 python -u bench.py --config c5r --stream-gib 128 --devices $dv --check > $OUT/bench_c5r_dev$dv.log 2>&1
done
echo done
