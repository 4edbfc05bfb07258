set -euo pipefail
OUT=gpurun_out/r2d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --config c5r --stream-gib 128 --devices 0 --jobs-in-flight 3 --check > $OUT/bench_c5r_dev0_j3.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --stream-gib 128 --devices 0 --jobs-in-flight 3 > $OUT/bench_c5_dev0_j3.log 2>&1
bash profiles/collect.sh r2_c3e2 --config c3e2 --steps 3 --warmup 1 --no-cpu-baseline
echo done
