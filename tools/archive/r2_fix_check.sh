#!/bin/bash
# After the scratch-pool fix: the C++ mirror twice, the GPU suite, cp_bench.
set -euo pipefail
OUT=${1:-gpurun_out/r2_fix}
mkdir -p "$OUT"
timeout -k 10 300 ./tests/cpp/reference_mirror_test > "$OUT/mirror1.log" 2>&1
timeout -k 10 300 ./tests/cpp/reference_mirror_test > "$OUT/mirror2.log" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 ./tools/cp_bench 4 > "$OUT/cp_bench.log" 2>&1
timeout -k 10 300 ./tools/cp_bench 4 0,0 > "$OUT/cp_bench_2shards.log" 2>&1
echo "fix check done"
