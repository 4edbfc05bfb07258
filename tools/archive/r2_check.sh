#!/bin/bash
# Round-2 GPU check: the GPU suite, smoke, and the new bench modes (each step time-limited; the
# chain stops at the first failure).  Usage: bash tools/r2_check.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/r2}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py --config c3e2 --steps 10 --warmup 2 --check > "$OUT/bench_c3e2.log" 2>&1
timeout -k 10 300 python -u bench.py --config c5 --stream-gib 64 > "$OUT/bench_c5.log" 2>&1
timeout -k 10 300 python -u bench.py --config c5 --stream-gib 64 --devices 0 > "$OUT/bench_c5_dev0.log" 2>&1
timeout -k 10 300 python -u bench.py --config c5 --stream-gib 64 --devices 0,0 > "$OUT/bench_c5_dev00.log" 2>&1
timeout -k 10 300 python -u bench.py --config c5r --stream-gib 64 --devices 0 --check > "$OUT/bench_c5r_dev0.log" 2>&1
echo "r2_check done"
