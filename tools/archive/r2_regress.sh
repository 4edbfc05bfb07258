#!/bin/bash
# Bench lines touched by the scratch-pool change (read / reconstruct paths, per-call tier).
set -euo pipefail
OUT=${1:-gpurun_out/r2_regress}
mkdir -p "$OUT"
for c in c3 c3e2 c3r; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --check > "$OUT/bench_$c.log" 2>&1
done
timeout -k 10 300 python -u bench.py --config c5r --stream-gib 64 --check > "$OUT/bench_c5r.log" 2>&1
timeout -k 10 300 ./tools/percall_bench 10 100 256 > "$OUT/percall.log" 2>&1
echo "regress done"
