#!/bin/bash
# Full GPU check of the tree (round 2): the GPU suite, smoke, and the bench lines.
#   bash tools/r2_full_check.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/r2_full}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python -u bench.py > "$OUT/bench_c2.log" 2>&1
for c in c3 c3e2 c3r c4 c2enc; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --check > "$OUT/bench_$c.log" 2>&1
done
timeout -k 10 300 python -u bench.py --config c5 --stream-gib 128 > "$OUT/bench_c5.log" 2>&1
timeout -k 10 300 python -u bench.py --config c5r --stream-gib 128 --check > "$OUT/bench_c5r.log" 2>&1
echo "full check done"
