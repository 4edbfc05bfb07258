#!/bin/bash
# rocprofv3 kernel + memory-copy trace of the c5r read stream (per-run and packed uploads):
# where the link time goes between batches.
#   bash tools/r2_c5r_trace.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/r2_c5r_trace}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/runs" -o run -- \
    python3 bench.py --config c5r --stream-gib 32 > "$OUT/bench_runs.log" 2>&1
CEC_C5R_PACKED=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/packed" -o run -- \
    python3 bench.py --config c5r --stream-gib 32 > "$OUT/bench_packed.log" 2>&1
echo "trace done"
