#!/bin/bash
# c5r traced with the shared upload stream (CEC_READ_UPSTREAM=1), packed uploads; and C5 write
# traced for comparison.
set -euo pipefail
OUT=${1:-gpurun_out/r2_c5r_trace2}
mkdir -p "$OUT"
export TMPDIR=/tmp
CEC_READ_UPSTREAM=1 CEC_C5R_PACKED=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/up" -o run -- \
    python3 bench.py --config c5r --stream-gib 32 > "$OUT/bench_up.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/c5" -o run -- \
    python3 bench.py --config c5 --stream-gib 32 > "$OUT/bench_c5.log" 2>&1
echo "trace2 done"
