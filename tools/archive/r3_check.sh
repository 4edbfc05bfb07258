#!/bin/bash
# Round-3 check: GPU suite, the default bench line (north_star block, end-to-end forms), the
# per-call tier at 64/100/256 callers (device-side wait for the early parity download).
set -o pipefail
OUT=${1:-gpurun_out/r3}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python -u bench.py --check > "$OUT/bench_c2.log" 2>&1 && \
timeout -k 10 150 ./tools/percall_bench 10 64 100 256 > "$OUT/percall.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"; grep -v amdgpu.ids "$OUT/bench_c2.log" | tail -3; cat "$OUT/percall.log" 2>/dev/null | tail -12
exit $rc
