# Round-end check on one GPU box: the whole -m gpu suite, smoke(), the default bench line.
# Each step under its own time limit; stops at the first failure.
set -o pipefail
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.log" 2>&1 || { echo "bench failed"; exit 1; }
echo "bench ok"
