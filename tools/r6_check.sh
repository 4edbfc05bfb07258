# Round-6 check of the final tree on one GPU box (logs under gpurun_out/<tag>/): the -m gpu suite,
# smoke(), the default bench line, a kernel trace of the default command, C5 verify/repair over
# 1 TiB (the read pipeline changed this round), tools/cp_bench's damaged read with and without
# carry (1 shard at 24 GiB, 2 shards at 8 GiB), and a 4-rank gloo rehearsal of `bench.py --gpus 4` starting
# its own ranks.  Each step under its own time limit; stops at the first failure.
#   bash tools/r6_check.sh <tag>
set -o pipefail
T=gpurun_out/${1:-r6final}
mkdir -p "$T"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
    > "$T/pytest_gpu.log" 2>&1 || { tail -30 "$T/pytest_gpu.log"; exit 1; }
tail -1 "$T/pytest_gpu.log"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$T/smoke.log" 2>&1 \
    || { tail -20 "$T/smoke.log"; exit 1; }
timeout -k 10 300 python -u bench.py > "$T/bench_default.log" 2>&1 || { tail -20 "$T/bench_default.log"; exit 1; }
echo "default line done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$T/trace" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$T/trace_bench.log" 2>&1 \
    || { tail -20 "$T/trace_bench.log"; exit 1; }
echo "trace done"
timeout -k 10 300 python -u bench.py --config c5r > "$T/bench_c5r.log" 2>&1 || { tail -20 "$T/bench_c5r.log"; exit 1; }
timeout -k 10 300 ./tools/cp_bench 24 0 0.01 > "$T/cp_bench_24g_1shard.log" 2>&1 || { tail "$T/cp_bench_24g_1shard.log"; exit 1; }
timeout -k 10 250 ./tools/cp_bench 8 0,0 0.01 > "$T/cp_bench_2shards.log" 2>&1 || { tail "$T/cp_bench_2shards.log"; exit 1; }
CEC_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 4 --parts 1024 --steps 3 \
    --warmup 1 --e2e-gib 0 > "$T/bench_gpus4_gloo.json" 2> "$T/bench_gpus4_gloo.err" \
    || { tail -20 "$T/bench_gpus4_gloo.err"; exit 1; }
echo "all done"
