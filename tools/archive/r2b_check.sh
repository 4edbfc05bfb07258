set -euo pipefail
OUT=gpurun_out/r2b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread > $OUT/t_multi.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --stream-gib 128 --devices 0 > $OUT/bench_c5_dev0.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --stream-gib 128 --devices 0,0 > $OUT/bench_c5_dev00.log 2>&1
timeout -k 10 300 python -u bench.py --config c5r --stream-gib 128 --devices 0 --check > $OUT/bench_c5r_dev0.log 2>&1
timeout -k 10 300 python -u bench.py --config c5r --stream-gib 128 > $OUT/bench_c5r.log 2>&1
timeout -k 10 200 tools/percall_bench 10 > $OUT/percall_if1.log 2>&1
CEC_COALESCE_INFLIGHT=2 timeout -k 10 200 tools/percall_bench 10 100 > $OUT/percall_if2.log 2>&1
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- tools/ubench_fetch > $OUT/ubench_fetch.log 2>&1
echo done
