# Device-side carry stash (dev tool): the read-stream GPU tests, then c5r with and without carry
# on plain slot streams, alternating.
set -o pipefail
OUT=gpurun_out/r5s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_readstream.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_readstream.log 2>&1 || { tail -30 $OUT/pytest_readstream.log; exit 1; }
tail -1 $OUT/pytest_readstream.log
for r in 1 2; do
  for c in 1 0; do
    CEC_BENCH_CARRY=$c timeout -k 10 240 python3 bench.py --config c5r > $OUT/c5r_c${c}_$r.log 2>&1 || { tail -20 $OUT/c5r_c${c}_$r.log; exit 1; }
    echo "carry=$c run=$r $(grep -o '"value": [0-9.]*' $OUT/c5r_c${c}_$r.log | head -1)"
  done
done
