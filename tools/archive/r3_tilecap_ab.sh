#!/bin/bash
# Column tile x residency cap for the GF kernels under the round-3 defaults (caps, compile-time-d
# reconstruct), interleaved on one box.
set -o pipefail
T=gpurun_out/${1:-r3_tilecap_ab}
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 150 --timeout-method thread -k "reconstruct or encode or split or read" > $T/pytest.log 2>&1 || { tail -30 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
run() {  # tag config env...
  local tag=$1 c=$2; shift 2
  env "$@" timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline > $T/bench_${c}_$tag.log 2>&1 || exit 1
  echo "$c $tag $(grep -o '"ms_per_step": [0-9.]*' $T/bench_${c}_$tag.log | head -1)"
}
for rep in 1 2 3; do
  for tile in 8192 16384 32768; do
    for cap in 2 3; do
      run "t${tile}_cap${cap}_$rep" c2enc CEC_APPLY_TILE=$tile CEC_APPLY_BLOCKS_PER_CU=$cap
      run "t${tile}_cap${cap}_$rep" c3e2 CEC_APPLY_TILE=$tile CEC_APPLY_BLOCKS_PER_CU=$cap
    done
    run "t${tile}_$rep" c3 CEC_APPLY_TILE=$tile
  done
done
timeout -k 10 120 ./tools/ubench_stream 4096 c > $T/ubench_caps.log 2>&1 || exit 1
cat $T/ubench_caps.log
