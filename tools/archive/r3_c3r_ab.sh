#!/bin/bash
# c3r (batched read: verify beside the speculative decode, which reserves 100 KiB of LDS per
# block) under the round-3 reconstruct defaults: 8 KiB tiles + compile-time d, against 16 KiB
# tiles and/or the run-time-d kernel, interleaved.
set -o pipefail
T=gpurun_out/${1:-r3_c3r_ab}
mkdir -p $T
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config c3r --no-cpu-baseline > $T/bench_c3r_$tag.log 2>&1 || exit 1
  echo "c3r $tag $(grep -o '"ms_per_step": [0-9.]*' $T/bench_c3r_$tag.log | head -1)"
}
for rep in 1 2 3; do
  run "t8k_cd1_$rep"
  run "t16k_cd1_$rep" CEC_APPLY_TILE=16384
  run "t8k_cd0_$rep" CEC_APPLY_CD=0
  run "t16k_cd0_$rep" CEC_APPLY_TILE=16384 CEC_APPLY_CD=0
  run "t32k_cd1_$rep" CEC_APPLY_TILE=32768
done
