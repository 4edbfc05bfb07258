#!/bin/bash
# LLVM scheduler-strategy A/B of the SHA-256 kernels: the product library vs
# tools/ab_sched/<strategy>/libchunky_ec.so (make -C chunky-bits_amd/csrc ab_sched SCHED=...),
# bench lines interleaved (CONFIGS, default "c2"), each build's SHA / fused GPU tests first.
#   bash tools/sched_ab.sh <outdir> [reps]
set -euo pipefail
OUT=${1:-gpurun_out/sched_ab}
REPS=${2:-2}
CONFIGS=${CONFIGS:-c2}
mkdir -p "$OUT"
VARIANTS=$(ls tools/ab_sched)
for v in $VARIANTS; do
  CEC_LIBRARY=$PWD/tools/ab_sched/$v/libchunky_ec.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sha or fused or encode_hash" > "$OUT/pytest_$v.log" 2>&1
done
for i in $(seq 1 $REPS); do
  for v in prod $VARIANTS; do
    if [ $v = prod ]; then unset CEC_LIBRARY; else export CEC_LIBRARY=$PWD/tools/ab_sched/$v/libchunky_ec.so; fi
    for c in $CONFIGS; do
      timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --check > "$OUT/${c}_${v}_$i.log" 2>&1
    done
  done
done
unset CEC_LIBRARY
echo "sched ab done"
