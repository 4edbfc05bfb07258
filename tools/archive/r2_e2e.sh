#!/bin/bash
# Headline bench with the end-to-end (PCIe-inclusive) figure: N=1, then a 2-rank gloo rehearsal
# of the N>1 path on one GPU.
#   bash tools/r2_e2e.sh <outdir>
set -euo pipefail
OUT=${1:-gpurun_out/r2_e2e}
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py > "$OUT/bench_c2.log" 2>&1
CEC_BENCH_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 > "$OUT/bench_c2_n2_gloo.log" 2>&1
echo "e2e done"
