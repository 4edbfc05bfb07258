#!/bin/bash
# 4-rank gloo rehearsal of the headline bench on one GPU (1024 parts per rank): the N>1 path
# (barriers, max over ranks, the end-to-end figure on every rank).
set -euo pipefail
OUT=${1:-gpurun_out/r2_n4}
mkdir -p "$OUT"
CEC_BENCH_BACKEND=gloo timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --parts 1024 --e2e-gib 16 > "$OUT/bench_c2_n4_gloo.log" 2>&1
echo "n4 done"
