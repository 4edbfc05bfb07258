#!/bin/bash
# 4-rank gloo rehearsal of the N > 1 bench line on the one-GPU box (the per-rank array).
set -o pipefail
OUT=gpurun_out/${1:-r3_n4}
mkdir -p "$OUT"
CEC_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 4 \
  --parts 1024 --e2e-gib 16 > "$OUT/bench_n4.log" 2>&1
rc=$?
grep -v amdgpu.ids "$OUT/bench_n4.log" | tail -5
exit $rc
