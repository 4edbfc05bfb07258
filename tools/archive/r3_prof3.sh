#!/bin/bash
# rocprofv3 trace + PMC of the GF configs on the round-3 kernels (bit-sliced encode, capped
# reconstruct classes), for profiles/traffic.json.
set -o pipefail
bash profiles/collect.sh r3c_c2enc --config c2enc --steps 5 --warmup 1 --no-cpu-baseline && \
bash profiles/collect.sh r3c_c3 --config c3 --steps 5 --warmup 1 --no-cpu-baseline && \
bash profiles/collect.sh r3c_c3e2 --config c3e2 --steps 5 --warmup 1 --no-cpu-baseline
