# HIP API + kernel + copy trace of the first CEC_READ_CARRY pipeline in a process (dev tool):
# where the host blocks in the slow first carry run.
set -euo pipefail
OUT=gpurun_out/r5m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv \
    -d $OUT/api -o run -- python3 tools/carry_diag.py 24 10 > $OUT/api.log 2>&1
grep carry $OUT/api.log
