#!/bin/bash
# Round-3 evidence: the format-fixture GPU tests, rocprofv3 trace + PMC of the default bench
# command (north_star block and end-to-end forms included), per-call repeat at 64/100/256.
set -o pipefail
OUT=gpurun_out/r3b
mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_format_fixture.py tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -k "format or host_buffer or present_flag" > "$OUT/pytest_fixture.log" 2>&1 && \
bash profiles/collect.sh r3_c2 --steps 10 --warmup 3 --no-cpu-baseline && \
timeout -k 10 150 ./tools/percall_bench 64 100 256 > "$OUT/percall_1.log" 2>&1 && \
timeout -k 10 150 ./tools/percall_bench 64 100 256 > "$OUT/percall_2.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_fixture.log"; grep -h pinned "$OUT"/percall_*.log
exit $rc
