#!/bin/bash
# Per-call tier: early parity download waiting on the device vs on the host, interleaved on one
# box (pinned and pageable callers at 64 / 100 / 256), plus the two ordering regression tests.
set -o pipefail
OUT=gpurun_out/r3_d2h_ab
mkdir -p "$OUT"
for r in 1 2; do
  for w in device host; do
    echo "== wait=$w run $r" >> "$OUT/percall.log"
    CEC_COALESCE_D2H_WAIT=$w timeout -k 10 150 ./tools/percall_bench 64 100 256 >> "$OUT/percall.log" 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_stress.py -m gpu -x -v --timeout 150 --timeout-method thread -k "two_batches_in_flight or many_streams or three_keys" > "$OUT/pytest_order.log" 2>&1
rc=$?
grep -E "==|pinned|pageable" "$OUT/percall.log"; tail -3 "$OUT/pytest_order.log"
exit $rc
