#!/bin/bash
# Repeat the ordering-sensitive suites to look for timing-dependent failures.
set -uo pipefail
OUT=${1:-gpurun_out/r2_repeat}
mkdir -p "$OUT"
for i in 1 2 3 4 5; do
  timeout -k 10 300 ./tests/cpp/reference_mirror_test > "$OUT/mirror_$i.log" 2>&1
  rc=$?; echo "mirror $i rc=$rc" >> "$OUT/summary.txt"
  [ $rc -gt 1 ] && exit $rc
done
for i in 1 2; do
  timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_stress.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread > "$OUT/pytest_$i.log" 2>&1
  rc=$?; echo "pytest $i rc=$rc $(tail -n 1 $OUT/pytest_$i.log)" >> "$OUT/summary.txt"
  [ $rc -gt 1 ] && exit $rc
done
echo "repeat done"
exit 0
