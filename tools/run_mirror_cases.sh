#!/bin/bash
# Runs reference_mirror_test cases one per process (dev aid); stops at a crash or timeout.
#   bash tools/run_mirror_cases.sh <outdir> case...
OUT=$1; shift
mkdir -p "$OUT"
for c in "$@"; do
  timeout -k 10 120 ./tests/cpp/reference_mirror_test "$c" > "$OUT/$c.log" 2>&1
  rc=$?
  echo "rc=$rc" >> "$OUT/$c.log"
  if [ $rc -gt 1 ]; then echo "stopping after $c (rc=$rc)"; exit $rc; fi
done
echo "cases done"
