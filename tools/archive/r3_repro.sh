#!/bin/bash
# Stream-order checks with no engine code: allocation reuse across streams
# (independent / event / same) and round 2's read-path fork/join shape (join); fills by
# hipMemsetD32Async or by a kernel, host buffers pageable or page-locked.
set -o pipefail
OUT=gpurun_out/r3_repro2
mkdir -p "$OUT"
for fillm in memset kernel; do
  for pin in 0 1; do
    for m in same independent join; do
      reps=4000; [ $m = join ] && reps=400
      REPRO_FILL=$fillm REPRO_PINNED=$pin timeout -k 10 120 ./tools/repro_free_async $m 12 $reps > "$OUT/${m}_${fillm}_pin${pin}.log" 2>&1
      rc=$?
      echo "$fillm pinned=$pin: $(tail -1 "$OUT/${m}_${fillm}_pin${pin}.log")"
      if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
    done
  done
done
exit 0
