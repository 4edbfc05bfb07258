#!/bin/bash
# Stream-ordered allocation reuse: does hipMallocAsync on another stream get memory whose
# hipFreeAsync is queued behind a kernel still reading it?  
set -o pipefail
OUT=gpurun_out/r3_repro
mkdir -p "$OUT"
for m in independent event same join; do
  timeout -k 10 120 ./tools/repro_free_async $m 20 $([ $m = join ] && echo 400 || echo 4000) > "$OUT/$m.log" 2>&1
  rc=$?
  tail -1 "$OUT/$m.log"
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
done
exit 0
