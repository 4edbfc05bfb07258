#!/bin/bash
# Freshly mapped device memory written right after allocation: hipMallocAsync after a pool trim,
# and hipMalloc; fills by kernel and by hipMemsetD32Async; round 2's join shape once more.
set -o pipefail
OUT=gpurun_out/r3_repro4
mkdir -p "$OUT"
uname -r > "$OUT/host.txt"
for a in async sync; do
  for f in kernel memset; do
    REPRO_ALLOC=$a REPRO_FILL=$f REPRO_PINNED=1 timeout -k 10 120 ./tools/repro_free_async fresh 16 2000 > "$OUT/fresh_${a}_${f}.log" 2>&1
    rc=$?
    echo "fill=$f: $(tail -1 "$OUT/fresh_${a}_${f}.log")"
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  done
done
REPRO_FILL=kernel REPRO_PINNED=1 timeout -k 10 120 ./tools/repro_free_async join 12 400 > "$OUT/join.log" 2>&1
echo "$(tail -1 "$OUT/join.log")"
exit 0
