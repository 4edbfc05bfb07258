#!/bin/bash
# Which part of stream-ordered allocation loses data under running kernels: the free queued
# behind the work (default) vs the free after a sync (control), and the default pool's release
# threshold (0: trims at sync points) vs max (keeps freed memory).
set -o pipefail
OUT=gpurun_out/r3_repro3
mkdir -p "$OUT"
for cfg in "stream default" "late default" "stream max"; do
  set -- $cfg
  for m in same independent join; do
    reps=4000; [ $m = join ] && reps=400
    REPRO_FILL=kernel REPRO_PINNED=1 REPRO_FREE=$1 REPRO_THRESHOLD=$2 timeout -k 10 120 ./tools/repro_free_async $m 12 $reps > "$OUT/${m}_$1_$2.log" 2>&1
    rc=$?
    echo "free=$1 threshold=$2: $(tail -1 "$OUT/${m}_$1_$2.log")"
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
  done
done
uname -r > "$OUT/host.txt"; cat /sys/module/amdgpu/version >> "$OUT/host.txt" 2>/dev/null; /opt/rocm/bin/rocminfo 2>/dev/null | grep -m3 -E "Runtime Version|Marketing|gfx" >> "$OUT/host.txt"
exit 0
