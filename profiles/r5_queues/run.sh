# Slot streams on their own hardware queues (CEC_SLOT_QUEUES) A/B (dev tool): the read-repair
# stream with and without carry, the queue each slot stream landed on, and bench c5r.
set -euo pipefail
OUT=gpurun_out/r5n
mkdir -p $OUT
export TMPDIR=/tmp
for q in 0 1; do
  CEC_SLOT_QUEUES=$q timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
      -d $OUT/q$q -o run -- python3 tools/carry_diag.py 24 1010 > $OUT/diag_q$q.log 2>&1
  grep carry $OUT/diag_q$q.log
done
for q in 1 0; do
  for c in 1 0; do
    CEC_SLOT_QUEUES=$q CEC_BENCH_CARRY=$c timeout -k 10 240 python3 bench.py --config c5r > $OUT/c5r_q${q}_c$c.log 2>&1
    echo "q=$q carry=$c $(grep -o '"value": [0-9.]*' $OUT/c5r_q${q}_c$c.log | head -1)"
  done
done
