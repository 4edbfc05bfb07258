# Kernel + memory-copy trace of the c5r stream with and without CEC_READ_CARRY (dev tool).
set -euo pipefail
OUT=gpurun_out/r5l
mkdir -p $OUT
export TMPDIR=/tmp
for c in 1 0; do
  CEC_BENCH_CARRY=$c timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
      -d $OUT/carry$c -o run -- python3 bench.py --config c5r --stream-gib 64 > $OUT/carry$c.log 2>&1
  grep -o '"value": [0-9.]*' $OUT/carry$c.log | head -1
done
