# HIP hardware queues per process (GPU_MAX_HW_QUEUES, 4 by default): with 4 the null stream takes
# one and the read pipeline's 4 slot streams share the other 3 (profiles/r6/trace_c5r: two slots'
# SHA-256 kernels on one queue run one after the other).  The read-repair stream and the C++
# drop-in read with 1 % damaged copies, at the default and at 8 queues.
set -o pipefail
mkdir -p gpurun_out/hwq
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --config c5r --stream-gib 64 > gpurun_out/hwq/c5r_64_q$q.log 2>&1 || { tail -5 gpurun_out/hwq/c5r_64_q$q.log; exit 1; }
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 ./tools/cp_bench 24 0 0.01 > gpurun_out/hwq/cp_bench_24g_q$q.log 2>&1 || { tail -5 gpurun_out/hwq/cp_bench_24g_q$q.log; exit 1; }
done
for f in gpurun_out/hwq/c5r*.log; do echo "$f $(grep -o '"value": [0-9.]*\|"seconds": [0-9.]*' $f | tr '\n' ' ')"; done
for f in gpurun_out/hwq/cp*.log; do echo "== $f"; grep -i "GB/s" $f | tail -6; done
