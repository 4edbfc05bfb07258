#!/bin/bash
# Round-3 full check: the -m gpu suite, smoke, every bench config, and the scheduler's pageable
# path with 8 copy threads (A/B against the default 4).
#   bash tools/r3_full_check.sh <tag>      (logs under gpurun_out/<tag>/)
set -o pipefail
T=gpurun_out/${1:-r3_full}
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { tail -40 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $T/bench_c2.log 2>&1 || exit 1
for c in c2enc c3 c3e2 c3r c4; do
  timeout -k 10 300 python -u bench.py --config $c --check --no-cpu-baseline > $T/bench_$c.log 2>&1 || exit 1
done
for c in c5 c5r; do
  timeout -k 10 300 python -u bench.py --config $c --stream-gib 128 --check > $T/bench_$c.log 2>&1 || exit 1
done
CEC_MULTI_COPY_THREADS=8 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-north-star > $T/bench_c2_copy8.log 2>&1 || exit 1
timeout -k 10 120 ./tools/ubench_stream 4096 m > $T/ubench_mix.log 2>&1 || exit 1
timeout -k 10 120 ./tools/ubench_stream 4096 x > $T/ubench_w_xcd.log 2>&1 || exit 1
cat $T/ubench_w_xcd.log
cat $T/ubench_mix.log
grep -v amdgpu.ids $T/smoke.log
for c in c2 c2enc c3 c3e2 c3r c4 c5 c5r c2_copy8; do grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"check[a-z_]*": [a-z]*' $T/bench_$c.log | tr '\n' ' '; echo " $c"; done
