# Round check on the GPU box: full -m gpu suite, then the measurements touched this round.
#   bash tools/round_check.sh <tag>      (logs under gpurun_out/<tag>/)
set -o pipefail
T=gpurun_out/${1:-r1y}
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { tail -40 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
timeout -k 10 200 ./tools/percall_bench > $T/percall.log 2>&1 || exit 1
for parts in 1 10 256 1024; do
  echo "parts=$parts" >> $T/sha_ab_small.log
  timeout -k 10 120 python -u tools/sha_ab.py --parts $parts --variants 1,2 >> $T/sha_ab_small.log 2>&1 || exit 1
done
for c in c2 c3r c5 c5r; do
  extra=""; [ $c = c5 -o $c = c5r ] && extra="--stream-gib 128"
  timeout -k 10 300 python -u bench.py --config $c --check $extra > $T/bench_$c.log 2>&1 || exit 1
done
cat $T/percall.log $T/sha_ab_small.log | grep -v amdgpu.ids
for c in c2 c3r c5 c5r; do grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"check[a-z_]*": [a-z]*' $T/bench_$c.log | tr '\n' ' '; echo " $c"; done
