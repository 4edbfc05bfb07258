set -o pipefail
mkdir -p gpurun_out/r4d
for c in c2enc c3 c3e2 c3r c4 c4enc c1enc; do
  timeout -k 10 150 python -u bench.py --config $c --check > gpurun_out/r4d/bench_$c.log 2>&1 || { echo "fail $c"; exit 1; }
  echo "done $c"
done
timeout -k 10 200 python -u bench.py > gpurun_out/r4d/bench_c2.log 2>&1 && echo done c2
