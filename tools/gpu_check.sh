set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u bench.py --check > gpurun_out/bench_c2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c2 --separate --no-cpu-baseline --check > gpurun_out/bench_c2sep.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c2enc --no-cpu-baseline --check > gpurun_out/bench_c2enc.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c3r --check > gpurun_out/bench_c3r.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c4 --check > gpurun_out/bench_c4.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --stream-gib 128 > gpurun_out/bench_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5r --stream-gib 128 --check > gpurun_out/bench_c5r.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench_*.log gpurun_out/smoke.log | grep -v amdgpu.ids
exit $rc
