# Early-round GPU check: the -m gpu suite, smoke, the default bench line.
#   bash tools/early_check.sh <tag>      (logs under gpurun_out/<tag>/)
set -o pipefail
T=gpurun_out/${1:-r5a}
mkdir -p $T
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $T/pytest_gpu.log 2>&1 || { tail -40 $T/pytest_gpu.log; exit 1; }
tail -1 $T/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.log 2>&1 || { cat $T/smoke.log; exit 1; }
grep -v amdgpu.ids $T/smoke.log
timeout -k 10 300 python -u bench.py > $T/bench.log 2>&1 || { tail -30 $T/bench.log; exit 1; }
tail -c 1500 $T/bench.log
