# Round 5: location-walk loops on the GPU (new tests + the drop-in store), then the early check.
set -o pipefail
T=gpurun_out/${1:-r5b}
mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_gpu_batchreader.py tests/test_gpu_batchcheck.py tests/test_gpu_dropin.py tests/test_cpp_mirror.py -x -v --timeout 150 --timeout-method thread > $T/pytest_loc.log 2>&1 || { tail -60 $T/pytest_loc.log; exit 1; }
tail -3 $T/pytest_loc.log
timeout -k 10 200 python -u tools/dropin_cp_repair.py gpurun_out/dropin > $T/dropin.log 2>&1 || { tail -30 $T/dropin.log; exit 1; }
bash tools/early_check.sh ${1:-r5b}_early
