# The C++ mirror test against the host-AddressSanitizer build of the library
# (make -C chunky-bits_amd/csrc asan): heap / stack errors in the host code of the C-ABI, the
# pipelines and the scheduler (one- and two-shard schedulers made and freed) on a real GPU.
# Device code is not instrumented.  Leak checking is off: the HIP runtime keeps its allocations to
# process exit.
set -o pipefail
mkdir -p gpurun_out/asan
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1 timeout -k 10 600 \
    ./tools/asan/reference_mirror_test > gpurun_out/asan/mirror_asan.log 2>&1
s=$?
tail -25 gpurun_out/asan/mirror_asan.log
exit $s
