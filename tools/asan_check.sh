# The C++ mirror test against the host-AddressSanitizer build of the library
# (make -C chunky-bits_amd/csrc asan; remove ./tools/asan from .gpurunignore to ship it): heap / stack errors in the host code of the C-ABI, the
# pipelines and the scheduler (one- and two-shard schedulers made and freed) on a real GPU.
# Device code is not instrumented.  Leak checking is off: the HIP runtime keeps its allocations to
# process exit.
set -o pipefail
mkdir -p gpurun_out/asan
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1 timeout -k 10 600 \
    ./tools/asan/reference_mirror_test > gpurun_out/asan/mirror_asan.log 2>&1
s=$?
tail -25 gpurun_out/asan/mirror_asan.log
# The HIP runtime's own finalizer trips an AddressSanitizer CHECK at process exit
# (sanitizer_allocator_device.h, "dev_runtime_unloaded_"), after main has returned: judge the run
# by the tests' verdict and the absence of an ASan error report instead of the exit status.
grep -q "^all passed" gpurun_out/asan/mirror_asan.log || exit 1
! grep -q "ERROR: AddressSanitizer" gpurun_out/asan/mirror_asan.log
