# Round 5: the literal per-call wiring beside part_encode, and the N > 1 host copy bound under the
# job's CPU quota (no GPU work).   bash tools/r5_host_check.sh <tag>
set -o pipefail
T=gpurun_out/${1:-r5d}
mkdir -p $T
timeout -k 10 400 ./tools/percall_bench --literal 10 64 > $T/percall_literal.log 2>&1 || { tail -20 $T/percall_literal.log; exit 1; }
grep -v amdgpu.ids $T/percall_literal.log
timeout -k 10 300 python -u tools/quota_copy_bench.py --seconds 10 > $T/quota_copy.log 2>&1 || { tail -20 $T/quota_copy.log; exit 1; }
tail -1 $T/quota_copy.log
