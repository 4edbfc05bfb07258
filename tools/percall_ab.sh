# Per-call tier A/B on one box, interleaved runs of tools/percall_bench under env settings.
#   bash tools/percall_ab.sh <out-log> "ENV=.. ENV=..;ENV=..;..." [rounds]
set -o pipefail
OUT=${1:-gpurun_out/percall_ab.log}
IFS=';' read -ra SETS <<< "${2:-CEC_COALESCE_INFLIGHT=1;CEC_COALESCE_INFLIGHT=4}"
mkdir -p $(dirname $OUT)
for r in $(seq ${3:-2}); do
  for e in "${SETS[@]}"; do
    echo "== $e (run $r)" >> $OUT
    env $e timeout -k 10 200 ./tools/percall_bench >> $OUT 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $OUT | grep -o '^==.*\|^part_encode.*'
