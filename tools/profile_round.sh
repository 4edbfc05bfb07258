#!/bin/bash
# rocprofv3 evidence for bench configs of a round: profiles/collect.sh per config.
#   bash tools/profile_round.sh <round-tag> [configs...]   (default: c2 c2enc c3 c4)
set -euo pipefail
R=${1:-r1d}; shift || true
CONFIGS=${@:-"c2 c2enc c3 c4"}
for c in $CONFIGS; do
  bash profiles/collect.sh ${R}_${c} --config $c --steps 3 --warmup 1 --no-cpu-baseline
done
echo done
