#!/bin/bash
# rocprofv3 evidence for every bench config of a round: profiles/collect.sh per config.
#   bash tools/profile_round.sh <round-tag>
set -euo pipefail
R=${1:-r1d}
bash profiles/collect.sh ${R}_c2 --config c2 --steps 3 --warmup 1 --no-cpu-baseline
bash profiles/collect.sh ${R}_c2enc --config c2enc --steps 3 --warmup 1 --no-cpu-baseline
bash profiles/collect.sh ${R}_c3 --config c3 --steps 3 --warmup 1 --no-cpu-baseline
bash profiles/collect.sh ${R}_c4 --config c4 --steps 3 --warmup 1 --no-cpu-baseline
echo done
