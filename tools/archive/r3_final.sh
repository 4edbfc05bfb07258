#!/bin/bash
# Round-3 check of the tuned tree: the full check (tests, smoke, every config, stream ceilings),
# then the rocprofv3 trace + PMC passes of the default bench command.
set -o pipefail
bash tools/r3_full_check.sh ${1:-r3_full3} || exit 1
bash profiles/collect.sh ${2:-r3c_c2} --steps 10 --warmup 3 --no-cpu-baseline
