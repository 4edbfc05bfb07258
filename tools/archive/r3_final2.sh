#!/bin/bash
# Final check of the round-3 tree: the full check (tests, smoke, every config) and the 4-rank
# gloo rehearsal of the N > 1 line.
set -o pipefail
bash tools/r3_full_check.sh ${1:-r3_full4} || exit 1
bash tools/r3_n4.sh ${2:-r3_n4b}
