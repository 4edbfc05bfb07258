#!/bin/bash
# The default bench line with BASELINE's C3 / C4 configurations in it, and the c3 config alone
# (its erasure sets now come from the same helper) checked against the oracle.
set -o pipefail
T=gpurun_out/${1:-r3_bcfg}
mkdir -p $T
timeout -k 10 300 python -u bench.py > $T/bench_c2.log 2>&1 || { tail -30 $T/bench_c2.log; exit 1; }
timeout -k 10 200 python -u bench.py --config c3 --check --no-cpu-baseline > $T/bench_c3.log 2>&1 || { tail -30 $T/bench_c3.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"check_vs_oracle": [a-z]*' $T/bench_c3.log
