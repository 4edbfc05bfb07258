#!/bin/bash
# Collect rocprofv3 evidence for the bench on a GPU box:
#   profiles/collect.sh <tag> [bench args...]
# Writes raw output under gpurun_out/prof_<tag>/ ; summaries are copied into profiles/ by hand.
# Kernel trace + stats first, then PMC passes in separate runs (never combined with tracing
# of other domains).  Each run is time-limited; the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r1}; shift || true
ARGS=${@:-"--steps 3 --warmup 1 --no-cpu-baseline"}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
echo "python3 bench.py $ARGS" > "$OUT/command.txt"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/trace_bench.log" 2>&1
echo "trace pass done" >> "$OUT/progress.txt"
# SQ counters: issue / waves / cycles (one pass)
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py $ARGS > "$OUT/pmc_sq.log" 2>&1
echo "sq pass done" >> "$OUT/progress.txt"
# HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slot limits)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 bench.py $ARGS > "$OUT/pmc_write.log" 2>&1
echo "collected into $OUT"
