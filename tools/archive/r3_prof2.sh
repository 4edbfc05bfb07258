#!/bin/bash
# After the bit-sliced encoder (8 KiB tiles): the apply/encode GPU tests, the rocprofv3 trace +
# PMC of the default bench command (north_star encode now rs_encode_bs_kernel), and the
# encode-only configs with the oracle check.
set -o pipefail
OUT=gpurun_out/r3c
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash profiles/collect.sh r3c_c2 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
for c in c2enc c4enc; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --check > $OUT/bench_$c.log 2>&1 || exit 1
  echo "$c: $(grep -o '"kernels": {"[^"]*": {"ms": [0-9.]*' $OUT/bench_$c.log) $(grep -o '"frac": [0-9.]*' $OUT/bench_$c.log | head -1) $(grep -o '"check[a-z_]*": [a-z]*' $OUT/bench_$c.log | head -1)"
done
grep -o '"north_star": {"encode": {[^}]*}' gpurun_out/prof_r3c_c2/trace_bench.log
