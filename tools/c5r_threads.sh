# The read-repair stream's host copy threads (CEC_E2E_THREADS) at 256 GiB: does a slower fetch
# leave the host DRAM to the uploads (the fetch of a batch writes 2.7 GB into the page-locked slot
# in ~23 ms with 8 threads while the previous batch's DMA reads host memory)?
set -o pipefail
mkdir -p gpurun_out/c5r_threads
for n in 8 4 3 6; do
  CEC_E2E_THREADS=$n timeout -k 10 200 python -u bench.py --config c5r --stream-gib 256 > gpurun_out/c5r_threads/c5r_256_t$n.log 2>&1 || { tail -5 gpurun_out/c5r_threads/c5r_256_t$n.log; exit 1; }
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/c5r_threads/*.log")):
    for l in open(f):
        if l.startswith("{"):
            j = json.loads(l); r = j["read_repair"]
            print(f, j["value"], j["seconds"], r["fetch_s"], r["wait_s"], r["loop_s"])
PY
