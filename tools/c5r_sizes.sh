# The read-repair stream (bench.py --config c5r) at several sizes, and once with no damage: the
# fit time = fixed + bytes / rate separates the stream's start and tail from its steady rate.
set -o pipefail
mkdir -p gpurun_out/c5r_sizes
for g in 16 64 256; do
  timeout -k 10 240 python -u bench.py --config c5r --stream-gib $g > gpurun_out/c5r_sizes/c5r_$g.log 2>&1 || { tail -5 gpurun_out/c5r_sizes/c5r_$g.log; exit 1; }
done
timeout -k 10 240 python -u bench.py --config c5r --stream-gib 64 --corrupt 0 > gpurun_out/c5r_sizes/c5r_64_clean.log 2>&1 || exit 1
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/c5r_sizes/*.log")):
    for l in open(f):
        if l.startswith("{"):
            j = json.loads(l); r = j["read_repair"]
            print(f, j["value"], j["seconds"], j["config"]["stream_bytes"], r["batches"], r["retry_batches"],
                  r["chunks_loaded"], r["fetch_s"], r["wait_s"], r["loop_s"])
PY
