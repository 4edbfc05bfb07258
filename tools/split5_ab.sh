set -euo pipefail
mkdir -p gpurun_out/split5
timeout -k 10 90 python -u tools/sha_ab.py --parts 64 --chunk 1000 --variants 1,9,10 --rounds 1 > gpurun_out/split5/small.log 2>&1
timeout -k 10 90 python -u tools/sha_ab.py --parts 300 --chunk 65536 --variants 1,9,10 --rounds 1 >> gpurun_out/split5/small.log 2>&1
timeout -k 10 200 python -u tools/sha_ab.py --parts 4096 --variants 1,4,9,10 --rounds 3 > gpurun_out/split5/c2.log 2>&1
