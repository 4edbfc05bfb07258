"""CPU side of the per-call comparison (dev tool): the oracle's restatement of the crate path
(scalar galois_8 encode_sep + SHA-NI SHA-256 of all d+p chunks, one part per task) on T host
threads -- the reference's own shape at `concurrency` T (writer.rs:130).

python tools/cpu_percall_baseline.py [threads...]   (default 1 10 16)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

d, p, L = 10, 4, 1 << 20
for t in [int(x) for x in sys.argv[1:]] or [1, 10, 16]:
    parts = max(2 * t, 8)
    sec = oracle.baseline_encode_sha(d, p, L, parts, 2, t, True, True)
    print(f"cpu part_encode RS(10,4) 1 MiB, {t:3d} thread(s): {parts * d * L / sec / 1e9:6.2f} GB/s "
          f"of data ({parts} parts, {sec:.2f} s, SHA-NI={'yes' if oracle.has_shani() else 'no'})",
          flush=True)
