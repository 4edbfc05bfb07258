#!/usr/bin/env python3
"""Make, use and free read pipelines one after another and time each (dev tool): whether slot
streams on their own hardware queues (CEC_SLOT_QUEUES=1) slow down as pipelines come and go.

  python tools/queue_churn.py [n_pipelines] [live]   (live: how many are kept alive at once)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chunky-bits_amd"))

import numpy as np  # noqa: E402
import chunky_ec as ce  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    live = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    d, p, L, P, depth = 4, 2, 4096, 8, 4
    codec = ce.ReedSolomon(d, p)
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, (P, d, L), dtype=np.uint8)
    par = [bytearray(L) for _ in range(p)]
    kept = []
    for k in range(n):
        t0 = time.perf_counter()
        rp = ce.ReadPipeline(codec, L, P, depth, ce.ReadPipeline.REBUILT_ONLY)
        t1 = time.perf_counter()
        for _ in range(2 * depth):
            slot, chunks, present, expected = rp.acquire()
            chunks[:, :d] = data
            present[:] = 0
            present[:, :d] = 1
            expected[:] = 0  # every chunk fails verification: exercises the redo path too
            rp.submit(slot, P)
            rp.wait(slot)
        rp.drain()
        t2 = time.perf_counter()
        kept.append(rp)
        if len(kept) > live:
            kept.pop(0)
        print(json.dumps({"pipeline": k, "make_ms": round(1e3 * (t1 - t0), 2),
                          "use_ms": round(1e3 * (t2 - t1), 2)}), flush=True)
    del par


if __name__ == "__main__":
    main()
