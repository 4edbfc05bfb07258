#!/usr/bin/env python3
"""Where the time of bench.py's read-repair stream goes, with and without CEC_READ_CARRY: host
seconds inside each ReadPipeline call and inside the reader's fetch (dev tool).

  python tools/carry_diag.py [gib] [sequence of 1 = carry / 0 = not, default 1010]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "chunky-bits_amd"))

import bench  # noqa: E402
import chunky_ec as ce  # noqa: E402


def timed(obj, name, acc):
    fn = getattr(obj, name)

    def wrap(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
            acc[name + "_n"] = acc.get(name + "_n", 0) + 1
    setattr(obj, name, wrap)


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 64
    import torch
    dev = torch.device("cuda", 0)
    d, p, L, P, depth = 10, 4, 1 << 20, 256, 4
    codec = ce.ReedSolomon(d, p)
    ring, ring_dig = bench.encoded_ring(codec, d, p, L, 2 * P, 0xC5C5, dev, P)
    n_parts = int(gib * (1 << 30)) // (d * L)
    copier = bench.HostCopier(8)
    seq = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "1010")]
    for carry in seq:
        flags = ce.ReadPipeline.REBUILT_ONLY | (ce.ReadPipeline.CARRY if carry else 0)
        rp = ce.ReadPipeline(codec, L, P, depth, flags)
        acc = {}
        for name in ("wait", "submit", "submit_carried", "acquire", "carry_ids"):
            timed(rp, name, acc)
        el, stats, _ = bench.timed_read_repair(codec, ring, ring_dig, L, P, depth, 0, n_parts, 1,
                                               0.01, copier, 0x5EED, rp=rp)
        out = {"carry": carry, "GBs": round(n_parts * d * L / el / 1e9, 2), "seconds": round(el, 3)}
        out.update({k: (round(v, 3) if isinstance(v, float) else v) for k, v in acc.items()})
        print(json.dumps(out), flush=True)
        for name in ("wait", "submit", "submit_carried", "acquire", "carry_ids"):
            delattr(rp, name)  # the wrappers hold rp: free it here, not at a gc mid-run
        del rp
    copier.close()


if __name__ == "__main__":
    main()
