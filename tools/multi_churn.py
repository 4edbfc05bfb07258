"""Scheduler create / read / free churn on one GPU: two-shard (and one-shard) BatchReaders made,
used for a damaged read (retry rounds on the AHEAD slots' priority streams, carry ids) and freed,
`--cycles` times, in one process -- the teardown path one full GPU-suite run aborted in
(profiles/HISTORY.md, round 6).  Prints one line per cycle; exit 0 iff every read was bit-exact.

    python tools/multi_churn.py [--cycles 30]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "chunky-bits_amd"), os.path.join(ROOT, "tests"), ROOT):
    sys.path.insert(0, p)
from _stores import Locations, make_parts  # noqa: E402
from chunky_ec.batchreader import BatchReader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=30)
    args = ap.parse_args()
    d, p, L, n = 4, 2, 8192, 23
    chunks, dig = make_parts(n, d, p, L, 5)
    for c in range(args.cycles):
        st = Locations(chunks)
        rng = np.random.default_rng(c)
        for k in rng.choice(n, 6, replace=False):
            st.set(int(k), int(rng.integers(0, d)), "bad", "good")
        devices = [0, 0] if c % 3 else [0]
        r = BatchReader(d, p, L, 3, 2, devices)
        got = []
        r.read(n, st.fetch, lambda k: dig[k],
               lambda k, data: got.append(b"".join(bytes(x) for x in data)))
        ok = got == [chunks[k, :d].tobytes() for k in range(n)]
        print(f"cycle {c}: shards {len(devices)} retries {r.retries} bit-exact {ok}", flush=True)
        if not ok:
            return 1
        del r  # cec_multi_free: the workers drain, the pipelines are freed one shard at a time
    return 0


if __name__ == "__main__":
    sys.exit(main())
