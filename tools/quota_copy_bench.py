#!/usr/bin/env python3
"""Host-side bound of the N > 1 end-to-end legs under the job's CPU quota: the
reader's copy -- a pageable source ring copied part by part into the part buffers by a rank's host
threads (bench.py's ring_reader / HostCopier) -- run by N processes at once, as N ranks would on
one node, with NO GPU work, for each thread sizing:

  python tools/quota_copy_bench.py [--seconds 8] [--ring-gib 1]

  1 x 8      one rank, 8 threads (the N = 1 line's sizing)
  8 x quota  8 ranks, each with sharding.rank_threads(8) threads (its quota share less one)
  8 x 8      8 ranks x 8 threads (the round-4 sizing, which ignored the quota)

Prints one JSON line: the aggregate copy rate of each case (GB/s of part bytes written), the
cgroup quota, the affinity, and the per-process rates.  The destinations are pageable buffers,
first-touched before timing (a page-locked destination, cec_host_alloc, is the same DRAM write;
this tool keeps the GPU out of the measurement)."""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chunky-bits_amd", "chunky_ec"))

PART = 10 << 20  # one RS(10,4) part of 1 MiB chunks


def _worker(threads, seconds, ring_gib, start, out_q):
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    n_ring = max(2, int(ring_gib * (1 << 30)) // PART)
    n_dst = max(1, n_ring // 4)
    ring = np.empty((n_ring, PART), np.uint8)
    dst = np.empty((n_dst, PART), np.uint8)
    pool = ThreadPoolExecutor(threads)

    def copy(d, s):
        def job(a, b):
            d[a:b] = s[a:b]
        n = len(s)
        futs = [pool.submit(job, n * i // threads, n * (i + 1) // threads) for i in range(threads)]
        for f in futs:
            f.result()
    ring[:] = 7  # first touch (not timed)
    copy(dst, ring[:n_dst])
    start.wait()
    t0 = time.perf_counter()
    done, at = 0, 0
    while time.perf_counter() - t0 < seconds:
        m = min(n_dst, n_ring - at)
        copy(dst[:m], ring[at:at + m])
        done += m * PART
        at = (at + m) % n_ring
    el = time.perf_counter() - t0
    pool.shutdown()
    out_q.put((done, el))


def run_case(procs, threads, seconds, ring_gib):
    ctx = mp.get_context("spawn")
    q, start = ctx.Queue(), ctx.Event()
    ps = [ctx.Process(target=_worker, args=(threads, seconds, ring_gib, start, q))
          for _ in range(procs)]
    for p in ps:
        p.start()
    time.sleep(2.0 + 0.5 * procs)  # rings allocated and first-touched
    start.set()
    res = [q.get(timeout=seconds + 300) for _ in range(procs)]
    for p in ps:
        p.join(timeout=60)
    total = sum(b for b, _ in res)
    el = max(e for _, e in res)
    return {"procs": procs, "threads_per_proc": threads, "GBs": round(total / el / 1e9, 2),
            "per_proc_GBs": [round(b / e / 1e9, 2) for b, e in res]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--ring-gib", type=float, default=1.0)
    args = ap.parse_args()
    import sharding
    aff, quota = sharding.cpu_quota()
    cases = [(1, 8), (8, sharding.rank_threads(8)), (8, 8)]
    out = {"tool": "quota_copy_bench", "affinity_cpus": aff, "cgroup_cpu_quota": quota,
           "rank_threads_world8": sharding.rank_threads(8), "seconds": args.seconds,
           "cases": []}
    for procs, threads in cases:
        out["cases"].append(run_case(procs, threads, args.seconds, args.ring_gib))
        print(json.dumps(out["cases"][-1]), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
