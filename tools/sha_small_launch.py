"""How long one SHA-256 launch of 1 MiB chunks takes as a function of its size (the product
library's default kernel choice): a read retry round hashes a few chunks, a window hundreds, and
the chain time of one chunk bounds both.  Each size alone, then beside a busy second stream (torch
elementwise work on the other CUs) to see whether the chip's load changes the chain time.

    python tools/sha_small_launch.py [--sizes 1,4,16,96,256] [--reps 5]"""
import argparse
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chunky-bits_amd"))
import torch  # noqa: E402
import chunky_ec as ce  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,4,16,96,256")
    ap.add_argument("--chunks", type=int, default=14)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sizes = [int(x) for x in args.sizes.split(",")]
    L = 1 << 20
    buf = torch.empty((max(sizes), args.chunks, L), dtype=torch.uint8, device=dev)
    batch = ce.PartBatch.from_tensor(buf)
    ce.fill_synthetic(batch, args.chunks, 7)
    dig = torch.empty((max(sizes), args.chunks, 32), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    bg = torch.cuda.Stream()
    busy = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    stop = threading.Event()

    def background():
        with torch.cuda.stream(bg):
            while not stop.is_set():
                for _ in range(20):
                    busy.mul_(1.0000001)
                bg.synchronize()

    def run(n):
        sub = ce.PartBatch(batch.base, batch.part_stride, batch.chunk_stride, n, batch.chunk_len)
        out = []
        for r in range(args.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            ce.sha256_batch(sub, 0, args.chunks, dig.data_ptr(), s.cuda_stream)
            e1.record(s)
            e1.synchronize()
            if r:
                out.append(e0.elapsed_time(e1))
        out.sort()
        return out[len(out) // 2], out[0]

    for label in ("alone", "beside a busy stream"):
        th = None
        if label != "alone":
            th = threading.Thread(target=background)
            th.start()
        for n in sizes:
            med, lo = run(n)
            print(f"{label:22s} parts {n:4d} ({n * args.chunks:5d} chunks): median {med:7.2f} ms  "
                  f"min {lo:7.2f} ms", flush=True)
        if th:
            stop.set()
            th.join()


if __name__ == "__main__":
    main()
