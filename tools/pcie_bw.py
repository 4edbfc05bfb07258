"""PCIe ceiling for the C5 host-staged stream (dev tool): pinned host -> device and device ->
host copy rates alone and both directions at once (torch copies on separate streams).

python tools/pcie_bw.py [--gib 4]
"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    args = ap.parse_args()
    n = int(args.gib * (1 << 30))
    h_in = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn, reps=3):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    def h2d():
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    def both():
        h2d()
        d2h()

    t = timed(h2d)
    print(f"H2D {n / t / 1e9:.1f} GB/s", flush=True)
    t = timed(d2h)
    print(f"D2H {n / t / 1e9:.1f} GB/s", flush=True)
    t = timed(both)
    print(f"H2D+D2H concurrent: {2 * n / t / 1e9:.1f} GB/s total, {n / t / 1e9:.1f} GB/s each way",
          flush=True)


if __name__ == "__main__":
    main()
