"""Stress: many host threads call cec_read_batch at once, each on its own HIP stream (the read's
speculative decode runs on a pooled side stream with fork/join events, so the process has many
more streams than hardware queues).  Every read must rebuild its parts bit-exact.

    python tools/stress_read_batch.py [--threads 16] [--iters 20]
"""
import argparse
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "chunky-bits_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import chunky_ec as ce  # noqa: E402


def worker(i, args, errors):
    try:
        d, p, L, n = 10, 4, 65536, 8
        t = d + p
        dev = torch.device("cuda", 0)
        s = torch.cuda.Stream(dev)
        rs = ce.ReedSolomon(d, p)
        with torch.cuda.stream(s):
            buf = torch.empty((n, t, L), dtype=torch.uint8, device=dev)
            dig = torch.empty((n, t, 32), dtype=torch.uint8, device=dev)
        batch = ce.PartBatch.from_tensor(buf, L)
        ce.fill_synthetic(batch, d, 1000 + i, s)
        ce.encode_hash_batch(rs, batch, dig.data_ptr(), s)
        s.synchronize()
        ref = buf.clone()
        rng = np.random.default_rng(i)
        for it in range(args.iters):
            pres = np.zeros((n, t), np.uint8)
            for k in range(n):
                pres[k, rng.choice(t, d, replace=False)] = 1
            mask = torch.from_numpy(pres).to(dev).view(n, t, 1)
            with torch.cuda.stream(s):
                buf.mul_(mask)  # chunks not loaded start zeroed
            ver, st = ce.read_batch(rs, batch, pres.tobytes(), dig.data_ptr(), s)
            s.synchronize()
            assert all(x == 0 for x in st), (i, it, st)
            if not torch.equal(buf[:, :d], ref[:, :d]):
                raise AssertionError(f"thread {i} iter {it}: data mismatch")
            buf.copy_(ref)
            s.synchronize()
    except Exception as e:  # noqa: BLE001
        errors.append(f"{i}: {e!r}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    errors = []
    ths = [threading.Thread(target=worker, args=(i, args, errors)) for i in range(args.threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    print("errors:", errors if errors else "none", flush=True)
    sys.exit(1 if errors else 0)


if __name__ == "__main__":
    main()
