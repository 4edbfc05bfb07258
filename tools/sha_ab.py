"""A/B the SHA-256 kernel variants (CEC_SHA_VARIANT) in ONE process on the C2 shape.

python tools/sha_ab.py [--parts 4096] [--rounds 3] [--variants 1,2,3,4]
Prints per-variant median/min kernel ms (HIP events on the launch stream) and checks that all
variants produce identical digests.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "chunky-bits_amd"))
# The attribution modes live only in the A/B build (`make -C chunky-bits_amd/csrc ab`).
os.environ.setdefault("CEC_LIBRARY", os.path.join(ROOT, "tools", "ab", "libchunky_ec.so"))
import torch  # noqa: E402
import chunky_ec as ce  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=4096)
    ap.add_argument("--chunks", type=int, default=14)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--encode-first", action="store_true",
                    help="launch an RS(10,4) encode on the same stream right before each SHA")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    buf = torch.empty((args.parts, args.chunks, args.chunk), dtype=torch.uint8, device=dev)
    batch = ce.PartBatch.from_tensor(buf)
    ce.fill_synthetic(batch, args.chunks, 99)
    variants = [int(v) for v in args.variants.split(",")]
    codec = ce.ReedSolomon(10, 4) if args.chunks == 14 else None
    digs = {v: torch.empty((args.parts, args.chunks, 32), dtype=torch.uint8, device=dev)
            for v in variants}
    times = {v: [] for v in variants}
    s = torch.cuda.current_stream()
    for r in range(args.rounds + 1):
        for v in variants:
            os.environ["CEC_SHA_VARIANT"] = str(v)
            ce.reload_knobs()  # the library reads its knobs once per process
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if args.encode_first:
                ce.encode_batch(codec, ce.PartBatch(batch.base, batch.part_stride,
                                                    batch.chunk_stride, batch.n_parts,
                                                    batch.chunk_len), s)
            e0.record(s)
            ce.sha256_batch(batch, 0, args.chunks, digs[v].data_ptr(), s)
            e1.record(s)
            torch.cuda.synchronize()
            if r:
                times[v].append(e0.elapsed_time(e1))
    ref = digs[variants[0]]
    nbytes = args.parts * args.chunks * args.chunk
    for v in variants:
        t = sorted(times[v])
        same = torch.equal(digs[v], ref)
        print(f"variant {v}: median {t[len(t)//2]:.2f} ms  min {t[0]:.2f} ms  "
              f"{nbytes / t[0] / 1e6:.1f} GB/s  digests_equal={same}", flush=True)


if __name__ == "__main__":
    main()
