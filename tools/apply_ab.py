"""A/B the rs_apply_kernel tuning variants (CEC_APPLY_TUNE) in ONE process on the C2 encode.

python tools/apply_ab.py [--rounds 5] [--variants "plain,nt,v1,v1+nt,g8,nt+g8"]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "chunky-bits_amd"))
# CEC_APPLY_TUNE is read only by the A/B build (make -C chunky-bits_amd/csrc ab)
os.environ.setdefault("CEC_LIBRARY", os.path.join(ROOT, "tools", "ab", "libchunky_ec.so"))
import torch  # noqa: E402
import chunky_ec as ce  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=4096)
    ap.add_argument("--d", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="plain,nt,v1,v1+nt,g8,nt+g8")
    args = ap.parse_args()
    t = args.d + args.p
    dev = torch.device("cuda", 0)
    buf = torch.empty((args.parts, t, args.chunk), dtype=torch.uint8, device=dev)
    batch = ce.PartBatch.from_tensor(buf)
    ce.fill_synthetic(batch, t, 5)
    rs = ce.ReedSolomon(args.d, args.p)
    variants = args.variants.split(",")
    times = {v: [] for v in variants}
    ref = None
    s = torch.cuda.current_stream()
    for r in range(args.rounds + 1):
        for v in variants:
            os.environ["CEC_APPLY_TUNE"] = v
            ce.reload_knobs()  # the library reads its knobs once per process
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            ce.encode_batch(rs, batch, s)
            e1.record(s)
            torch.cuda.synchronize()
            if r:
                times[v].append(e0.elapsed_time(e1))
            par = buf[:, args.d:, ::4093].to(torch.int64).sum().item()  # sampled checksum
            ref = par if ref is None else ref
            assert par == ref, v
    nbytes = args.parts * t * args.chunk
    for v in variants:
        ts = sorted(times[v])
        print(f"variant '{v}': median {ts[len(ts)//2]:.3f} ms  min {ts[0]:.3f} ms  "
              f"{nbytes / ts[len(ts)//2] / 1e6:.0f} GB/s (median)", flush=True)


if __name__ == "__main__":
    main()
