"""A/B the fused encode+hash kernel's attribution modes (CEC_FUSED_MODE) and the separate path
(CEC_FUSED=0) in ONE process on the C2 shape.  Dev tool: modes 1/2 give wrong outputs by design.

python tools/fused_ab.py [--parts 4096] [--d 10 --p 4 --chunk 1048576] [--modes 0,1,2,sep]
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
    ap.add_argument("--d", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", default="0,1,2,sep")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t = args.d + args.p
    buf = torch.empty((args.parts, t, args.chunk), dtype=torch.uint8, device=dev)
    batch = ce.PartBatch.from_tensor(buf)
    ce.fill_synthetic(batch, t, 7)
    codec = ce.ReedSolomon(args.d, args.p)
    dig = torch.empty((args.parts, t, 32), dtype=torch.uint8, device=dev)
    modes = args.modes.split(",")
    times = {m: [] for m in modes}
    s = torch.cuda.current_stream()
    for r in range(args.rounds + 1):
        for m in modes:
            os.environ["CEC_FUSED"] = "0" if m == "sep" else "1"
            os.environ["CEC_FUSED_PRIO"] = {"noprio": "0", "prio": "1", "shaprio": "2"}.get(m, "")
            os.environ["CEC_FUSED_MODE"] = m if m in ("1", "2", "3") else "0"
            os.environ["CEC_FUSED_ENC3"] = "0" if m == "enc3off" else "1"
            os.environ["CEC_FUSED_BE"] = {"le": "0", "be": "1"}.get(m, "")
            ce.reload_knobs()  # the library reads its knobs once per process
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            ce.encode_hash_batch(codec, batch, dig.data_ptr(), s)
            e1.record(s)
            torch.cuda.synchronize()
            if r:
                times[m].append(e0.elapsed_time(e1))
    nbytes = args.parts * args.d * args.chunk
    for m in modes:
        tt = sorted(times[m])
        print(f"mode {m}: median {tt[len(tt)//2]:.2f} ms  min {tt[0]:.2f} ms  "
              f"{nbytes / tt[0] / 1e6:.1f} GB/s data", flush=True)


if __name__ == "__main__":
    main()
