#!/usr/bin/env python3
"""cp / cat / repair of one file through the engine, in the reference's on-disk format, so that
the REFERENCE's own reader can check what the GPU wrote and repaired (run on the GPU box; the
reader runs afterwards in the build container: tests/golden/make_dropin_record.py).

  python tools/dropin_cp_repair.py [out_dir]      (default gpurun_out/dropin)

1. cp: the file (tests/_gen.py gen_bytes(0xD801, 22 MiB + 777), d=3, p=2, 1 MiB chunks: 7 full
   parts and a short one) goes through chunky_ec.batchwriter.BatchWriter -- the Python twin of the
   Rust BatchWriter -- on the GPU; every chunk is stored as a `sha256-<hex>` file
   (location.rs:612) and the FileReference as YAML in the reference's serde layout
   (file_reference.rs:39-46, file_part.rs:57-65, chunk.rs:10-17).
2. damage (tests/cluster.rs:145-231's scenario, plus a bad copy): one data and one parity chunk
   file deleted in parts 1 and 4, one data chunk file of part 5 overwritten with a flipped byte.
3. cat: chunky_ec.batchreader.BatchReader reads the file back (missing chunks skipped, the
   damaged one rejected by the SHA-256 verification and replaced); its bytes must equal the
   input.
4. repair: FilePart::resilver's compute over the scheduler (cec_multi_resilver): every stored
   chunk loaded and verified, every missing or invalid chunk rebuilt and written back.
5. The store (chunk files + file.yaml) and a summary.json are left in out_dir for the reference
   reader.
"""
import hashlib
import io
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "chunky-bits_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime for torch and the engine)
import yaml  # noqa: E402

import chunky_ec as ce  # noqa: E402
from _gen import gen_bytes  # noqa: E402
from chunky_ec.batchreader import BatchReader  # noqa: E402
from chunky_ec.batchwriter import BatchWriter  # noqa: E402

SEED, LENGTH, D, P, CHUNK = 0xD801, (22 << 20) + 777, 3, 2, 1 << 20
T = D + P


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "dropin")
    os.makedirs(out_dir, exist_ok=True)
    for f in os.listdir(out_dir):
        os.remove(os.path.join(out_dir, f))
    data = gen_bytes(SEED, LENGTH)

    # 1. cp
    parts = []

    def store(part):
        hexes = [h.hex() for h in part.digests]
        for h, c in zip(hexes, part.chunks):
            with open(os.path.join(out_dir, f"sha256-{h}"), "wb") as fh:
                fh.write(bytes(c))
        parts.append({"chunksize": part.chunksize,
                      "data": [{"sha256": h, "locations": [f"sha256-{h}"]} for h in hexes[:D]],
                      "parity": [{"sha256": h, "locations": [f"sha256-{h}"]} for h in hexes[D:]]})

    writer = BatchWriter(D, P, CHUNK, 2, 2, [0])
    written = writer.write(io.BytesIO(data.tobytes()), store)
    assert written == LENGTH
    ref = {"length": LENGTH, "parts": parts}
    with open(os.path.join(out_dir, "file.yaml"), "w") as fh:
        yaml.safe_dump(ref, fh, sort_keys=False)

    def path(k, i):
        ch = (parts[k]["data"] + parts[k]["parity"])[i]
        return os.path.join(out_dir, ch["locations"][0])

    # 2. damage
    deleted = [(1, 0), (1, D), (4, 2), (4, D + 1)]
    for k, i in deleted:
        os.remove(path(k, i))
    corrupted = (5, 1)
    with open(path(*corrupted), "r+b") as fh:
        b = fh.read(1)
        fh.seek(0)
        fh.write(bytes([b[0] ^ 0x20]))

    def fetch(k, i):
        try:
            with open(path(k, i), "rb") as fh:
                return fh.read()
        except FileNotFoundError:
            return None

    def digests_of(k):
        return np.array([np.frombuffer(bytes.fromhex(c["sha256"]), np.uint8)
                         for c in parts[k]["data"] + parts[k]["parity"]])

    full = sum(1 for p in parts if p["chunksize"] == CHUNK)

    # 3. cat: the full parts through BatchReader, the short last part per call (its own shape)
    back = bytearray()
    reader = BatchReader(D, P, CHUNK, 2, 2, [0])
    reader.read(full, fetch, digests_of, lambda k, ds: back.extend(b"".join(map(bytes, ds))))
    rs = ce.ReedSolomon(D, P)
    for k in range(full, len(parts)):
        shards = []
        for i in range(T):
            b = fetch(k, i)
            ok = b is not None and ce.Sha256Hash.from_buf(b).digest.hex() == \
                (parts[k]["data"] + parts[k]["parity"])[i]["sha256"]
            shards.append(bytearray(b) if ok else None)
        rs.reconstruct_data(shards)
        back.extend(b"".join(bytes(s) for s in shards[:D]))
    back = bytes(back[:LENGTH])
    cat_ok = back == data.tobytes()

    # 4. repair (FilePart::resilver over the scheduler), full parts
    m = ce.Multi(rs, CHUNK, 2, 2, [0])
    chunks = ce.HostBuffer(full * T * CHUNK)
    cv = chunks.view(full, T, CHUNK)
    present = np.zeros((full, T), np.uint8)
    expected = np.zeros((full, T, 32), np.uint8)
    for k in range(full):
        expected[k] = digests_of(k)
        for i in range(T):
            b = fetch(k, i)
            if b is not None and len(b) == CHUNK:
                cv[k, i] = np.frombuffer(b, np.uint8)
                present[k, i] = 1
    rebuilt = ce.HostBuffer(full * T * CHUNK)
    verified = np.zeros((full, T), np.uint8)
    status = np.zeros(full, np.int32)
    m.resilver_sync(chunks, present, expected, full, rebuilt, verified, status)
    rv = rebuilt.view(full, T, CHUNK)
    repaired = []
    for k in range(full):
        assert status[k] == ce.OK, (k, status[k])
        for i in range(T):
            if verified[k, i]:
                continue
            blob = rv[k, i].tobytes()
            assert hashlib.sha256(blob).hexdigest() == \
                (parts[k]["data"] + parts[k]["parity"])[i]["sha256"], (k, i)
            with open(path(k, i), "wb") as fh:
                fh.write(blob)
            repaired.append([k, i])

    summary = {"length": LENGTH, "seed": SEED, "d": D, "p": P, "chunk_size": CHUNK,
               "parts": len(parts), "full_parts": full, "deleted": deleted,
               "corrupted": list(corrupted), "cat_equals_input": cat_ok,
               "read_retries": reader.retries, "repaired": repaired,
               "input_sha256": hashlib.sha256(data.tobytes()).hexdigest(),
               "device": torch.cuda.get_device_name(0)}
    with open(os.path.join(out_dir, "summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary))
    assert cat_ok and sorted(map(tuple, repaired)) == sorted(deleted + [corrupted])


if __name__ == "__main__":
    main()
