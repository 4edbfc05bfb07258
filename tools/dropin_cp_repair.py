#!/usr/bin/env python3
"""cp / cat / verify / repair through the engine, in the reference's on-disk format, so that the
REFERENCE's own reader can check what the GPU wrote and repaired (run on the GPU box; the reader
runs afterwards in the build container: tests/golden/make_dropin_record.py).

  python tools/dropin_cp_repair.py [out_dir]      (default gpurun_out/dropin)

Two files go into one store directory (chunks as `sha256-<hex>` files, location.rs:612; a
FileReference YAML per file in the reference's serde layout, file_reference.rs:39-46,
file_part.rs:57-65, chunk.rs:10-17: every chunk has a list of locations):

file.yaml -- tests/_gen.py gen_bytes(0xD801, 22 MiB + 777), d=3, p=2, 1 MiB chunks: 7 full parts
  and a short one.
  1. cp through chunky_ec.batchwriter.BatchWriter (the Python twin of the Rust BatchWriter).
  2. damage (tests/cluster.rs:145-231's scenario, plus a bad copy): one data and one parity chunk
     file deleted in parts 1 and 4, one data chunk file of part 5 overwritten with a flipped byte.
  3. cat through chunky_ec.batchreader.FileReader (full parts batched, the short last part per
     call): equal to the input.
  4. verify through chunky_ec.batchcheck.FileChecker: exactly the 4 deleted locations
     unavailable and the damaged one invalid.
  5. resilver through FileChecker: only the chunks with no valid copy are rebuilt; each is
     written back as `sha256-<hex>` (the destination's OnConflict default, Overwrite,
     location.rs:505) and its location APPENDED to the chunk's list (file_part.rs:346), so a
     repaired chunk is listed twice; the YAML is rewritten (cluster_location.rs:364).  Verify is
     then ideal and cat equals the input again.

stale.yaml -- gen_bytes(0x57A1, 7 MiB + 333): 2 full parts and a short one, where p + 1 chunks of
  EVERY part are listed [stale copy, good copy]: a damaged replica under `stale/` first, then the
  chunk's file.  Fewer than d first copies verify, so the reference's read only succeeds because
  it walks each chunk's locations (file_part.rs:100-107); cat through FileReader must equal the
  input, verify must flag exactly the stale locations invalid, and resilver must rebuild nothing.
  (The reference's python reader checks only each data chunk's FIRST location, so on this file
  it must report exactly the stale data copies: make_dropin_record.py records that.)

A summary.json is left beside the store.
"""
import hashlib
import io
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "chunky-bits_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime for torch and the engine)
import yaml  # noqa: E402

from _gen import gen_bytes  # noqa: E402
from chunky_ec.batchcheck import FileChecker  # noqa: E402
from chunky_ec.batchreader import FileReader  # noqa: E402
from chunky_ec.batchwriter import BatchWriter  # noqa: E402

SEED, LENGTH, D, P, CHUNK = 0xD801, (22 << 20) + 777, 3, 2, 1 << 20
STALE_SEED, STALE_LENGTH = 0x57A1, (7 << 20) + 333
T = D + P


class Store:
    """One directory of chunk files plus the FileReference of one file in it."""

    def __init__(self, root):
        self.root = root
        self.parts = []

    def chunk(self, k, i):
        return (self.parts[k]["data"] + self.parts[k]["parity"])[i]

    def read_loc(self, loc):  # Location::read: None where it does not read
        try:
            with open(os.path.join(self.root, loc), "rb") as fh:
                return fh.read()
        except FileNotFoundError:
            return None

    def write_loc(self, loc, blob):
        path = os.path.join(self.root, loc)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "wb") as fh:
            fh.write(bytes(blob))

    def fetch(self, k, i, start):  # read_with_context over locations[start..]
        locs = self.chunk(k, i)["locations"]
        for j in range(start, len(locs)):
            b = self.read_loc(locs[j])
            if b is not None:
                return j, b
        return None

    def read_all(self, k, i):
        return [self.read_loc(loc) for loc in self.chunk(k, i)["locations"]]

    def digests(self, k):
        return np.array([np.frombuffer(bytes.fromhex(c["sha256"]), np.uint8)
                         for c in self.parts[k]["data"] + self.parts[k]["parity"]])

    def shapes(self):
        return [(D, P, p["chunksize"]) for p in self.parts]

    def cp(self, data):
        def sink(part):
            hexes = [h.hex() for h in part.digests]
            for h, c in zip(hexes, part.chunks):
                self.write_loc(f"sha256-{h}", c)
            self.parts.append({
                "chunksize": part.chunksize,
                "data": [{"sha256": h, "locations": [f"sha256-{h}"]} for h in hexes[:D]],
                "parity": [{"sha256": h, "locations": [f"sha256-{h}"]} for h in hexes[D:]]})
        n = BatchWriter(D, P, CHUNK, 2, 2, [0]).write(io.BytesIO(data), sink)
        assert n == len(data)

    def dump(self, name, length):
        with open(os.path.join(self.root, name), "w") as fh:
            yaml.safe_dump({"length": length, "parts": self.parts}, fh, sort_keys=False)


def cat(store, reader, length):
    out = bytearray()
    reader.read(store.shapes(), store.fetch, store.digests,
                lambda k, data: out.extend(b"".join(bytes(x) for x in data)))
    return bytes(out[:length])


def verify(store, checker):
    reports = {}
    checker.verify(store.shapes(), store.read_all, store.digests,
                   lambda k, part: reports.__setitem__(k, part))
    return [reports[k] for k in range(len(store.parts))]


def resilver(store, checker):
    repaired, errors = [], []

    def sink(k, part):
        if part.error is not None:
            errors.append([k, part.error])
        for i, blob in part.rebuilt.items():
            c = store.chunk(k, i)
            assert hashlib.sha256(bytes(blob)).hexdigest() == c["sha256"], (k, i)
            loc = f"sha256-{c['sha256']}"
            store.write_loc(loc, blob)
            c["locations"].append(loc)  # chunk.locations.extend(new locations)
            repaired.append([k, i])
    checker.resilver(store.shapes(), store.read_all, store.digests, sink)
    return repaired, errors


def counts(reports):
    return {"unavailable": [[k, i, j] for k, r in enumerate(reports)
                            for i, locs in enumerate(r.locations) for j, x in enumerate(locs)
                            if x is None],
            "invalid": [[k, i, j] for k, r in enumerate(reports)
                        for i, locs in enumerate(r.locations) for j, x in enumerate(locs)
                        if x is False],
            "unhealthy_chunks": sum(T - r.healthy_chunks() for r in reports)}


def main():
    out_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "dropin")
    if os.path.isdir(out_dir):
        shutil.rmtree(out_dir)
    os.makedirs(out_dir)
    reader = FileReader(2, 2, [0])
    checker = FileChecker(2, 2, [0])

    # file.yaml: cp, damage, cat, verify, resilver (append), verify, cat
    data = gen_bytes(SEED, LENGTH).tobytes()
    st = Store(out_dir)
    st.cp(data)
    deleted = [(1, 0), (1, D), (4, 2), (4, D + 1)]
    for k, i in deleted:
        os.remove(os.path.join(out_dir, st.chunk(k, i)["locations"][0]))
    corrupted = (5, 1)
    path = os.path.join(out_dir, st.chunk(*corrupted)["locations"][0])
    blob = bytearray(open(path, "rb").read())
    blob[0] ^= 0x20
    open(path, "wb").write(blob)
    cat_ok = cat(st, reader, LENGTH) == data
    before = counts(verify(st, checker))
    repaired, errors = resilver(st, checker)
    after = counts(verify(st, checker))
    cat_after = cat(st, reader, LENGTH) == data
    st.dump("file.yaml", LENGTH)

    # stale.yaml: p + 1 chunks of every part listed [stale copy, good copy]
    sdata = gen_bytes(STALE_SEED, STALE_LENGTH).tobytes()
    ss = Store(out_dir)
    ss.cp(sdata)
    stale = []
    for k in range(len(ss.parts)):
        for m in range(P + 1):
            i = (k + 2 * m) % T
            c = ss.chunk(k, i)
            good = ss.read_loc(c["locations"][0])
            bad = bytearray(good)
            bad[len(bad) // 2] ^= 0x04
            loc = f"stale/sha256-{c['sha256']}"
            ss.write_loc(loc, bad)
            c["locations"].insert(0, loc)
            stale.append([k, i])
    stale_cat = cat(ss, reader, STALE_LENGTH) == sdata
    stale_verify = counts(verify(ss, checker))
    stale_repaired, stale_errors = resilver(ss, checker)
    ss.dump("stale.yaml", STALE_LENGTH)

    summary = {
        "length": LENGTH, "seed": SEED, "d": D, "p": P, "chunk_size": CHUNK,
        "parts": len(st.parts), "full_parts": sum(1 for p in st.parts if p["chunksize"] == CHUNK),
        "deleted": deleted, "corrupted": list(corrupted), "cat_equals_input": cat_ok,
        "verify_before": before, "repaired": repaired, "resilver_errors": errors,
        "verify_after": after, "cat_after_repair_equals_input": cat_after,
        "input_sha256": hashlib.sha256(data).hexdigest(),
        "stale": {"length": STALE_LENGTH, "seed": STALE_SEED, "parts": len(ss.parts),
                  "stale_chunks": stale, "cat_equals_input": stale_cat,
                  "verify": stale_verify, "repaired": stale_repaired,
                  "resilver_errors": stale_errors,
                  "input_sha256": hashlib.sha256(sdata).hexdigest()},
        "device": torch.cuda.get_device_name(0)}
    with open(os.path.join(out_dir, "summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary))
    want_bad = sorted(map(list, deleted + [corrupted]))
    assert cat_ok and cat_after and sorted(repaired) == want_bad and not errors
    assert sorted(x[:2] for x in before["unavailable"]) == sorted(map(list, deleted))
    assert [x[:2] for x in before["invalid"]] == [list(corrupted)]
    # the rewritten files sit at the deleted / damaged locations: every location reads and verifies
    assert after["unhealthy_chunks"] == 0 and not after["unavailable"] and not after["invalid"]
    assert stale_cat and not stale_repaired and not stale_errors
    assert sorted(x[:2] for x in stale_verify["invalid"]) == sorted(stale)
    assert all(x[2] == 0 for x in stale_verify["invalid"]) and stale_verify["unhealthy_chunks"] == 0


if __name__ == "__main__":
    main()
