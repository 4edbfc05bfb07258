"""Chunk stores with per-chunk location lists for the batched-loop tests (CPU and GPU): the
reference's Chunk { hash, locations } (src/file/chunk.rs:10-17), where a location may be
unreadable or hold a damaged copy, and a resilver appends the rebuilt copy's location
(src/file/file_part.rs:346)."""
import hashlib

import numpy as np

import oracle


def make_parts(n, d, p, L, seed):
    """n parts of RS(d, p) with L-byte chunks: (chunks [n][d+p][L], digests [n][d+p][32]), the
    parity by the oracle."""
    rng = np.random.default_rng(seed)
    t = d + p
    chunks = np.zeros((n, t, L), np.uint8)
    dig = np.zeros((n, t, 32), np.uint8)
    for k in range(n):
        data = rng.integers(0, 256, size=(d, L), dtype=np.uint8)
        st, par = oracle.encode_sep(d, p, list(data))
        assert st == 0
        chunks[k, :d], chunks[k, d:] = data, np.stack(par)
        for i in range(t):
            dig[k, i] = np.frombuffer(hashlib.sha256(chunks[k, i].tobytes()).digest(), np.uint8)
    return chunks, dig


class Locations:
    """A store whose chunks have location lists: copies[(part, chunk)] = [bytes | None, ...] in
    the metadata's order (None: the location does not read).  Default: one good copy each."""

    def __init__(self, chunks):
        self.chunks = chunks
        self.copies = {}
        self.calls = []

    def locs(self, k, i):
        return self.copies.get((k, i), [self.chunks[k, i].tobytes()])

    def set(self, k, i, *spec):
        """spec per location: "good", "bad" (a flipped byte), "gone" (unreadable), "short"."""
        good = self.chunks[k, i].tobytes()
        out = []
        for s in spec:
            if s == "good":
                out.append(good)
            elif s == "bad":
                b = bytearray(good)
                b[3] ^= 1
                out.append(bytes(b))
            elif s == "short":
                out.append(good[:-1])
            else:
                out.append(None)
        self.copies[(k, i)] = out

    def fetch(self, k, i, start):
        """Location::read_with_context over locations[start..]: the first one that reads."""
        self.calls.append((k, i, start))
        locs = self.locs(k, i)
        for j in range(start, len(locs)):
            if locs[j] is not None:
                return j, locs[j]
        return None

    def read_all(self, k, i):
        return self.locs(k, i)

    def append(self, k, i, blob):
        """resilver's write-back: a new location holding `blob`, appended to the chunk's list
        (chunk.locations.extend, file_part.rs:346); returns its index."""
        locs = list(self.locs(k, i))
        locs.append(bytes(blob))
        self.copies[(k, i)] = locs
        return len(locs) - 1
