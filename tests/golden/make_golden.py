"""Generate tests/golden/golden_vectors.json from the oracle (oracle/cec_oracle.c).

The oracle is first pinned by tests/golden/crate_kats.json (tests/test_oracle.py); this script
freezes its outputs for the hot-path shapes so the GPU parity tests on the box (and any later
change to the oracle) are checked against committed bytes.  Run from the repo root:

    python tests/golden/make_golden.py
"""
import hashlib
import itertools
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from _gen import cluster_reader_bytes, gen_bytes  # noqa: E402


def h(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def encode_cases():
    cases = []
    shapes = [
        (3, 2, 1), (3, 2, 683), (3, 2, 1024), (3, 2, 699051),
        (10, 4, 1), (10, 4, 17), (10, 4, 4096), (10, 4, 65539),
        (20, 8, 261), (5, 5, 2), (1, 1, 33), (2, 7, 100), (17, 3, 4111),
    ]
    for seed, (d, p, L) in enumerate(shapes, start=1000):
        data = gen_bytes(seed, d * L).reshape(d, L)
        st, par = oracle.encode_sep(d, p, list(data))
        assert st == 0
        case = {"d": d, "p": p, "len": L, "seed": seed,
                "parity_sha256": [h(x) for x in par],
                "data_sha256": [h(x) for x in data]}
        if L <= 64:
            case["parity_hex"] = [bytes(x).hex() for x in par]
        cases.append(case)
    return cases


def reconstruct_cases():
    cases = []
    # RS(3,2), 683-byte chunks: every erasure set of size 1..2 (and the 3-missing error).
    d, p, L, seed = 3, 2, 683, 77
    data = gen_bytes(seed, d * L).reshape(d, L)
    st, par = oracle.encode_sep(d, p, list(data))
    full = list(data) + par
    t = d + p
    for k in (1, 2, 3):
        for miss in itertools.combinations(range(t), k):
            for data_only in (False, True):
                shards = [None if i in miss else bytes(full[i]) for i in range(t)]
                st, out = oracle.reconstruct(d, p, shards, data_only=data_only)
                case = {"d": d, "p": p, "len": L, "seed": seed, "missing": list(miss),
                        "data_only": data_only, "status": st}
                if st == 0:
                    case["out_sha256"] = [None if o is None else h(o) for o in out]
                cases.append(case)
    # RS(10,4), 97-byte chunks: 40 seeded patterns of 1..4 erasures.
    d, p, L, seed = 10, 4, 97, 78
    data = gen_bytes(seed, d * L).reshape(d, L)
    st, par = oracle.encode_sep(d, p, list(data))
    full = list(data) + par
    t = d + p
    sel = np.frombuffer(gen_bytes(79, 400), dtype=np.uint8)
    for n in range(40):
        k = 1 + n % 4
        miss = sorted(set(int(x) % t for x in sel[n * 10:(n + 1) * 10]))[:k]
        while len(miss) < k:
            miss = sorted(set(miss) | {len(miss) * 3 % t})
        for data_only in (False, True):
            shards = [None if i in miss else bytes(full[i]) for i in range(t)]
            st, out = oracle.reconstruct(d, p, shards, data_only=data_only)
            cases.append({"d": d, "p": p, "len": L, "seed": seed, "missing": miss,
                          "data_only": data_only, "status": st,
                          "out_sha256": [None if o is None else h(o) for o in out]})
    return cases


def cluster_case():
    """tests/cluster.rs: 20 480 bytes, chunk_size 2^10, d=3 (p=2: writer.rs:55 default)."""
    data = cluster_reader_bytes()
    d, p, chunk = 3, 2, 1 << 10
    parts = []
    for off in range(0, len(data), d * chunk):
        piece = data[off:off + d * chunk]
        cs, par, dig = oracle.part_encode(d, p, np.frombuffer(piece, np.uint8), len(piece))
        parts.append({"length": len(piece), "chunksize": cs,
                      "sha256": [bytes(x).hex() for x in dig]})
    return {"d": d, "p": p, "chunk_size": chunk, "total": len(data),
            "data_sha256": h(data), "parts": parts}


def zeros_case():
    """tests/file.rs:26-56: zeros of length 2^23+7 for d, p in 1..=3 with 1 MiB chunks."""
    length, chunk = (1 << 23) + 7, 1 << 20
    out = []
    for d in (1, 2, 3):
        for p in (1, 2, 3):
            parts = []
            for off in range(0, length, d * chunk):
                n = min(d * chunk, length - off)
                L = (n + d - 1) // d
                zero = hashlib.sha256(bytes(L)).hexdigest()
                parts.append({"length": n, "chunksize": L, "sha256": [zero] * (d + p)})
            out.append({"d": d, "p": p, "length": length, "n_parts": len(parts),
                        "parts": parts})
    return out


def main():
    doc = {
        "_about": "Oracle outputs (oracle/cec_oracle.c, pinned by crate_kats.json) for the hot-path "
                  "shapes; inputs are tests/_gen.py gen_bytes(seed, d*len) split into d chunks.",
        "encode": encode_cases(),
        "reconstruct": reconstruct_cases(),
        "cluster": cluster_case(),
        "zeros": zeros_case(),
    }
    path = os.path.join(HERE, "golden_vectors.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
