"""Pin the oracle (oracle/cec_oracle.c) before trusting it (CPU only).

- the reference's own SHA-256 KAT (reference tests/hash.rs:7-8) and FIPS 180-2 vectors;
- hashlib (OpenSSL) on every length class, scalar and SHA-NI paths;
- the crate's / JavaReedSolomon's / klauspost's published GF, matrix-inverse and RS(5,5) known
  answers;
- structural properties of the coding matrix and reconstruct (first-d-present rule);
- the committed golden vectors (tests/golden/golden_vectors.json) reproduce exactly.
"""
import hashlib
import itertools

import numpy as np
import pytest

import oracle
from _gen import gen_bytes


def _kat_input(v):
    if "input_utf8" in v:
        return v["input_utf8"].encode()
    ch, n = v["input_repeat"]
    return ch.encode() * n


def test_sha256_reference_kat(kats):
    for v in kats["sha256_reference"]:
        assert oracle.sha256(_kat_input(v)).hex() == v["digest"]


def test_sha256_fips_vectors(kats):
    for v in kats["sha256_fips"]:
        assert oracle.sha256(_kat_input(v)).hex() == v["digest"]
        if oracle.has_shani():
            assert oracle.sha256_shani(_kat_input(v)).hex() == v["digest"]


@pytest.mark.parametrize("n", [0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 683,
                               1000, 4096, 65539, 699051])
def test_sha256_vs_hashlib(n):
    b = gen_bytes(n + 5, n).tobytes()
    ref = hashlib.sha256(b).digest()
    assert oracle.sha256(b) == ref
    if oracle.has_shani():
        assert oracle.sha256_shani(b) == ref


def test_gf_kats(kats):
    for a, b, r in kats["gf_mul"]:
        assert oracle.gf_mul(a, b) == r
    for a, n, r in kats["gf_exp"]:
        assert oracle.gf_exp(a, n) == r


def test_gf_field_axioms():
    # every nonzero element has an inverse; mul is commutative; distributive over xor
    for a in range(1, 256):
        assert oracle.gf_mul(a, oracle.gf_div(1, a)) == 1
    rng = np.frombuffer(gen_bytes(5, 3000), np.uint8).reshape(-1, 3)
    for a, b, c in rng:
        a, b, c = int(a), int(b), int(c)
        assert oracle.gf_mul(a, b) == oracle.gf_mul(b, a)
        assert oracle.gf_mul(a, b ^ c) == oracle.gf_mul(a, b) ^ oracle.gf_mul(a, c)


def test_rs_one_encode_kat(kats):
    k = kats["rs_one_encode"]
    st, par = oracle.encode_sep(k["data_shards"], k["parity_shards"], k["data"])
    assert st == 0
    assert [list(map(int, x)) for x in par] == k["parity"]


def test_gf_mul_slice_kat(kats):
    for v in kats["gf_mul_slice"]:
        assert [oracle.gf_mul(v["c"], x) for x in v["in"]] == v["out"]


def _gf_matmul(a, b):
    out = np.zeros((len(a), len(b[0])), np.uint8)
    for i, j in itertools.product(range(len(a)), range(len(b[0]))):
        acc = 0
        for k in range(len(b)):
            acc ^= oracle.gf_mul(int(a[i][k]), int(b[k][j]))
        out[i, j] = acc
    return out


def test_matrix_kats(kats):
    """The crate's / JavaReedSolomon's matrix tests: the Gauss-Jordan inversion the decode path
    uses (oracle/cec_oracle.c gf_invert), and GF matrix products."""
    for v in kats["matrix_inverse"]:
        m = np.array(v["m"], np.uint8)
        inv = oracle.gf_invert(m)
        assert inv.tolist() == v["inv"]
        assert np.array_equal(_gf_matmul(m, inv), np.eye(len(m), dtype=np.uint8))
    for m in kats["matrix_singular"]:
        with pytest.raises(ValueError):
            oracle.gf_invert(np.array(m, np.uint8))
    for v in kats["matrix_multiply"]:
        assert _gf_matmul(v["a"], v["b"]).tolist() == v["ab"]
    # the second inverse case is RS(5,5)'s decode matrix for data shard 2 lost: coding-matrix
    # rows 0, 1, 3, 4 and the first parity row (so it also pins that row of V * inv(V_top))
    m = np.array(kats["matrix_inverse"][1]["m"], np.uint8)
    assert np.array_equal(oracle.coding_matrix(5, 5)[[0, 1, 3, 4, 5]], m)


@pytest.mark.parametrize("d,p", [(1, 1), (3, 2), (10, 4), (20, 8), (5, 5), (128, 128), (255, 1)])
def test_matrix_systematic_and_mds(d, p):
    m = oracle.coding_matrix(d, p)
    assert m.shape == (d + p, d)
    assert np.array_equal(m[:d], np.eye(d, dtype=np.uint8))
    # MDS: a sample of d-row subsets is invertible
    t = d + p
    sel = np.frombuffer(gen_bytes(d * 131 + p, 8 * t), np.uint8)
    for trial in range(4):
        rows = sorted(set(int(x) % t for x in sel[trial * t:(trial + 1) * t]))
        rows = (rows + [r for r in range(t) if r not in rows])[:d]
        oracle.gf_invert(m[sorted(rows)])


def test_matrix_errors():
    with pytest.raises(ValueError) as e:
        oracle.coding_matrix(0, 2)
    assert e.value.args[0] == oracle.TOO_FEW_DATA_SHARDS
    with pytest.raises(ValueError) as e:
        oracle.coding_matrix(2, 0)
    assert e.value.args[0] == oracle.TOO_FEW_PARITY_SHARDS
    with pytest.raises(ValueError) as e:
        oracle.coding_matrix(200, 57)
    assert e.value.args[0] == oracle.TOO_MANY_SHARDS
    oracle.coding_matrix(200, 56)


def test_encode_sep_errors():
    d4 = [b"abcd"] * 3
    assert oracle.encode_sep(3, 2, d4[:2])[0] == oracle.TOO_FEW_DATA_SHARDS
    assert oracle.encode_sep(3, 2, d4 + [b"abcd"])[0] == oracle.TOO_MANY_DATA_SHARDS
    assert oracle.encode_sep(3, 2, d4, [4])[0] == oracle.TOO_FEW_PARITY_SHARDS
    assert oracle.encode_sep(3, 2, d4, [4, 4, 4])[0] == oracle.TOO_MANY_PARITY_SHARDS
    assert oracle.encode_sep(3, 2, [b"abcd", b"abc", b"abcd"])[0] == oracle.INCORRECT_SHARD_SIZE
    assert oracle.encode_sep(3, 2, d4, [4, 5])[0] == oracle.INCORRECT_SHARD_SIZE
    assert oracle.encode_sep(3, 2, d4, [5, 5])[0] == oracle.INCORRECT_SHARD_SIZE
    assert oracle.encode_sep(3, 2, [b"", b"", b""], [0, 0])[0] == oracle.EMPTY_SHARD


def test_reconstruct_roundtrip_all_patterns():
    d, p, L = 4, 3, 129
    data = gen_bytes(11, d * L).reshape(d, L)
    st, par = oracle.encode_sep(d, p, list(data))
    full = [bytes(x) for x in data] + [bytes(x) for x in par]
    t = d + p
    for k in range(0, t + 1):
        for miss in itertools.combinations(range(t), k):
            shards = [None if i in miss else full[i] for i in range(t)]
            st, out = oracle.reconstruct(d, p, shards)
            if k > p:
                assert st == oracle.TOO_FEW_SHARDS_PRESENT
                continue
            assert st == 0
            assert [bytes(o) for o in out] == full
            st, out = oracle.reconstruct(d, p, shards, data_only=True)
            assert st == 0
            for i in range(t):
                if i < d:
                    assert bytes(out[i]) == full[i]
                elif i in miss:
                    assert out[i] is None


def test_reconstruct_uses_first_d_present():
    """reconstruct_internal inverts the rows of the FIRST d present shards: corrupting a later
    present shard must not change the result (the crate never reads it)."""
    d, p, L = 3, 3, 40
    data = gen_bytes(12, d * L).reshape(d, L)
    st, par = oracle.encode_sep(d, p, list(data))
    full = [bytes(x) for x in data] + [bytes(x) for x in par]
    shards = [None, full[1], full[2], full[3], b"\xff" * L, full[5]]
    st, out = oracle.reconstruct(d, p, shards, data_only=True)
    assert st == 0 and bytes(out[0]) == full[0]


def test_reconstruct_errors():
    d, p = 3, 2
    ok = b"abcd"
    assert oracle.reconstruct(d, p, [ok] * 4)[0] == oracle.TOO_FEW_SHARDS
    assert oracle.reconstruct(d, p, [ok] * 6)[0] == oracle.TOO_MANY_SHARDS
    assert oracle.reconstruct(d, p, [ok, ok, b"abc", None, None])[0] == oracle.INCORRECT_SHARD_SIZE
    assert oracle.reconstruct(d, p, [ok, b"", ok, None, None])[0] == oracle.EMPTY_SHARD
    assert oracle.reconstruct(d, p, [ok, None, None, None, ok])[0] == oracle.TOO_FEW_SHARDS_PRESENT
    assert oracle.reconstruct(d, p, [ok] * 5)[0] == 0


def test_golden_encode(golden):
    for c in golden["encode"]:
        data = gen_bytes(c["seed"], c["d"] * c["len"]).reshape(c["d"], c["len"])
        st, par = oracle.encode_sep(c["d"], c["p"], list(data))
        assert st == 0
        assert [hashlib.sha256(bytes(x)).hexdigest() for x in par] == c["parity_sha256"]
        if "parity_hex" in c:
            assert [bytes(x).hex() for x in par] == c["parity_hex"]


def test_golden_reconstruct(golden):
    cache = {}
    for c in golden["reconstruct"]:
        key = (c["d"], c["p"], c["len"], c["seed"])
        if key not in cache:
            data = gen_bytes(c["seed"], c["d"] * c["len"]).reshape(c["d"], c["len"])
            st, par = oracle.encode_sep(c["d"], c["p"], list(data))
            cache[key] = [bytes(x) for x in data] + [bytes(x) for x in par]
        full = cache[key]
        shards = [None if i in c["missing"] else full[i] for i in range(len(full))]
        st, out = oracle.reconstruct(c["d"], c["p"], shards, data_only=c["data_only"])
        assert st == c["status"]
        if st == 0:
            got = [None if o is None else hashlib.sha256(bytes(o)).hexdigest() for o in out]
            assert got == c["out_sha256"]


def test_golden_cluster_parts(golden):
    from _gen import cluster_reader_bytes
    c = golden["cluster"]
    data = cluster_reader_bytes()
    assert hashlib.sha256(data).hexdigest() == c["data_sha256"]
    step = c["d"] * c["chunk_size"]
    for i, part in enumerate(c["parts"]):
        piece = data[i * step:(i + 1) * step]
        cs, par, dig = oracle.part_encode(c["d"], c["p"], np.frombuffer(piece, np.uint8),
                                          len(piece))
        assert cs == part["chunksize"]
        assert [bytes(x).hex() for x in dig] == part["sha256"]


def _gf_tables():
    """GF(2^8) with polynomial 0x11D and generator 2, built here from the definition (the field
    galois_8's build.rs generates), independent of the oracle's C tables."""
    exp, log = [0] * 512, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x11D
    for i in range(255, 512):
        exp[i] = exp[i - 255]
    return exp, log


def test_coding_matrix_by_lagrange_interpolation():
    """M = V·inv(V_top) with V[r][c] = r^c means: parity row i, column j is the j-th Lagrange basis
    polynomial over the points 0..d-1 evaluated at the point d+i (the systematic code evaluates
    the polynomial through the d data values at d..d+p-1).  Computed here in pure Python from
    the field definition -- a second derivation of the coding matrix, by interpolation instead of
    the oracle's Gauss-Jordan inversion -- for the hot-path shapes and the Appendix A rows."""
    exp, log = _gf_tables()

    def mul(a, b):
        return 0 if a == 0 or b == 0 else exp[log[a] + log[b]]

    def div(a, b):
        return 0 if a == 0 else exp[log[a] - log[b] + 255]

    def lagrange_row(d, x):
        row = []
        for j in range(d):
            num = den = 1
            for m in range(d):
                if m != j:
                    num = mul(num, x ^ m)   # (x - m) in characteristic 2
                    den = mul(den, j ^ m)
            row.append(div(num, den))
        return row

    for d, p in [(3, 2), (10, 4), (20, 8), (5, 5), (4, 2), (17, 3), (1, 1), (128, 128)]:
        m = oracle.coding_matrix(d, p)
        for i in range(p):
            assert list(m[d + i]) == lagrange_row(d, d + i), (d, p, i)
    # SURVEY.md Appendix A
    assert lagrange_row(3, 3) == [1, 1, 1] and lagrange_row(3, 4) == [15, 8, 6]
    assert lagrange_row(10, 10) == [129, 150, 175, 184, 210, 196, 254, 232, 3, 2]
    assert lagrange_row(10, 12) == [191, 214, 98, 10, 6, 111, 223, 183, 5, 4]


@pytest.mark.parametrize("d,p,L", [(10, 4, 4096), (3, 2, 683), (20, 8, 1000), (1, 1, 64)])
def test_encode_hash_parts_matches_part_encode(d, p, L):
    """The bench's whole-batch digest checker equals part_encode + hashlib, part by part."""
    n = 9
    data = gen_bytes(d * 7 + p + L, n * d * L).reshape(n, d, L)
    for threads in (1, 3):
        dg = oracle.encode_hash_parts(d, p, data, threads)
        for k in range(n):
            cs, par, dig = oracle.part_encode(d, p, data[k].reshape(-1), d * L)
            assert cs == L and np.array_equal(dg[k], dig)
            chunks = list(data[k]) + list(par)
            assert [hashlib.sha256(c.tobytes()).digest() for c in chunks] == \
                [dg[k, i].tobytes() for i in range(d + p)]


def test_encode_hash_parts_parity_check():
    """With check_parity the checker compares the parts' own parity chunks with the computed
    ones: one flipped parity byte fails exactly that part, and the digests do not depend on it."""
    d, p, L, n = 10, 4, 1000, 5
    data = gen_bytes(77, n * d * L).reshape(n, d, L)
    full = np.zeros((n, d + p, L), np.uint8)
    full[:, :d] = data
    for k in range(n):
        full[k, d:] = np.stack(oracle.encode_sep(d, p, list(data[k]))[1])
    dg, ok = oracle.encode_hash_parts(d, p, full, 2, check_parity=True)
    assert ok.all() and np.array_equal(dg, oracle.encode_hash_parts(d, p, data, 2))
    full[3, d + 2, 999] ^= 0x10
    dg2, ok = oracle.encode_hash_parts(d, p, full, 2, check_parity=True)
    assert ok.tolist() == [True, True, True, False, True] and np.array_equal(dg, dg2)


def test_published_coding_matrix(kats):
    """A coding matrix printed by the JavaReedSolomon authors (RS(4,2)): the oracle's
    construction (V * inv(V_top), exp(0, 0) = 1) reproduces it at a second shape."""
    for v in kats["coding_matrix_published"]:
        d, p = v["data_shards"], v["parity_shards"]
        assert oracle.coding_matrix(d, p)[d:].tolist() == v["parity_rows"]
