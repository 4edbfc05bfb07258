"""GPU parity tests: the HIP path (through the C-ABI) against the oracle, hashlib and the
committed golden vectors.  Bit-exact everywhere (integer / byte work).

Cases follow the reference's tests and SURVEY.md §8d: KATs (tests/hash.rs), part slicing and
counts (tests/file.rs:26-56, zeros 2^23+7 bytes), the tests/cluster.rs generator (chunk 2^10,
d=3, p=2, 683-byte last chunks), delete-and-rebuild (tests/cluster.rs:145-231), every erasure
pattern of small codes, odd lengths, unaligned layouts, and the full BASELINE shapes via
size-independent properties (encode -> erase -> reconstruct -> same digests).
"""
import hashlib
import itertools

import numpy as np
import pytest

import oracle
from _gen import cluster_reader_bytes, gen_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import chunky_ec as ce  # noqa: E402  (after torch: one HIP runtime)

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda", 0)


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


# ----------------------------------------------------------------------------------------------
# SHA-256 (Sha256Hash::from_buf)
# ----------------------------------------------------------------------------------------------

def test_sha256_reference_and_fips_kats(kats):
    for v in kats["sha256_reference"] + kats["sha256_fips"]:
        b = v["input_utf8"].encode() if "input_utf8" in v else \
            v["input_repeat"][0].encode() * v["input_repeat"][1]
        h = ce.Sha256Hash.from_buf(b)
        assert str(h) == v["digest"]
        assert h.verify(b)
        assert str(ce.AnyHash(h)) == "sha256-" + v["digest"]


@pytest.mark.parametrize("variant", ["", "1", "2"])  # by size (split here), lane, split
def test_sha256_many_lengths_vs_hashlib(variant, knob_env):
    knob_env.set("CEC_SHA_VARIANT", variant)
    lens = [0, 1, 2, 3, 15, 16, 17, 55, 56, 57, 63, 64, 65, 111, 112, 119, 120, 127, 128, 129,
            191, 192, 683, 1000, 1023, 1024, 4097, 65539, 699051, 1 << 20]
    bufs = [gen_bytes(900 + n, n).tobytes() for n in lens]
    hs = ce.Sha256Hash.from_bufs(bufs)
    for b, h in zip(bufs, hs):
        assert h.digest == hashlib.sha256(b).digest(), len(b)


def test_sha256_verify_detects_single_bit_flip():
    b = bytearray(gen_bytes(3, 4096).tobytes())
    h = ce.Sha256Hash.from_buf(bytes(b))
    b[1234] ^= 0x10
    assert not h.verify(bytes(b))


# ----------------------------------------------------------------------------------------------
# encode_sep (host-buffer API)
# ----------------------------------------------------------------------------------------------

def test_encode_one_encode_kat(kats):
    k = kats["rs_one_encode"]
    rs = ce.ReedSolomon(k["data_shards"], k["parity_shards"])
    par = [bytearray(2) for _ in range(k["parity_shards"])]
    rs.encode_sep([bytes(x) for x in k["data"]], par)
    assert [list(x) for x in par] == k["parity"]


def test_encode_golden(golden):
    for c in golden["encode"]:
        d, p, L = c["d"], c["p"], c["len"]
        data = gen_bytes(c["seed"], d * L).reshape(d, L)
        rs = ce.ReedSolomon(d, p)
        par = [bytearray(L) for _ in range(p)]
        rs.encode_sep([x.tobytes() for x in data], par)
        assert [sha(x) for x in par] == c["parity_sha256"], (d, p, L)
        if "parity_hex" in c:
            assert [bytes(x).hex() for x in par] == c["parity_hex"]


@pytest.mark.parametrize("d,p", [(1, 1), (2, 1), (3, 2), (4, 4), (6, 3), (10, 4), (12, 9),
                                 (20, 8), (16, 16), (30, 2), (64, 8), (200, 56)])
@pytest.mark.parametrize("L", [1, 7, 16, 33, 4095, 4097, 16385, 20000])
def test_encode_vs_oracle(d, p, L):
    data = gen_bytes(d * 1000 + p * 10 + L, d * L).reshape(d, L)
    st, ref = oracle.encode_sep(d, p, list(data))
    assert st == 0
    rs = ce.ReedSolomon(d, p)
    par = [bytearray(L) for _ in range(p)]
    rs.encode_sep([x.tobytes() for x in data], par)
    for i in range(p):
        assert bytes(par[i]) == ref[i].tobytes(), (d, p, L, i)


def test_encode_errors_match_crate():
    rs = ce.ReedSolomon(3, 2)
    four = [b"abcd"] * 3
    cases = [
        (four[:2], [bytearray(4)] * 2, ce.TOO_FEW_DATA_SHARDS),
        (four + [b"abcd"], [bytearray(4)] * 2, ce.TOO_MANY_DATA_SHARDS),
        (four, [bytearray(4)], ce.TOO_FEW_PARITY_SHARDS),
        (four, [bytearray(4)] * 3, ce.TOO_MANY_PARITY_SHARDS),
        ([b"abcd", b"abc", b"abcd"], [bytearray(4)] * 2, ce.INCORRECT_SHARD_SIZE),
        (four, [bytearray(4), bytearray(5)], ce.INCORRECT_SHARD_SIZE),
        (four, [bytearray(5), bytearray(5)], ce.INCORRECT_SHARD_SIZE),
        ([b"", b"", b""], [bytearray(0)] * 2, ce.EMPTY_SHARD),
    ]
    for data, par, code in cases:
        with pytest.raises(ce.Error) as e:
            rs.encode_sep(data, [bytearray(x) for x in par])
        assert e.value.code == code
        ost, _ = oracle.encode_sep(3, 2, data, [len(x) for x in par])
        assert ost == code


# ----------------------------------------------------------------------------------------------
# reconstruct / reconstruct_data (host-buffer API)
# ----------------------------------------------------------------------------------------------

def _encoded(d, p, L, seed):
    data = gen_bytes(seed, d * L).reshape(d, L)
    st, par = oracle.encode_sep(d, p, list(data))
    return [x.tobytes() for x in data] + [x.tobytes() for x in par]


def test_reconstruct_golden(golden):
    cache = {}
    for c in golden["reconstruct"]:
        key = (c["d"], c["p"], c["len"], c["seed"])
        if key not in cache:
            cache[key] = _encoded(*key)
        full = cache[key]
        rs = ce.ReedSolomon(c["d"], c["p"])
        shards = [None if i in c["missing"] else bytearray(full[i]) for i in range(len(full))]
        fn = rs.reconstruct_data if c["data_only"] else rs.reconstruct
        if c["status"] != 0:
            with pytest.raises(ce.Error) as e:
                fn(shards)
            assert e.value.code == c["status"]
            continue
        fn(shards)
        got = [None if s is None else sha(s) for s in shards]
        assert got == c["out_sha256"], (c["missing"], c["data_only"])


@pytest.mark.parametrize("d,p,L", [(3, 2, 683), (4, 3, 129), (5, 5, 1), (2, 6, 4096)])
def test_reconstruct_every_pattern(d, p, L):
    full = _encoded(d, p, L, d * 97 + L)
    rs = ce.ReedSolomon(d, p)
    t = d + p
    for k in range(1, p + 1):
        for miss in itertools.combinations(range(t), k):
            shards = [None if i in miss else bytearray(full[i]) for i in range(t)]
            rs.reconstruct(shards)
            assert [bytes(s) for s in shards] == full, miss
            shards = [None if i in miss else bytearray(full[i]) for i in range(t)]
            rs.reconstruct_data(shards)
            for i in range(t):
                if i < d:
                    assert bytes(shards[i]) == full[i]
                elif i in miss:
                    assert shards[i] is None


@pytest.mark.parametrize("d,p,L", [(128, 128, 1000), (1, 255, 4097), (255, 1, 513),
                                   (100, 156, 64)])
def test_max_shard_counts_vs_oracle(d, p, L):
    """The largest codes the crate allows (d + p = 256, galois_8's field size): encode, then the
    most erasures a part survives (p of them, drawn at random, data and parity mixed), through
    reconstruct and reconstruct_data, against the oracle."""
    full = _encoded(d, p, L, d * 7 + p)
    rs = ce.ReedSolomon(d, p)
    par = [bytearray(L) for _ in range(p)]
    rs.encode_sep(full[:d], par)
    assert [bytes(x) for x in par] == full[d:]
    t = d + p
    rng = np.random.default_rng(d * 1000 + p)
    for _ in range(3):
        miss = set(rng.choice(t, p, replace=False).tolist())
        shards = [None if i in miss else bytearray(full[i]) for i in range(t)]
        rs.reconstruct(shards)
        assert [bytes(s) for s in shards] == full, sorted(miss)[:8]
        shards = [None if i in miss else bytearray(full[i]) for i in range(t)]
        rs.reconstruct_data(shards)
        st, ref = oracle.reconstruct(d, p, [None if i in miss else full[i] for i in range(t)],
                                     data_only=True)
        assert st == 0
        for i in range(t):
            if i < d:
                assert bytes(shards[i]) == full[i] == bytes(ref[i]), i
            elif i in miss:
                assert shards[i] is None and ref[i] is None


@pytest.mark.parametrize("d,p,L", [(128, 128, 4096), (200, 56, 1000), (1, 255, 777),
                                   (255, 1, 4096)])
def test_max_shard_counts_device_batch(d, p, L):
    """The device-batch kernels at d + p = 256: fused encode + SHA-256 of every chunk, then
    reconstruct_batch with p erasures per part (a different random set per part, so the
    mixed-pattern kernel runs with up to p output rows), against the oracle and hashlib."""
    n, t = 3, d + p
    buf, batch = _device_parts(n, t, L, None, seed=d + 3 * p)
    rs = ce.ReedSolomon(d, p)
    dig = torch.zeros((n, t, 32), dtype=torch.uint8, device=DEV)
    ce.encode_hash_batch(rs, batch, dig.data_ptr())
    torch.cuda.synchronize()
    full, hd = buf.cpu().numpy().copy(), dig.cpu().numpy()
    for k in range(n):
        st, par = oracle.encode_sep(d, p, [full[k, j] for j in range(d)])
        assert st == 0
        for i in range(p):
            assert np.array_equal(full[k, d + i], par[i]), (k, i)
        for i in range(t):
            assert hd[k, i].tobytes() == hashlib.sha256(full[k, i].tobytes()).digest(), (k, i)
    rng = np.random.default_rng(t * 7 + L)
    for data_only in (False, True):
        present = np.ones((n, t), np.uint8)
        for k in range(n):
            present[k, rng.choice(t, p, replace=False)] = 0
        dev = torch.from_numpy(full).to(DEV)
        dev[torch.from_numpy(present == 0).to(DEV)] = 0
        buf.copy_(dev)
        ce.reconstruct_batch(rs, batch, present.tobytes(), data_only)
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        for k in range(n):
            for i in range(t):
                if present[k, i] or i < d or not data_only:
                    assert np.array_equal(got[k, i], full[k, i]), (data_only, k, i)
                else:
                    assert not got[k, i].any(), (data_only, k, i)  # parity left missing


def test_reconstruct_first_d_present_rule():
    """A corrupt shard beyond the first d present ones is never read (crate behaviour)."""
    d, p, L = 3, 3, 40
    full = _encoded(d, p, L, 12)
    rs = ce.ReedSolomon(d, p)
    shards = [None, bytearray(full[1]), bytearray(full[2]), bytearray(full[3]),
              bytearray(b"\xff" * L), bytearray(full[5])]
    rs.reconstruct_data(shards)
    assert bytes(shards[0]) == full[0]
    st, ref = oracle.reconstruct(d, p, [None, full[1], full[2], full[3], b"\xff" * L, full[5]])
    shards = [None, bytearray(full[1]), bytearray(full[2]), bytearray(full[3]),
              bytearray(b"\xff" * L), bytearray(full[5])]
    rs.reconstruct(shards)
    assert [bytes(s) for s in shards] == [bytes(r) for r in ref]


def test_reconstruct_errors_match_crate():
    rs = ce.ReedSolomon(3, 2)
    ok = b"abcd"
    cases = [
        ([ok] * 4, ce.TOO_FEW_SHARDS),
        ([ok] * 6, ce.TOO_MANY_SHARDS),
        ([ok, ok, b"abc", None, None], ce.INCORRECT_SHARD_SIZE),
        ([ok, b"", ok, None, None], ce.EMPTY_SHARD),
        ([ok, None, None, None, ok], ce.TOO_FEW_SHARDS_PRESENT),
    ]
    for shards, code in cases:
        with pytest.raises(ce.Error) as e:
            rs.reconstruct([None if s is None else bytearray(s) for s in shards])
        assert e.value.code == code
        assert oracle.reconstruct(3, 2, shards)[0] == code


# ----------------------------------------------------------------------------------------------
# Part layer (FilePart::write_with_encoder compute)
# ----------------------------------------------------------------------------------------------

def test_part_encode_cluster_fixture(golden):
    """tests/cluster.rs generator through d=3,p=2 parts of 2^10-byte chunks (7 parts)."""
    c = golden["cluster"]
    data = cluster_reader_bytes()
    rs = ce.ReedSolomon(c["d"], c["p"])
    step = c["d"] * c["chunk_size"]
    assert len(c["parts"]) == (len(data) + step - 1) // step
    for i, part in enumerate(c["parts"]):
        piece = data[i * step:(i + 1) * step]
        enc = ce.part_encode(rs, piece, len(piece))
        assert enc.chunksize == part["chunksize"]
        assert [str(h) for h in enc.hashes] == part["sha256"]


def test_part_encode_zeros_fixture(golden):
    """tests/file.rs:26-56: zeros of 2^23+7 bytes, 1 MiB chunks, (d, p) in 1..=3."""
    for z in golden["zeros"]:
        if (z["d"], z["p"]) not in [(1, 1), (3, 2), (2, 3)]:
            continue
        rs = ce.ReedSolomon(z["d"], z["p"])
        chunk = 1 << 20
        length = z["length"]
        step = z["d"] * chunk
        n_parts = 0
        for k, off in enumerate(range(0, length, step)):
            n = min(step, length - off)
            enc = ce.part_encode(rs, bytes(n), n)
            assert enc.chunksize == z["parts"][k]["chunksize"]
            assert [str(h) for h in enc.hashes] == z["parts"][k]["sha256"]
            n_parts += 1
        assert n_parts == z["n_parts"]


@pytest.mark.parametrize("d,p,length", [(3, 2, 1), (3, 2, 50 * (1 << 20) % (3 << 20) or 7),
                                        (10, 4, 10 * 65536 + 13), (20, 8, 20 * 4096)])
def test_part_encode_vs_oracle(d, p, length):
    buf = gen_bytes(length, length).tobytes()
    rs = ce.ReedSolomon(d, p)
    enc = ce.part_encode(rs, buf, length)
    cs, par, dig = oracle.part_encode(d, p, np.frombuffer(buf, np.uint8), length)
    assert enc.chunksize == cs
    assert [bytes(x) for x in enc.parity] == [x.tobytes() for x in par]
    assert [h.digest for h in enc.hashes] == [x.tobytes() for x in dig]


def test_host_api_concurrent_part_tasks_share_one_codec():
    """FileWriteBuilder runs up to `concurrency` (10) part tasks that share one
    Arc<ReedSolomon> (src/file/writer.rs:130-131,200-210) and call it from blocking threads, and
    reads rebuild concurrently too (reader.rs:63 buffered(5)).  The C-ABI must be thread-safe and
    reentrant: 10 threads hammer one codec with part_encode / reconstruct / sha256 (ctypes drops
    the GIL during each call) and every result must equal the oracle's."""
    from concurrent.futures import ThreadPoolExecutor

    d, p = 10, 4
    rs = ce.ReedSolomon(d, p)

    def task(i):
        length = 10 * 4096 + 97 * i + 1
        buf = gen_bytes(1000 + i, length).tobytes()
        for _ in range(3):
            enc = ce.part_encode(rs, buf, length)
            cs, par, dig = oracle.part_encode(d, p, np.frombuffer(buf, np.uint8), length)
            assert enc.chunksize == cs
            assert [bytes(x) for x in enc.parity] == [x.tobytes() for x in par]
            assert [h.digest for h in enc.hashes] == [x.tobytes() for x in dig]
            data = np.frombuffer(buf + bytes(d * cs - length), np.uint8).reshape(d, cs)
            shards = [bytearray(data[j].tobytes()) for j in range(d)] + \
                     [bytearray(bytes(x)) for x in enc.parity]
            full = [bytes(x) for x in shards]
            lost = [(i + k * 3) % (d + p) for k in range(1 + i % p)]
            for k in lost:
                shards[k] = None
            rs.reconstruct(shards)
            assert [bytes(x) for x in shards] == full
        return i

    with ThreadPoolExecutor(max_workers=10) as ex:
        assert sorted(ex.map(task, range(20))) == list(range(20))


def test_per_call_coalescing_batches_concurrent_parts_bit_exact():
    """Concurrent cec_part_encode / cec_sha256 calls (the reference's part tasks) share launches
    through the coalescing queue; every caller still gets exactly its own part's parity and
    digests (vs the oracle), including callers with a different chunk length in the mix."""
    from concurrent.futures import ThreadPoolExecutor

    d, p = 10, 4
    rs = ce.ReedSolomon(d, p)
    c0, l0 = ce.coalesce_stats()

    def task(i):
        length = 10 * 65536 if i % 5 else 10 * 4096 + 3  # two chunk lengths in flight
        buf = gen_bytes(5000 + i, length).tobytes()
        enc = ce.part_encode(rs, buf, length)
        cs, par, dig = oracle.part_encode(d, p, np.frombuffer(buf, np.uint8), length)
        assert enc.chunksize == cs
        assert [bytes(x) for x in enc.parity] == [x.tobytes() for x in par]
        assert [h.digest for h in enc.hashes] == [x.tobytes() for x in dig]
        msg = gen_bytes(9000 + i, 1000 + 37 * i).tobytes()
        assert ce.Sha256Hash.from_buf(msg).digest == hashlib.sha256(msg).digest()
        return i

    with ThreadPoolExecutor(max_workers=48) as ex:
        assert sorted(ex.map(task, range(96))) == list(range(96))
    c1, l1 = ce.coalesce_stats()
    assert c1 - c0 == 2 * 96
    assert l1 - l0 < c1 - c0  # some calls shared a launch


# ----------------------------------------------------------------------------------------------
# Device-resident batches
# ----------------------------------------------------------------------------------------------

def _device_parts(n_parts, t, L, cstride=None, seed=1):
    cstride = cstride or L
    buf = torch.zeros((n_parts, t, cstride), dtype=torch.uint8, device=DEV)
    batch = ce.PartBatch.from_tensor(buf, L)
    ce.fill_synthetic(batch, t, seed)
    return buf, batch


@pytest.mark.parametrize("d,p,L,cstride", [
    (10, 4, 65536, None),          # aligned fast path
    (10, 4, 65536 + 13, 65536 + 16),  # aligned strides, ragged tail
    (3, 2, 683, 683),              # odd stride: unaligned path (reference's packed slices)
    (20, 8, 4096, None),
    (6, 10, 1000, 1008),           # > 8 output rows: two row groups
    (10, 4, 20512, None),          # aligned, last step partial: 2-column + single-column tails
])
def test_encode_hash_batch_vs_oracle(d, p, L, cstride):
    n_parts, t = 24, d + p
    buf, batch = _device_parts(n_parts, t, L, cstride, seed=d * 31 + L)
    # synthetic generator mirror: spot-check a few bytes against the host mirror
    host_before = buf.cpu().numpy()
    for (k, c, o) in [(0, 0, 0), (3, 1, L - 1), (n_parts - 1, d - 1, L // 2)]:
        assert host_before[k, c, o] == ce.synth_byte(d * 31 + L, k, c, o)
    dig = torch.zeros((n_parts, t, 32), dtype=torch.uint8, device=DEV)
    rs = ce.ReedSolomon(d, p)
    ce.encode_hash_batch(rs, batch, dig.data_ptr())
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    hdig = dig.cpu().numpy()
    for k in range(n_parts):
        st, par = oracle.encode_sep(d, p, [host[k, j, :L] for j in range(d)])
        for i in range(p):
            assert np.array_equal(host[k, d + i, :L], par[i]), (k, i)
        for j in range(t):
            assert hdig[k, j].tobytes() == hashlib.sha256(host[k, j, :L].tobytes()).digest()
    # bytes past chunk_len in the stride padding are untouched
    if cstride and cstride > L:
        assert not host[:, d:, L:].any()


@pytest.mark.parametrize("variant", ["1", "2"])
def test_sha256_batch_subrange(variant, knob_env):
    knob_env.set("CEC_SHA_VARIANT", variant)
    d, p, L = 4, 2, 5000
    buf, batch = _device_parts(8, d + p, L, 5008, seed=5)
    dig = torch.zeros((8, 3, 32), dtype=torch.uint8, device=DEV)
    ce.sha256_batch(batch, 2, 3, dig.data_ptr())
    torch.cuda.synchronize()
    host, hd = buf.cpu().numpy(), dig.cpu().numpy()
    for k in range(8):
        for c in range(3):
            assert hd[k, c].tobytes() == hashlib.sha256(host[k, 2 + c, :L].tobytes()).digest()


@pytest.mark.parametrize("data_only", [False, True])
@pytest.mark.parametrize("d,p,L", [(10, 4, 16384), (3, 2, 683), (20, 8, 4096 + 5),
                                   (10, 4, 12368),   # partial last 8 KiB step (2-column path)
                                   (10, 6, 3 * 8192 + 16),  # compile-time d=10, 8-row class
                                   (6, 10, 1024)])   # up to 10 rows: shared + row-group launches
def test_reconstruct_batch_random_patterns(d, p, L, data_only):
    n_parts, t = 96, d + p
    buf, batch = _device_parts(n_parts, t, L, None, seed=L + d)
    rs = ce.ReedSolomon(d, p)
    ce.encode_batch(rs, batch)
    ref = buf.clone()
    rng = np.random.default_rng(d * 7 + L)
    present = np.ones((n_parts, t), dtype=np.uint8)
    for k in range(n_parts):
        n_miss = k % (p + 1)  # includes parts with nothing missing
        present[k, rng.choice(t, n_miss, replace=False)] = 0
    # erase (zero) the missing chunks
    mask = torch.from_numpy(present).to(DEV).bool()
    buf[~mask] = 0
    ce.reconstruct_batch(rs, batch, present.tobytes(), data_only)
    torch.cuda.synchronize()
    got, want = buf.cpu().numpy(), ref.cpu().numpy()
    for k in range(n_parts):
        for i in range(t):
            if present[k, i] or i < d or not data_only:
                assert np.array_equal(got[k, i], want[k, i]), (k, i)
            else:  # data_only leaves missing parity untouched (None in the crate)
                assert not got[k, i].any()
    # cross-check a few parts against the oracle's reconstruct on the erased inputs
    for k in range(0, n_parts, 17):
        shards = [want[k, i].tobytes() if present[k, i] else None for i in range(t)]
        st, out = oracle.reconstruct(d, p, shards, data_only=data_only)
        assert st == 0
        for i in range(t):
            if out[i] is not None:
                assert out[i].tobytes() == got[k, i].tobytes()


@pytest.mark.parametrize("d,p,max_miss", [(10, 4, 1), (10, 4, 2), (10, 4, 3), (20, 8, 5),
                                          (20, 8, 8)])
def test_reconstruct_row_classes(d, p, max_miss):
    """The shared reconstruct launch compiles its kernel for the batch's widest pattern rounded
    up to 2, 4 or 8 rows (rs_kernels.hip launch_rs_apply_var): batches whose widest pattern sits
    on each side of a class boundary rebuild every chunk bit-exact, data + parity."""
    n_parts, t, L = 64, d + p, 2 * 8192 + 48
    buf, batch = _device_parts(n_parts, t, L, None, seed=d * 100 + max_miss)
    rs = ce.ReedSolomon(d, p)
    ce.encode_batch(rs, batch)
    ref = buf.clone()
    rng = np.random.default_rng(max_miss)
    present = np.ones((n_parts, t), dtype=np.uint8)
    for k in range(n_parts):
        present[k, rng.choice(t, 1 + k % max_miss, replace=False)] = 0
    buf[~torch.from_numpy(present).to(DEV).bool()] = 0
    ce.reconstruct_batch(rs, batch, present.tobytes(), False)
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    want = ref.cpu().numpy()
    k = n_parts - 1
    shards = [want[k, i].tobytes() if present[k, i] else None for i in range(t)]
    st, out = oracle.reconstruct(d, p, shards, data_only=False)
    assert st == 0 and all(out[i].tobytes() == want[k, i].tobytes() for i in range(t))


def test_reconstruct_batch_too_few_present_launches_nothing():
    d, p, L = 3, 2, 256
    buf, batch = _device_parts(4, d + p, L, None, seed=9)
    rs = ce.ReedSolomon(d, p)
    before = buf.clone()
    present = np.ones((4, d + p), dtype=np.uint8)
    present[2, :3] = 0  # 2 present < d
    with pytest.raises(ce.Error) as e:
        ce.reconstruct_batch(rs, batch, present.tobytes(), False)
    assert e.value.code == ce.TOO_FEW_SHARDS_PRESENT
    torch.cuda.synchronize()
    assert torch.equal(buf, before)


# ----------------------------------------------------------------------------------------------
# Full BASELINE shapes: size-independent properties
# ----------------------------------------------------------------------------------------------

def test_large_grid_capped_paths_ragged_length():
    """The paths that only large grids take (>= 65 536 blocks: residency caps, rs_kernels.hip
    apply_lds) at a ragged length (full 8 KiB bit-sliced steps + the v_perm byte tail): the
    bit-sliced encode must reproduce the fused kernel's parity byte for byte, the 2-row
    (data-only, 2 erasures) and 4-row (1-4 erasures, data + parity) reconstruct classes with
    the compile-time-d loop must rebuild chunks that hash to the fused step's digests, and a
    sampled part must match the oracle."""
    d, p, n_parts = 10, 4, 640
    L = (1 << 20) - 4096 + 48  # 128 tiles of 8 KiB, the last one ragged: 81 920 blocks
    t = d + p
    buf = torch.empty((n_parts, t, L), dtype=torch.uint8, device=DEV)
    batch = ce.PartBatch.from_tensor(buf, L)
    ce.fill_synthetic(batch, t, 5151)
    rs = ce.ReedSolomon(d, p)
    dig = torch.empty((n_parts, t, 32), dtype=torch.uint8, device=DEV)
    ce.encode_hash_batch(rs, batch, dig.data_ptr())
    torch.cuda.synchronize()
    ref = buf.clone()
    buf[:, d:] = 0
    ce.encode_batch(rs, batch)  # the bit-sliced kernel under the cap
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    k = n_parts // 3
    host = ref[k].cpu().numpy()
    st, par = oracle.encode_sep(d, p, [host[j] for j in range(d)])
    assert st == 0 and all(np.array_equal(host[d + i], par[i]) for i in range(p))
    rng = np.random.default_rng(51)
    for data_only, lo, hi in ((True, 2, 2), (False, 1, p)):
        present = np.ones((n_parts, t), dtype=np.uint8)
        for j in range(n_parts):
            present[j, rng.choice(t, int(rng.integers(lo, hi + 1)), replace=False)] = 0
        buf[~torch.from_numpy(present).to(DEV).bool()] = 0
        ce.reconstruct_batch(rs, batch, present.tobytes(), data_only)
        torch.cuda.synchronize()
        if data_only:
            assert torch.equal(buf[:, :d], ref[:, :d])
            buf.copy_(ref)
        else:
            dig2 = torch.empty_like(dig)
            ce.sha256_batch(batch, 0, t, dig2.data_ptr())
            torch.cuda.synchronize()
            assert torch.equal(dig, dig2) and torch.equal(buf, ref)
    del buf, ref
    torch.cuda.empty_cache()


@pytest.mark.slow
@pytest.mark.parametrize("d,p,L,n_parts", [(10, 4, 1 << 20, 4096), (20, 8, 256 << 10, 2048),
                                           (20, 8, 256 << 10, 4096)])  # C4 bench shape: the
# two-SHA-wave ENC3 / big-endian-ring build at 256 KiB
def test_full_size_encode_erase_reconstruct_roundtrip(d, p, L, n_parts):
    """C2 / C4 at full size: encode+hash, sampled parts vs oracle, then erase 1..p chunks per
    part, reconstruct, and re-hash: every digest must match the encode-time digest."""
    t = d + p
    buf = torch.empty((n_parts, t, L), dtype=torch.uint8, device=DEV)
    batch = ce.PartBatch.from_tensor(buf, L)
    ce.fill_synthetic(batch, t, 424242)
    rs = ce.ReedSolomon(d, p)
    dig = torch.empty((n_parts, t, 32), dtype=torch.uint8, device=DEV)
    ce.encode_hash_batch(rs, batch, dig.data_ptr())
    torch.cuda.synchronize()
    for k in (0, n_parts // 2 + 1, n_parts - 1):
        host = buf[k].cpu().numpy()
        st, par = oracle.encode_sep(d, p, [host[j] for j in range(d)])
        for i in range(p):
            assert np.array_equal(host[d + i], par[i])
        hd = dig[k].cpu().numpy()
        for j in range(t):
            assert hd[j].tobytes() == hashlib.sha256(host[j].tobytes()).digest()
    rng = np.random.default_rng(7)
    present = np.ones((n_parts, t), dtype=np.uint8)
    for k in range(n_parts):
        present[k, rng.choice(t, int(rng.integers(1, p + 1)), replace=False)] = 0
    mask = torch.from_numpy(present).to(DEV).bool()
    buf[~mask] = 0
    ce.reconstruct_batch(rs, batch, present.tobytes(), False)
    dig2 = torch.empty_like(dig)
    ce.sha256_batch(batch, 0, t, dig2.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dig, dig2)


# ----------------------------------------------------------------------------------------------
# Fused encode+hash kernel vs the separate kernels and the oracle
# ----------------------------------------------------------------------------------------------

@pytest.mark.parametrize("d,p,L,cstride,n_parts,mode", [(*c, "0")[:6] for c in [
    (10, 4, 4096 + 13, 4112, 40),     # ragged tail, 16 parts per workgroup, 3 workgroups
    (10, 4, 64, None, 17),            # exactly one SHA block, last workgroup with 1 part
    (10, 4, 4096 + 48, None, 19),     # RS(10,4) shape build with a 48-byte message tail
    (10, 4, 256 + 16, None, 7),       # shape build, tail 16 bytes in the second step
    (10, 4, 63, 64, 5),               # shorter than a block (tail only)
    (10, 4, 4096, None, 4100),        # > 256 workgroups: two passes
    (16, 8, 1000, 1008, 21),          # largest fused d; generic (p != 4) parity-row path
    (12, 3, 777, 784, 9),
    (1, 1, 1000, 1008, 17),
    (3, 2, 100, 112, 300),
    (3, 2, 683, 683, 30),             # odd stride: unaligned -> separate kernels
    (20, 8, 200, 208, 40),            # RS(20,8) build, 128-byte steps
    (20, 8, 256 * 1024, None, 20),    # C4 chunk shape
    (20, 4, 1000, 1008, 11),          # RS(20,p<8) on the p <= 8 build
    (20, 8, 1024, None, 2400),        # > 65 536 chunks: two SHA waves per SIMD, 64-byte steps
    (20, 4, 512 + 8, None, 2800),
    (24, 4, 300, 304, 5),             # d > 16, d != 20 -> separate kernels
    (6, 10, 500, 512, 4),             # p > 8 -> separate kernels
    (16, 8, 4096, None, 30),          # p = 8, d = 16: 128-byte steps (LDS budget)
    (10, 4, 4096 + 13, 4112, 40, "3"),  # generic-d build on the RS(10,4) shape
    (10, 4, 64, None, 17, "3"),
    (20, 8, 64 * 3 + 8, None, 4096),       # C4 part count: 16 parts/CU, encoders on SIMD 3
]])
def test_fused_encode_hash_matches_separate_and_oracle(d, p, L, cstride, n_parts, mode,
                                                       knob_env):
    knob_env.set("CEC_FUSED_MODE", mode)
    knob_env.set("CEC_FUSED", "1")  # the fused kernel whatever the batch size
    t = d + p
    buf, batch = _device_parts(n_parts, t, L, cstride, seed=L * 3 + d)
    ref = buf.clone()
    rs = ce.ReedSolomon(d, p)
    dig = torch.zeros((n_parts, t, 32), dtype=torch.uint8, device=DEV)
    ce.encode_hash_batch(rs, batch, dig.data_ptr())  # fused (p <= 8)
    fused_buf = buf.clone()
    buf.copy_(ref)
    dig2 = torch.zeros_like(dig)
    knob_env.set("CEC_FUSED", "0")
    ce.encode_hash_batch(rs, batch, dig2.data_ptr())  # encode kernel + sha256 kernel
    torch.cuda.synchronize()
    assert torch.equal(fused_buf, buf)
    assert torch.equal(dig, dig2)
    host, hd = buf.cpu().numpy(), dig.cpu().numpy()
    for k in sorted({0, n_parts // 2, n_parts - 1}):
        st, par = oracle.encode_sep(d, p, [host[k, j, :L] for j in range(d)])
        for i in range(p):
            assert np.array_equal(host[k, d + i, :L], par[i])
        for j in range(t):
            assert hd[k, j].tobytes() == hashlib.sha256(host[k, j, :L].tobytes()).digest()


# ----------------------------------------------------------------------------------------------
# Host-staged write pipeline
# ----------------------------------------------------------------------------------------------

@pytest.mark.parametrize("d,p,L,parts,depth,batches", [
    (10, 4, 4096, 16, 3, 7),      # more batches than slots: slot reuse
    (3, 2, 683, 5, 2, 3),         # odd chunk length (padded device stride)
    (20, 8, 1000, 4, 4, 4),
])
def test_pipeline_matches_oracle(d, p, L, parts, depth, batches):
    rs = ce.ReedSolomon(d, p)
    pl = ce.Pipeline(rs, L, parts, depth)
    sent, done, pending = {}, {}, {}
    for b in range(batches):
        slot, data = pl.acquire()  # waits for this slot's previous batch: collect it first
        if slot in pending:
            done[pending[slot]] = tuple(x.copy() for x in pl.wait(slot))
        n = parts if b % 2 == 0 else max(1, parts - 1)
        data[:n] = gen_bytes(700 + b, n * d * L).reshape(n, d, L)
        sent[b] = (slot, data[:n].copy())
        pl.submit(slot, n)  # up to `depth` batches in flight
        pending[slot] = b
    for slot, b in pending.items():
        if b not in done:
            done[b] = tuple(x.copy() for x in pl.wait(slot))
    pl.drain()
    for b, (slot, data) in sent.items():
        parity, digests = done[b]
        for k in range(data.shape[0]):
            st, par = oracle.encode_sep(d, p, [data[k, j] for j in range(d)])
            for i in range(p):
                assert np.array_equal(parity[k, i], par[i]), (b, k, i)
            chunks = [data[k, j] for j in range(d)] + par
            for j in range(d + p):
                assert digests[k, j].tobytes() == hashlib.sha256(chunks[j].tobytes()).digest()


@pytest.mark.parametrize("d,p,L,parts,depth,batches", [
    (10, 4, 4096, 12, 3, 5),      # more batches than slots: slot reuse
    (3, 2, 683, 9, 2, 3),         # odd chunk length (padded device stride)
    (20, 8, 1000, 6, 2, 2),
])
@pytest.mark.parametrize("flags", [0, ce.ReadPipeline.REBUILT_ONLY])
def test_read_pipeline_matches_read_with_context(d, p, L, parts, depth, batches, flags):
    """FileReadBuilder's loop batched: per part the loaded chunks (all; d random ones like
    file_part.rs:97; fewer than d; a corrupted loaded chunk with enough others; a corrupted one
    without), verification against the metadata digests, and the part's data rebuilt from the
    verified chunks.  Data must equal the written bytes; flags and statuses as the reference's
    read would see them (TooFewShardsPresent when fewer than d verify)."""
    t = d + p
    rs = ce.ReedSolomon(d, p)
    rp = ce.ReadPipeline(rs, L, parts, depth, flags)
    rng = np.random.default_rng(d * 100 + L)
    pending, want = {}, {}

    def check(b, slot):
        # before the slot's chunk buffer is refilled: REBUILT_ONLY data points into it
        data, ver, status = rp.wait(slot)
        exp_data, exp_ok, exp_status = want[b]
        assert list(status) == exp_status, b
        assert np.array_equal(ver, exp_ok), b
        for k, st in enumerate(exp_status):
            if st == 0:
                got = rp.part_bytes(slot, len(exp_status), k)
                assert got == exp_data[k].tobytes(), (b, k)
                if not flags:
                    assert np.array_equal(data[k], exp_data[k]), (b, k)

    for b in range(batches):
        slot, chunks, present, expected = rp.acquire()
        if slot in pending:
            check(pending[slot], slot)
        n = parts if b % 2 == 0 else parts - 1
        exp_data, exp_ok, exp_status = [], np.zeros((n, t), np.uint8), []
        for k in range(n):
            dat = gen_bytes(3000 + 97 * b + k, d * L).reshape(d, L)
            st, par = oracle.encode_sep(d, p, list(dat))
            full = [dat[j] for j in range(d)] + par
            for i in range(t):
                chunks[k, i] = full[i]
                expected[k, i] = np.frombuffer(hashlib.sha256(full[i].tobytes()).digest(), np.uint8)
            kind = (k + b) % 5
            if kind == 0:
                loaded = list(range(t))
            elif kind == 1:
                loaded = sorted(rng.choice(t, d, replace=False))
            elif kind == 2:
                loaded = sorted(rng.choice(t, d - 1, replace=False))
            else:
                loaded = sorted(rng.choice(t, d + 1 if kind == 3 else d, replace=False))
            present[k] = 0
            present[k, loaded] = 1
            ok = present[k].copy()
            if kind >= 3:  # corrupt one loaded chunk (a data chunk if one is loaded)
                victim = next((i for i in loaded if i < d), loaded[0])
                chunks[k, victim, L // 2] ^= 0x5A
                ok[victim] = 0
            exp_ok[k] = ok
            exp_status.append(0 if ok.sum() >= d else 10)
            exp_data.append(dat)
        rp.submit(slot, n)
        pending[slot] = b
        want[b] = (exp_data, exp_ok, exp_status)
    for slot, b in pending.items():
        check(b, slot)
    rp.drain()


@pytest.mark.parametrize("d,p,L,parts,depth,batches", [
    (10, 4, 4096, 12, 3, 5),
    (3, 2, 683, 9, 2, 3),         # odd chunk length: byte-wise placement kernel
])
@pytest.mark.parametrize("flags", [0, ce.ReadPipeline.REBUILT_ONLY])
@pytest.mark.parametrize("pinned", [False, True])
def test_read_pipeline_packed_submit(d, p, L, parts, depth, batches, flags, pinned):
    """cec_read_pipeline_submit_packed: the loaded chunks back to back in (part, index) order,
    one upload per batch and the move kernel placing them.  Same loaded sets and corruption as
    the unpacked test; data, flags and statuses as the oracle's rules give them, and the
    REBUILT_ONLY data_chunks pointers of loaded chunks point into the packed buffer."""
    t = d + p
    rs = ce.ReedSolomon(d, p)
    rp = ce.ReadPipeline(rs, L, parts, depth, flags | ce.PIPE_EXTERNAL)
    rng = np.random.default_rng(d * 31 + L)
    pending, want, keep = {}, {}, {}
    outs = [ce.HostBuffer(parts * d * L) for _ in range(depth)]

    def check(b, slot):
        data, ver, status = rp.wait(slot)
        exp_data, exp_ok, exp_status, packed, loaded_of = want[b]
        assert list(status) == exp_status, b
        assert np.array_equal(ver, exp_ok), b
        ptrs = rp.data_chunks(slot, len(exp_status))
        base = packed.ptr if pinned else packed.ctypes.data
        for k, st in enumerate(exp_status):
            if st != 0:
                continue
            assert rp.part_bytes(slot, len(exp_status), k) == exp_data[k].tobytes(), (b, k)
            if flags and exp_ok[k].sum() == len(loaded_of[k]):  # no redo: loaded data in place
                for j in range(d):
                    if j in loaded_of[k]:
                        pos = loaded_of[k][j]
                        assert int(ptrs[k, j]) == base + pos * L, (b, k, j)

    for b in range(batches):
        slot, _, present, expected = rp.acquire()
        if slot in pending:
            check(pending[slot], slot)
        n = parts if b % 2 == 0 else parts - 1
        exp_data, exp_ok, exp_status, pieces, loaded_of = [], np.zeros((n, t), np.uint8), [], [], []
        present_arr = np.zeros((n, t), np.uint8)
        expected_arr = np.zeros((n, t, 32), np.uint8)
        pos = 0
        for k in range(n):
            dat = gen_bytes(5000 + 97 * b + k, d * L).reshape(d, L)
            st, par = oracle.encode_sep(d, p, list(dat))
            full = [dat[j].copy() for j in range(d)] + [x.copy() for x in par]
            for i in range(t):
                expected_arr[k, i] = np.frombuffer(hashlib.sha256(full[i].tobytes()).digest(),
                                                   np.uint8)
            kind = (k + b) % 5
            if kind == 0:
                loaded = list(range(t))
            elif kind == 1:
                loaded = sorted(rng.choice(t, d, replace=False).tolist())
            elif kind == 2:
                loaded = sorted(rng.choice(t, d - 1, replace=False).tolist())
            else:
                loaded = sorted(rng.choice(t, d + 1 if kind == 3 else d, replace=False).tolist())
            present_arr[k, loaded] = 1
            ok = present_arr[k].copy()
            if kind >= 3:
                victim = next((i for i in loaded if i < d), loaded[0])
                full[victim][L // 2] ^= 0x5A
                ok[victim] = 0
            where = {}
            for i in loaded:
                pieces.append(full[i])
                where[i] = pos
                pos += 1
            loaded_of.append(where)
            exp_ok[k] = ok
            exp_status.append(0 if ok.sum() >= d else 10)
            exp_data.append(dat)
        flat = np.concatenate(pieces) if pieces else np.zeros(0, np.uint8)
        if pinned:
            packed = ce.HostBuffer(max(flat.size, 1))
            packed.array[: flat.size] = flat
        else:
            packed = flat
        rp.submit_packed(slot, packed, present_arr, expected_arr, n, outs[slot])
        keep[slot] = packed
        pending[slot] = b
        want[b] = (exp_data, exp_ok, exp_status, packed, loaded_of)
    for slot, b in pending.items():
        check(b, slot)
    rp.drain()


# ----------------------------------------------------------------------------------------------
# Verify / read / resilver (FilePart::verify, read_with_context, resilver compute)
# ----------------------------------------------------------------------------------------------

def _encoded_batch(d, p, L, n_parts, seed):
    t = d + p
    buf, batch = _device_parts(n_parts, t, L, None, seed=seed)
    rs = ce.ReedSolomon(d, p)
    dig = torch.zeros((n_parts, t, 32), dtype=torch.uint8, device=DEV)
    ce.encode_hash_batch(rs, batch, dig.data_ptr())
    torch.cuda.synchronize()
    return rs, buf, batch, dig


@pytest.mark.parametrize("variant", ["1", "2"])  # skip path of both kernels
def test_verify_batch_flags(variant, knob_env):
    knob_env.set("CEC_SHA_VARIANT", variant)
    d, p, L, n = 4, 2, 3000, 10
    rs, buf, batch, dig = _encoded_batch(d, p, L, n, 31)
    t = d + p
    buf[3, 1, 17] ^= 0x01            # corrupt one chunk
    present = torch.ones((n, t), dtype=torch.uint8, device=DEV)
    present[5, 4] = 0                # absent chunk: not read, ok = 0
    ok = torch.full((n, t), 7, dtype=torch.uint8, device=DEV)
    ce.verify_batch(batch, 0, t, dig.data_ptr(), ok.data_ptr(), present.data_ptr())
    torch.cuda.synchronize()
    want = torch.ones((n, t), dtype=torch.uint8)
    want[3, 1] = 0
    want[5, 4] = 0
    assert torch.equal(ok.cpu(), want)


@pytest.mark.parametrize("speculate", ["1"])  # CEC_READ_SPECULATE=0: A/B build only
def test_read_batch_restores_data_and_reports_undecodable_parts(speculate, knob_env):
    """file_part.rs:86-129 batched.  speculate=1: the decode runs from the loaded chunks
    alongside verification and is redone for parts with a failed chunk; 0: verify, then decode
    (CEC_READ_SPECULATE A/B knob).  Both must give the verified decode."""
    knob_env.set("CEC_READ_SPECULATE", speculate)
    d, p, L, n = 10, 4, 4096 + 5, 12
    rs, buf, batch, dig = _encoded_batch(d, p, L, n, 41)
    t = d + p
    ref = buf.clone()
    present = np.ones((n, t), dtype=np.uint8)
    present[0, [0, 3]] = 0           # two data chunks not fetched
    buf[1, 2, 100] ^= 0xFF           # a fetched chunk that fails its hash
    present[2, [0, 1, 2, 3, 4]] = 0  # 9 chunks left < d: undecodable
    buf[4, 13, 0] ^= 1               # corrupt parity: data intact, nothing to rebuild
    present[5, 1] = 0                # missing data chunk AND a corrupt chunk among the first d
    buf[5, 4, 7] ^= 0x10             # loaded: the speculative decode used it, must be redone
    present[6, [0, 1, 2, 3]] = 0     # exactly d loaded, one fails: < d verified, undecodable
    buf[6, 5, 0] ^= 0x80
    present[7, [10, 11, 12, 13]] = 0  # only the d data chunks loaded: nothing to rebuild
    present[8, [1, 6, 10, 12]] = 0   # d random chunks (the reference's read), one of them
    buf[8, 13, 9] ^= 2               # (parity 13) corrupt: 9 verified, undecodable
    for k, i in [(0, 0), (0, 3), (2, 0), (5, 1), (8, 1), (8, 6)]:
        buf[k, i] = 0
    before = buf.cpu()
    verified, status = ce.read_batch(rs, batch, present.tobytes(), dig.data_ptr())
    torch.cuda.synchronize()
    v = np.frombuffer(verified, np.uint8).reshape(n, t)
    assert v[1, 2] == 0 and v[0, 0] == 0 and v[4, 13] == 0 and v[3].all()
    assert v[5, 4] == 0 and v[5, 1] == 0 and v[6, 5] == 0 and v[8, 13] == 0
    bad = {2, 6, 8}                   # part 8: 9 verified after losing parity 13
    assert [status[k] for k in sorted(bad)] == [ce.TOO_FEW_SHARDS_PRESENT] * 3
    assert all(status[k] == ce.OK for k in range(n) if k not in bad)
    got, want = buf.cpu(), ref.cpu()
    for k in range(n):
        if k in bad:
            # loaded chunks of an undecodable part are never written
            for i in range(t):
                if present[k, i]:
                    assert torch.equal(got[k, i], before[k, i]), (k, i)
            continue
        assert torch.equal(got[k, :d], want[k, :d]), k   # data chunks are the read's output


def test_read_batch_present_flag_values():
    """ABI 2: only CEC_PRESENT_VERIFIED (0x80) marks a loaded chunk as trusted (used, not hashed
    again).  Any other nonzero flag -- 2 included, the ABI-1 value of the trusted mark -- means
    loaded and hashed, so a corrupt chunk flagged 2 (or 3, or 0xFF) is caught."""
    d, p, L, n = 4, 2, 1024, 4
    rs, buf, batch, dig = _encoded_batch(d, p, L, n, 47)
    t = d + p
    ref = buf.clone()
    present = np.ones((n, t), dtype=np.uint8)
    for k, flag in enumerate([2, 3, 0xFF, ce.PRESENT_VERIFIED]):
        present[k, 1] = flag
        buf[k, 1, 5] ^= 0x40  # the flagged chunk is corrupt
    verified, status = ce.read_batch(rs, batch, present.tobytes(), dig.data_ptr())
    torch.cuda.synchronize()
    v = np.frombuffer(verified, np.uint8).reshape(n, t)
    for k in range(3):  # hashed: fails, dropped, data chunk 1 rebuilt from the other 5
        assert v[k, 1] == 0 and status[k] == ce.OK, k
        assert torch.equal(buf[k, :d].cpu(), ref[k, :d].cpu()), k
    # trusted without hashing: reported verified and used as loaded (the caller vouched for it)
    assert v[3, 1] == 1 and status[3] == ce.OK
    assert ce.PRESENT_VERIFIED == 0x80 and ce.abi_version() == 3


@pytest.mark.parametrize("variant", ["1", "2"])  # compacted item list in both SHA kernels
@pytest.mark.parametrize("speculate", ["1"])  # CEC_READ_SPECULATE=0: A/B build only
def test_read_batch_random_patterns_vs_oracle(speculate, variant, knob_env):
    knob_env.set("CEC_SHA_VARIANT", variant)
    """d random chunks loaded per part (reader.rs / file_part.rs:86-122), a few corrupted;
    the rebuilt data chunks equal the oracle's reconstruct_data from the verified chunks."""
    knob_env.set("CEC_READ_SPECULATE", speculate)
    d, p, L, n = 10, 4, 1 << 12, 64
    rs, buf, batch, dig = _encoded_batch(d, p, L, n, 43)
    t = d + p
    ref = buf.cpu().numpy().copy()
    rng = np.random.default_rng(7)
    present = np.zeros((n, t), dtype=np.uint8)
    for k in range(n):
        present[k, rng.choice(t, size=d + int(rng.integers(0, p + 1)), replace=False)] = 1
    host = buf.cpu().numpy()
    host[present == 0] = 0
    corrupt = rng.choice(n, size=8, replace=False)
    for k in corrupt:
        i = int(rng.choice(np.flatnonzero(present[k])))
        host[k, i, int(rng.integers(0, L))] ^= 1 << int(rng.integers(0, 8))
    buf.copy_(torch.from_numpy(host))
    verified, status = ce.read_batch(rs, batch, present.tobytes(), dig.data_ptr())
    torch.cuda.synchronize()
    v = np.frombuffer(verified, np.uint8).reshape(n, t)
    got = buf.cpu().numpy()
    for k in range(n):
        good = v[k].astype(bool)
        assert np.array_equal(good, present[k].astype(bool) & (host[k] == ref[k]).all(1)), k
        if good.sum() < d:
            assert status[k] == ce.TOO_FEW_SHARDS_PRESENT
            continue
        assert status[k] == ce.OK
        shards = [ref[k, i] if good[i] else None for i in range(t)]
        st, out = oracle.reconstruct(d, p, shards, data_only=True)
        assert st == 0
        for i in range(d):
            assert np.array_equal(got[k, i], out[i]), (k, i)


def test_resilver_batch_cluster_style():
    """tests/cluster.rs:145-231: delete data[0] and parity[0] of every part, resilver, verify
    is ideal again (every chunk matches its digest)."""
    d, p, L, n = 3, 2, 683, 7
    rs, buf, batch, dig = _encoded_batch(d, p, L, n, 51)
    t = d + p
    ref = buf.clone()
    buf[:, 0] = 0
    buf[:, d] = 0
    present = np.ones((n, t), dtype=np.uint8)
    present[:, 0] = 0
    present[:, d] = 0
    verified, status = ce.resilver_batch(rs, batch, present.tobytes(), dig.data_ptr())
    assert status == [ce.OK] * n
    ok = torch.zeros((n, t), dtype=torch.uint8, device=DEV)
    ce.verify_batch(batch, 0, t, dig.data_ptr(), ok.data_ptr())
    torch.cuda.synchronize()
    assert bool(ok.all())
    assert torch.equal(buf, ref)


@pytest.mark.parametrize("speculate", ["1"])  # CEC_READ_SPECULATE=0: A/B build only
def test_resilver_batch_random_patterns_with_corruption(speculate, knob_env):
    """FilePart::resilver compute (file_part.rs:253-308) batched: random loaded sets (d..d+p),
    some loaded chunks corrupted (including ones the speculative decode uses); every decodable
    part ends with all d+p chunks equal to the written ones, flags mark the bad chunks."""
    knob_env.set("CEC_READ_SPECULATE", speculate)
    d, p, L, n = 6, 3, 2048 + 7, 40
    rs, buf, batch, dig = _encoded_batch(d, p, L, n, 61)
    t = d + p
    ref = buf.cpu().numpy().copy()
    rng = np.random.default_rng(11)
    present = np.zeros((n, t), dtype=np.uint8)
    for k in range(n):
        present[k, rng.choice(t, size=d + int(rng.integers(0, p + 1)), replace=False)] = 1
    host = ref.copy()
    host[present == 0] = 0
    bad = np.zeros((n, t), dtype=bool)
    for k in rng.choice(n, size=10, replace=False):
        i = int(np.flatnonzero(present[k])[0])  # the first loaded chunk: always decode input
        host[k, i, int(rng.integers(0, L))] ^= 0x21
        bad[k, i] = True
    buf.copy_(torch.from_numpy(host))
    verified, status = ce.resilver_batch(rs, batch, present.tobytes(), dig.data_ptr())
    torch.cuda.synchronize()
    v = np.frombuffer(verified, np.uint8).reshape(n, t).astype(bool)
    assert np.array_equal(v, present.astype(bool) & ~bad)
    got = buf.cpu().numpy()
    for k in range(n):
        if v[k].sum() < d:
            assert status[k] == ce.TOO_FEW_SHARDS_PRESENT
            continue
        assert status[k] == ce.OK
        assert np.array_equal(got[k], ref[k]), k


@pytest.mark.slow
def test_chunk_longer_than_4gib_encode_and_reconstruct():
    """ChunkSize allows chunks up to 2^32 bytes (cluster/sized_int.rs:139): byte offsets past
    32 bits.  RS(2,1) with L = 4 GiB + 4 KiB + 48 (not a multiple of the kernels' 16 KiB column
    range): encode, then lose data chunk 0 and rebuild it.  GF coding is column-local, so
    windows at the start, across the 2^32 boundary and at the end are checked against the
    oracle run on just those windows."""
    d, p = 2, 1
    L = (1 << 32) + 4096 + 48
    need = (d + p) * L
    free, _ = torch.cuda.mem_get_info()
    if free < need + (2 << 30):
        pytest.skip("not enough device memory")
    rs = ce.ReedSolomon(d, p)
    buf = torch.empty((1, d + p, L), dtype=torch.uint8, device=DEV)
    batch = ce.PartBatch.from_tensor(buf, L)
    ce.fill_synthetic(batch, d, 77)
    ce.encode_batch(rs, batch)
    torch.cuda.synchronize()
    windows = [(0, 8192), ((1 << 32) - 4096, 8192), (L - 8192, 8192)]

    def check_windows():
        for off, w in windows:
            host = buf[0, :, off:off + w].cpu().numpy()
            st, par = oracle.encode_sep(d, p, [host[j] for j in range(d)])
            assert st == 0
            assert np.array_equal(host[d], par[0]), off

    check_windows()
    want = [buf[0, 0, off:off + w].cpu().numpy().copy() for off, w in windows]
    buf[0, 0].zero_()
    present = np.array([0, 1, 1], np.uint8)
    ce.reconstruct_batch(rs, batch, present.tobytes(), True)
    torch.cuda.synchronize()
    for (off, w), v in zip(windows, want):
        assert np.array_equal(buf[0, 0, off:off + w].cpu().numpy(), v), off
    check_windows()
    del buf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("max_blocks", ["9", "64", "1000"])
def test_apply_launch_split_over_part_ranges(knob_env, max_blocks):
    """A dispatch holds at most 2^32-1 work-items, so encode / reconstruct batches of more
    blocks than that are split into launches over whole part ranges (rs_kernels.hip).  The test
    knob CEC_APPLY_MAX_BLOCKS lowers the limit to force splits at test size (here 9 tiles per
    part for the bit-sliced encoder's 8 KiB tiles, 5 for the v_perm reconstruct's 16 KiB; the
    smallest value is one part per launch for both): every byte must match the unsplit launch."""
    d, p, L, n = 10, 4, 4 * 16384 + 100, 37
    t = d + p
    rs = ce.ReedSolomon(d, p)
    buf = torch.zeros((n, t, L + 12), dtype=torch.uint8, device=DEV)
    batch = ce.PartBatch.from_tensor(buf, L)
    ce.fill_synthetic(batch, d, 4242)
    ce.encode_batch(rs, batch)
    torch.cuda.synchronize()
    ref = buf.clone()
    rng = np.random.default_rng(int(max_blocks))
    present = np.ones((n, t), np.uint8)
    for k in range(n):
        present[k, rng.choice(t, int(rng.integers(1, p + 1)), replace=False)] = 0
    knob_env.set("CEC_APPLY_MAX_BLOCKS", max_blocks)
    buf[:, d:] = 0
    ce.encode_batch(rs, batch)  # encode split
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    buf[~torch.from_numpy(present).to(DEV).bool()] = 0
    ce.reconstruct_batch(rs, batch, present.tobytes(), False)  # reconstruct split (var kernel)
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)


@pytest.mark.parametrize("d,p", [(3, 2), (10, 4), (20, 8)])
@pytest.mark.parametrize("L", [16, 8192, 8192 + 16, 3 * 8192 - 16, 16384 + 5, 65536 + 4096])
def test_bitsliced_encode_matches_vperm_and_oracle(knob_env, d, p, L):
    """The compiled shapes' encode takes the bit-sliced kernel (rs_encode_bs_kernel: full
    8 KiB column steps bit-sliced, the ragged rest through the v_perm byte path).  Every byte
    must equal the v_perm kernel's (CEC_APPLY_BS=0) and, on sampled parts, the oracle's."""
    t, n = d + p, 9
    cstride = (L + 15) // 16 * 16 + 32  # 16-byte aligned, not a power of two
    rs = ce.ReedSolomon(d, p)
    buf = torch.zeros((n, t, cstride), dtype=torch.uint8, device=DEV)
    batch = ce.PartBatch.from_tensor(buf, L)
    ce.fill_synthetic(batch, d, 9000 + L)
    ce.encode_batch(rs, batch)
    torch.cuda.synchronize()
    got = buf.clone()
    knob_env.set("CEC_APPLY_BS", "0")
    buf[:, d:] = 0
    ce.encode_batch(rs, batch)
    torch.cuda.synchronize()
    assert torch.equal(got, buf)
    assert not got[:, d:, L:].any()  # nothing written past the chunk
    host = got.cpu().numpy()
    for k in (0, n - 1):
        st, par = oracle.encode_sep(d, p, [host[k, j, :L] for j in range(d)])
        assert st == 0
        for i in range(p):
            assert np.array_equal(host[k, d + i, :L], par[i]), (k, i)
