"""Seeded randomized parity checks over the whole shape space the reference allows per part
(d in 1..24, p in 1..10, any chunk length, any layout), through the device-batch C-ABI, against
the oracle and hashlib.  Each case draws its code, chunk length, part count, chunk stride (16-byte
aligned or not) and erasure / corruption pattern from a fixed seed, so a failure names a
reproducible case.
"""
import hashlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import chunky_ec as ce  # noqa: E402

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda", 0)
N_CASES = 40


def _case(seed):
    rng = np.random.default_rng(seed)
    d = int(rng.integers(1, 25))
    p = int(rng.integers(1, 11))
    L = int(rng.choice([int(rng.integers(1, 300)), int(rng.integers(300, 9000)),
                        64 * int(rng.integers(1, 100))]))
    n = int(rng.integers(1, 40))
    aligned = bool(rng.integers(0, 2))
    stride = (L + 15) // 16 * 16 if aligned else L + int(rng.integers(0, 5))
    return rng, d, p, L, n, stride


def _batch(d, p, L, n, stride, seed):
    t = d + p
    buf = torch.zeros((n, t, stride), dtype=torch.uint8, device=DEV)
    batch = ce.PartBatch.from_tensor(buf, L)
    ce.fill_synthetic(batch, d, seed)
    return buf, batch


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_encode_hash_reconstruct(seed):
    rng, d, p, L, n, stride = _case(1000 + seed)
    t = d + p
    rs = ce.ReedSolomon(d, p)
    buf, batch = _batch(d, p, L, n, stride, seed)
    dig = torch.zeros((n, t, 32), dtype=torch.uint8, device=DEV)
    ce.encode_hash_batch(rs, batch, dig.data_ptr())
    torch.cuda.synchronize()
    host, hd = buf.cpu().numpy(), dig.cpu().numpy()
    for k in range(n):
        st, par = oracle.encode_sep(d, p, [host[k, j, :L] for j in range(d)])
        assert st == 0
        for i in range(p):
            assert np.array_equal(host[k, d + i, :L], par[i]), (seed, k, i)
        for j in range(t):
            assert hd[k, j].tobytes() == hashlib.sha256(host[k, j, :L].tobytes()).digest(), \
                (seed, k, j)
    # random erasures (0..p per part), data_only drawn per case
    data_only = bool(rng.integers(0, 2))
    present = np.ones((n, t), np.uint8)
    for k in range(n):
        present[k, rng.choice(t, int(rng.integers(0, p + 1)), replace=False)] = 0
    ref = host.copy()
    mask = torch.from_numpy(present).to(DEV).bool()
    buf[~mask] = 0
    ce.reconstruct_batch(rs, batch, present.tobytes(), data_only)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    for k in range(n):
        shards = [ref[k, i, :L].tobytes() if present[k, i] else None for i in range(t)]
        st, out = oracle.reconstruct(d, p, shards, data_only=data_only)
        assert st == 0
        for i in range(t):
            if out[i] is not None:
                assert got[k, i, :L].tobytes() == out[i].tobytes(), (seed, k, i)
            else:
                assert not got[k, i, :L].any(), (seed, k, i)  # left as None: untouched


@pytest.mark.parametrize("seed", range(N_CASES))
def test_fuzz_read_batch(seed):
    """read_with_context batched: a random loaded set per part (d-1 .. d+p chunks) with random
    corruption; verified flags, statuses and rebuilt data as the oracle's rules give them."""
    rng, d, p, L, n, stride = _case(5000 + seed)
    t = d + p
    rs = ce.ReedSolomon(d, p)
    buf, batch = _batch(d, p, L, n, stride, 7000 + seed)
    dig = torch.zeros((n, t, 32), dtype=torch.uint8, device=DEV)
    ce.encode_hash_batch(rs, batch, dig.data_ptr())
    torch.cuda.synchronize()
    ref = buf.cpu().numpy().copy()
    present = np.zeros((n, t), np.uint8)
    for k in range(n):
        size = int(rng.integers(max(d - 1, 1), t + 1))
        present[k, rng.choice(t, size, replace=False)] = 1
    host = ref.copy()
    host[present == 0] = 0
    bad = np.zeros((n, t), bool)
    for k in range(n):
        if rng.random() < 0.3:
            i = int(rng.choice(np.flatnonzero(present[k])))
            host[k, i, int(rng.integers(0, L))] ^= 1 << int(rng.integers(0, 8))
            bad[k, i] = True
    buf.copy_(torch.from_numpy(host))
    verified, status = ce.read_batch(rs, batch, present.tobytes(), dig.data_ptr())
    torch.cuda.synchronize()
    v = np.frombuffer(verified, np.uint8).reshape(n, t).astype(bool)
    assert np.array_equal(v, present.astype(bool) & ~bad), seed
    got = buf.cpu().numpy()
    for k in range(n):
        if v[k].sum() < d:
            assert status[k] == ce.TOO_FEW_SHARDS_PRESENT, (seed, k)
            continue
        assert status[k] == ce.OK, (seed, k)
        for j in range(d):
            assert got[k, j, :L].tobytes() == ref[k, j, :L].tobytes(), (seed, k, j)


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_read_stream_carry(seed):
    """The read-repair loop (file_part.rs:92-107) on the pipeline with and without
    CEC_READ_CARRY, same seeded store and damage: the same parts decode, to the stored bytes,
    the same parts are undecodable, and with carry the retries take their verified chunks from
    the device (slot bytes for them are garbage) instead of fetching them again."""
    from chunky_ec.readstream import ReadRepairStream
    rng = np.random.default_rng(9000 + seed)
    d = int(rng.integers(1, 13))
    p = int(rng.integers(1, 7))
    t = d + p
    L = int(rng.choice([int(rng.integers(1, 300)), 64 * int(rng.integers(1, 40))]))
    n = int(rng.integers(5, 60))
    P = int(rng.integers(1, 12))
    depth = int(rng.integers(1, 5))
    corrupt = float(rng.choice([0.05, 0.15, 0.3]))
    stored = rng.integers(0, 256, (n, t, L), dtype=np.uint8)
    dig = np.zeros((n, t, 32), np.uint8)
    for k in range(n):
        st, par = oracle.encode_sep(d, p, [stored[k, j] for j in range(d)])
        assert st == 0
        stored[k, d:] = np.stack(par)
        for i in range(t):
            dig[k, i] = np.frombuffer(hashlib.sha256(stored[k, i].tobytes()).digest(), np.uint8)
    damage = rng.random((n, t)) < corrupt  # per (part, chunk): a chunk is fetched fresh once
    runs = {}
    for carry in (False, True):
        rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, P, depth, ce.ReadPipeline.REBUILT_ONLY |
                             (ce.ReadPipeline.CARRY if carry else 0))
        def fetch(slot_chunks, rows):
            for k, part, flags in rows:
                slot_chunks[k] = 0xA5
                for j in np.flatnonzero(flags):
                    slot_chunks[k, j] = stored[part, j]
                    if flags[j] == 1 and damage[part, j]:
                        slot_chunks[k, j, (part * 31 + j) % L] ^= 0x24

        got = {}

        def on_part(slot, nb, k, part, attempts, rp=rp, got=got):
            got[part] = rp.part_bytes(slot, nb, k)

        s = ReadRepairStream(rp, fetch, lambda ids: dig[ids], seed=seed, on_part=on_part).run(0, n)
        for part, out in got.items():
            assert out == stored[part, :d].tobytes(), (seed, carry, part)
        assert set(got) | set(s.undecodable) == set(range(n))
        runs[carry] = (set(got), s)
        del rp
    assert runs[False][0] == runs[True][0], seed
    s0, s1 = runs[False][1], runs[True][1]
    assert s1.retried_parts == s0.retried_parts and s1.rejected_chunks == s0.rejected_chunks
    # the same batches: every chunk the carry run did not fetch came from the pool
    assert s1.chunks_loaded + s1.carried_chunks == s0.chunks_loaded and s0.carried_chunks == 0
