"""chunky_ec.readstream over the real cec_read_pipeline (HIP verify + decode): the batched
read_with_context retry loop (file_part.rs:86-122) against oracle-encoded stored chunks with
damaged fetches -- every decoded part equals the stored data, every damaged chunk is rejected,
parts that run out of chunks are reported, and the same loop through bench.py's
timed_read_repair (the c5r / end_to_end.read_repair path)."""
import hashlib
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

import chunky_ec as ce  # noqa: E402
import oracle  # noqa: E402
from chunky_ec.readstream import ReadRepairStream  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _store(n, d, p, L, seed):
    rng = np.random.default_rng(seed)
    chunks = np.zeros((n, d + p, L), np.uint8)
    dig = np.zeros((n, d + p, 32), np.uint8)
    for k in range(n):
        data = rng.integers(0, 256, size=(d, L), dtype=np.uint8)
        st, par = oracle.encode_sep(d, p, list(data))
        assert st == 0
        chunks[k, :d], chunks[k, d:] = data, np.stack(par)
        for i in range(d + p):
            dig[k, i] = np.frombuffer(hashlib.sha256(chunks[k, i].tobytes()).digest(), np.uint8)
    return chunks, dig


@pytest.mark.parametrize("carry", [False, True])
@pytest.mark.parametrize("d,p,L,corrupt", [(10, 4, 4096, 0.05), (3, 2, 1000, 0.2),
                                           (20, 8, 777, 0.03)])
def test_read_repair_stream_on_the_pipeline(d, p, L, corrupt, carry):
    """carry: CEC_READ_CARRY -- a retried part's verified chunks come from the device carry pool
    (the slot's bytes for them are overwritten with garbage here, so a path that uploaded them
    anyway, or read them back from the slot, would decode wrong), its data chunks among them
    come back like rebuilt ones; odd L (1000, 777) takes the pitched copies."""
    n, P, depth = 61, 8, 3
    chunks, dig = _store(n, d, p, L, d * 100 + p)
    codec = ce.ReedSolomon(d, p)
    flags_ = ce.ReadPipeline.REBUILT_ONLY | (ce.ReadPipeline.CARRY if carry else 0)
    rp = ce.ReadPipeline(codec, L, P, depth, flags_)
    rng = np.random.default_rng(5)
    damaged = [0]

    def fetch(slot_chunks, rows):
        for k, part, flags in rows:
            slot_chunks[k] = 0x3C  # nothing the reader did not fetch may be trusted
            for j in np.flatnonzero(flags):
                slot_chunks[k, j] = chunks[part, j]
                if flags[j] == 1 and rng.random() < corrupt:
                    slot_chunks[k, j, rng.integers(L)] ^= 0x81
                    damaged[0] += 1

    got = {}

    def on_part(slot, nb, k, part, attempts):
        got[part] = (rp.part_bytes(slot, nb, k), attempts)

    s = ReadRepairStream(rp, fetch, lambda ids: dig[ids], seed=1, on_part=on_part).run(0, n)
    assert s.parts + s.undecodable_parts == n
    assert s.rejected_chunks == damaged[0] > 0 and s.retried_parts > 0
    assert (s.carried_chunks > 0) == carry
    for part, (out, _) in got.items():
        assert out == chunks[part, :d].tobytes(), part
    assert any(a > 1 for _, a in got.values())
    assert set(got) | set(s.undecodable) == set(range(n))


@pytest.mark.parametrize("carry", [False, True])
def test_read_repair_stream_runs_out_of_chunks_on_the_pipeline(carry):
    d, p, L, n = 3, 2, 512, 10
    chunks, dig = _store(n, d, p, L, 4)
    rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, 4, 2, ce.ReadPipeline.REBUILT_ONLY |
                         (ce.ReadPipeline.CARRY if carry else 0))

    def fetch(slot_chunks, rows):
        for k, part, flags in rows:
            for j in np.flatnonzero(flags):
                slot_chunks[k, j] = chunks[part, j]
                # part 7: chunks 0-1 always served damaged (3 good of 5: it decodes after
                # retries); part 3: chunks 0-2 (2 good of 5 < d: undecodable)
                if flags[j] == 1 and ((part == 7 and j < 2) or (part == 3 and j < 3)):
                    slot_chunks[k, j, 0] ^= 1

    s = ReadRepairStream(rp, fetch, lambda ids: dig[ids], seed=0).run(0, n)
    assert s.undecodable == [3] and s.parts == n - 1


def test_carry_ids_contract():
    """CEC_READ_CARRY's API: ids only for parts reported TooFewShardsPresent with a verified chunk;
    an id is used once (a second use or a released id is refused before anything is queued)."""
    d, p, L = 3, 2, 256
    chunks, dig = _store(2, d, p, L, 8)
    rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, 2, 2, ce.ReadPipeline.REBUILT_ONLY |
                         ce.ReadPipeline.CARRY)
    slot, ch, pres, exp = rp.acquire()
    pres[:2] = 0
    pres[0, :3] = 1          # part 0: chunks 0-2, chunk 2 damaged -> TooFew, 2 verified kept
    pres[1, [0, 1, 3]] = 1   # part 1: decodes
    ch[:2] = chunks[:2]
    ch[0, 2, 5] ^= 1
    exp[:2] = dig[:2]
    rp.submit(slot, 2)
    _, ver, st = rp.wait(slot)
    assert list(st) == [ce.TOO_FEW_SHARDS_PRESENT, ce.OK]
    ids = rp.carry_ids(slot, 2)
    assert ids[0] >= 0 and ids[1] == -1
    # the retry: chunks 0-1 from the pool (slot bytes garbage), chunk 3 fetched
    slot, ch, pres, exp = rp.acquire()
    pres[:1] = 0
    pres[0, :2] = ce.PRESENT_VERIFIED
    pres[0, 3] = 1
    ch[0] = 0x77
    ch[0, 3] = chunks[0, 3]
    exp[:1] = dig[:1]
    rp.submit_carried(slot, 1, ids[:1])
    _, ver, st = rp.wait(slot)
    assert list(st) == [ce.OK] and list(ver[0]) == [1, 1, 0, 1, 0]
    assert rp.part_bytes(slot, 1, 0) == chunks[0, :d].tobytes()
    slot, ch, pres, exp = rp.acquire()
    with pytest.raises(ce.Error):  # used once
        rp.submit_carried(slot, 1, ids[:1])
    with pytest.raises(ce.Error):
        rp.carry_release(int(ids[0]))


def test_carry_from_a_packed_batch():
    """The stash runs in every batch of a CARRY pipeline, packed ones included: a part whose
    packed load fails verification gets a carry id, and its unpacked retry takes the verified
    chunks from the pool (the slot's copy of them is garbage)."""
    d, p, L = 4, 2, 2048
    chunks, dig = _store(3, d, p, L, 21)
    rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, 3, 2, ce.ReadPipeline.REBUILT_ONLY |
                         ce.ReadPipeline.CARRY)
    present = np.zeros((3, d + p), np.uint8)
    present[:, :d] = 1
    packed = np.concatenate([chunks[k, :d] for k in range(3)]).copy()
    packed[1 * d + 2, 9] ^= 0x10  # part 1, chunk 2 damaged
    slot, _, _, _ = rp.acquire()
    rp.submit_packed(slot, packed, present, dig.copy(), 3)
    _, ver, st = rp.wait(slot)
    assert list(st) == [ce.OK, ce.TOO_FEW_SHARDS_PRESENT, ce.OK]
    ids = rp.carry_ids(slot, 3)
    assert ids[0] == -1 and ids[1] >= 0 and ids[2] == -1
    for k in (0, 2):
        assert rp.part_bytes(slot, 3, k) == chunks[k, :d].tobytes()
    slot, ch, pres, exp = rp.acquire()
    pres[:1] = 0
    pres[0, [0, 1, 3]] = ce.PRESENT_VERIFIED
    pres[0, 4] = 1
    ch[0] = 0x6B
    ch[0, 4] = chunks[1, 4]
    exp[:1] = dig[1:2]
    rp.submit_carried(slot, 1, ids[1:2])
    _, ver, st = rp.wait(slot)
    assert list(st) == [ce.OK]
    assert rp.part_bytes(slot, 1, 0) == chunks[1, :d].tobytes()


def test_carry_reservation_runs_out():
    """A batch reserves max(8, parts/4) pool entries for its stash: with 40 parts
    all failing, the first 10 in part order get carry ids and the rest -1; the retry mixes
    carried parts (slot bytes of their verified chunks garbage) with parts that send their
    verified chunks again, and every part decodes to the stored bytes."""
    d, p, L, n = 4, 2, 1024, 40
    chunks, dig = _store(n, d, p, L, 12)
    rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, n, 2, ce.ReadPipeline.REBUILT_ONLY |
                         ce.ReadPipeline.CARRY)
    slot, ch, pres, exp = rp.acquire()
    pres[:] = 0
    pres[:, :d] = 1
    ch[:] = chunks
    ch[:, 1, 7] ^= 0x40       # chunk 1 of every part damaged: 3 verified of 4 -> TooFew
    ch[5, 2, 0] ^= 1          # part 5: chunks 1 and 2 damaged, 2 verified
    exp[:] = dig
    rp.submit(slot, n)
    _, ver, st = rp.wait(slot)
    assert all(s == ce.TOO_FEW_SHARDS_PRESENT for s in st)
    good = ver.astype(bool).copy()
    ids = rp.carry_ids(slot, n)
    assert list(ids[:10] >= 0) == [True] * 10 and list(ids[10:]) == [-1] * (n - 10)
    assert len(set(ids[:10].tolist())) == 10
    slot, ch, pres, exp = rp.acquire()
    pres[:] = np.where(good, ce.PRESENT_VERIFIED, 0)
    ch[:] = 0x5A
    for k in range(n):
        if ids[k] < 0:  # no entry: its verified chunks go up again from the slot
            for j in np.flatnonzero(good[k]):
                ch[k, j] = chunks[k, j]
        for j in [4, 5] if k == 5 else [4]:  # the parity chunk(s) still needed
            pres[k, j] = 1
            ch[k, j] = chunks[k, j]
    exp[:] = dig
    rp.submit_carried(slot, n, ids)
    _, ver, st = rp.wait(slot)
    assert list(st) == [ce.OK] * n
    for k in range(n):
        assert rp.part_bytes(slot, n, k) == chunks[k, :d].tobytes(), k


def test_bench_timed_read_repair_small():
    sys.path.insert(0, ROOT)
    import bench
    d, p, L, P, depth = 10, 4, 65536, 16, 3
    chunks, dig = _store(40, d, p, L, 9)
    copier = bench.HostCopier(4)
    try:
        el, stats, checks = bench.timed_read_repair(ce.ReedSolomon(d, p), chunks, dig, L, P, depth,
                                                    0, 200, 1, 0.05, copier, 3)
    finally:
        copier.close()
    assert el > 0 and stats["parts"] == 200 and stats["undecodable_parts"] == 0
    assert stats["rejected_chunks"] == stats["damaged_loads"] > 0
    assert checks and all(c["ok"] for c in checks)
    assert any(c["attempts"] > 1 for c in checks)
