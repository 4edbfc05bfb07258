"""chunky_ec.readstream on the CPU: the batched read_with_context retry loop (file_part.rs:86-122)
driven against a stand-in pipeline that hashes with hashlib and decodes with the oracle, with the
same per-part contract as cec_read_pipeline (status TooFewShardsPresent when fewer than d loaded
chunks verify; CEC_PRESENT_VERIFIED chunks used but not hashed).  The GPU form of the same loop
is tests/test_gpu_parity.py::test_read_repair_stream_* and bench.py's c5r / read_repair."""
import hashlib

import numpy as np
import pytest

import oracle
from chunky_ec import OK, PRESENT_VERIFIED, TOO_FEW_SHARDS_PRESENT
from chunky_ec.readstream import ReadRepairStream


class FakeReadPipeline:
    """cec_read_pipeline's contract on the CPU (oracle decode, hashlib verify)."""

    def __init__(self, d, p, L, parts, depth):
        self.d, self.p, self.t, self.L, self.parts, self.depth = d, p, d + p, L, parts, depth
        self.slots = [dict(chunks=np.zeros((parts, d + p, L), np.uint8),
                           present=np.zeros((parts, d + p), np.uint8),
                           expected=np.zeros((parts, d + p, 32), np.uint8), n=0, res=None)
                      for _ in range(depth)]
        self.next = 0
        self.submitted = []  # (slot, present rows) per batch

    def acquire(self):
        i = self.next
        self.next = (self.next + 1) % self.depth
        s = self.slots[i]
        s["res"] = None
        return i, s["chunks"], s["present"], s["expected"]

    def submit(self, slot, n):
        s = self.slots[slot]
        s["n"] = n
        self.submitted.append((slot, s["present"][:n].copy()))
        d, t = self.d, self.t
        out = np.zeros((n, d, self.L), np.uint8)
        ver = np.zeros((n, t), np.uint8)
        st = np.zeros(n, np.int32)
        for k in range(n):
            pr = s["present"][k]
            for i in range(t):
                if pr[i] == PRESENT_VERIFIED:
                    ver[k, i] = 1
                elif pr[i]:
                    ver[k, i] = hashlib.sha256(s["chunks"][k, i].tobytes()).digest() == \
                        s["expected"][k, i].tobytes()
            if ver[k].sum() < d:
                st[k] = TOO_FEW_SHARDS_PRESENT
                continue
            shards = [s["chunks"][k, i].copy() if ver[k, i] else None for i in range(t)]
            code, rec = oracle.reconstruct(d, self.p, shards, data_only=True)
            assert code == 0
            out[k] = np.stack([rec[i] for i in range(d)])
        s["res"] = (out, ver, st)

    def wait(self, slot):
        return self.slots[slot]["res"]

    def drain(self):
        pass


def _store(n_parts, d, p, L, seed):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, size=(n_parts, d, L), dtype=np.uint8)
    chunks = np.zeros((n_parts, d + p, L), np.uint8)
    dig = np.zeros((n_parts, d + p, 32), np.uint8)
    for k in range(n_parts):
        st, par = oracle.encode_sep(d, p, list(data[k]))
        assert st == 0
        chunks[k, :d] = data[k]
        chunks[k, d:] = np.stack(par)
        for i in range(d + p):
            dig[k, i] = np.frombuffer(hashlib.sha256(chunks[k, i].tobytes()).digest(), np.uint8)
    return chunks, dig


@pytest.mark.parametrize("corrupt", [0.0, 0.1, 0.35])
def test_read_repair_stream_rebuilds_every_part(corrupt):
    d, p, L, P, depth, n = 4, 3, 96, 5, 3, 37
    chunks, dig = _store(n, d, p, L, 7)
    rng = np.random.default_rng(11)
    bad_loads = []

    def fetch(slot_chunks, rows):
        for k, part, flags in rows:
            for j in np.flatnonzero(flags):
                slot_chunks[k, j] = chunks[part, j]
                if flags[j] == 1 and rng.random() < corrupt:  # a fresh read comes back damaged
                    slot_chunks[k, j, rng.integers(L)] ^= 0x5A
                    bad_loads.append((part, j))

    fp = FakeReadPipeline(d, p, L, P, depth)
    got = {}

    attempts = {}

    def on_part(slot, nb, k, part, tries):
        got[part] = fp.slots[slot]["res"][0][k].copy()
        attempts[part] = tries

    s = ReadRepairStream(fp, fetch, lambda ids: dig[ids], seed=3, on_part=on_part).run(0, n)
    # every part either decoded to its data or ran out of chunks to try
    assert s.parts + s.undecodable_parts == n
    assert set(got) | set(s.undecodable) == set(range(n))
    for part, out in got.items():
        assert np.array_equal(out, chunks[part, :d]), part
    # every corrupted first load was caught (a re-sent verified chunk is never hashed again)
    assert s.rejected_chunks == len(bad_loads)
    assert sum(attempts.values()) - len(attempts) <= s.retried_parts
    if corrupt == 0.0:
        assert s.retried_parts == 0 and s.retry_batches == 0 and s.mixed_batches == 0
        assert s.undecodable_parts == 0 and s.batches == (n + P - 1) // P
    else:
        # retries ride in the next batch ahead of new parts: every batch but the trailing
        # retry-only ones is full
        assert s.retried_parts > 0 and s.mixed_batches > 0
        sizes = [len(rows) for _, rows in fp.submitted]
        assert all(k == P for k in sizes[:s.batches - s.retry_batches - 1])
    # the load rule: first loads are d distinct chunks; a retry re-sends the verified chunks as
    # PRESENT_VERIFIED and adds exactly (d - verified) chunks never tried before
    for _, rows in fp.submitted:
        for row in rows:
            assert np.count_nonzero(row) == d
            assert set(np.unique(row)) <= {0, 1, PRESENT_VERIFIED}


def test_read_repair_stream_undecodable_when_chunks_run_out():
    """Every load of part 2 is corrupted: it is retried until fewer than d untried chunks remain,
    then counted undecodable (the reference's read fails TooFewShardsPresent); the other parts
    still decode."""
    d, p, L, P, depth, n = 3, 2, 64, 4, 2, 9
    chunks, dig = _store(n, d, p, L, 1)

    def fetch(slot_chunks, rows):
        for k, part, flags in rows:
            for j in np.flatnonzero(flags):
                slot_chunks[k, j] = chunks[part, j]
                if part == 2:
                    slot_chunks[k, j, 0] ^= 1

    fp = FakeReadPipeline(d, p, L, P, depth)
    s = ReadRepairStream(fp, fetch, lambda ids: dig[ids], seed=0).run(0, n)
    assert s.undecodable == [2] and s.undecodable_parts == 1 and s.parts == n - 1
    # part 2: 3 loaded, all rejected -> 2 untried left < d = 3 -> undecodable, no retry batch
    assert s.rejected_chunks == 3


def test_read_repair_stream_status_other_than_too_few_raises():
    d, p, L = 2, 1, 16
    chunks, dig = _store(3, d, p, L, 2)

    class Broken(FakeReadPipeline):
        def submit(self, slot, n):
            super().submit(slot, n)
            self.slots[slot]["res"][2][:] = 9  # IncorrectShardSize

    fp = Broken(d, p, L, 2, 2)

    def fetch(c, rows):
        for k, part, flags in rows:
            idx = np.flatnonzero(flags)
            c[k, idx] = chunks[part, idx]
    import chunky_ec
    with pytest.raises(chunky_ec.Error):
        ReadRepairStream(fp, fetch, lambda ids: dig[ids]).run(0, 3)
    assert OK == 0


class FakeCarryPipeline(FakeReadPipeline):
    """cec_read_pipeline with CEC_READ_CARRY: each batch keeps the verified chunks of every part
    it reports TooFewShardsPresent in a pool of 2 x parts entries (-1 when none is free; the real
    pipeline's stash kernels do this on the device); submit_carried takes a carried part's
    CEC_PRESENT_VERIFIED chunks from the pool, whatever the slot holds there."""
    carry = True

    def __init__(self, *a, cap=None):
        super().__init__(*a)
        self.cap = 2 * self.parts if cap is None else cap
        self.pool = {}       # id -> [t][L] chunks
        self.free = list(range(self.cap))
        self.ids = {}        # slot -> ids of its last batch
        self.released = []

    def submit(self, slot, n):
        self._carried = None
        super().submit(slot, n)
        self._keep(slot, n)

    def submit_carried(self, slot, n, ids):
        s = self.slots[slot]
        for k in range(n):
            if ids[k] >= 0:
                assert ids[k] in self.pool, "carry id not held"
                vpos = s["present"][k] == PRESENT_VERIFIED
                s["chunks"][k, vpos] = 0xEE  # whatever the caller left there is not used...
                s["chunks"][k, vpos] = self.pool.pop(int(ids[k]))[vpos]  # ...the pool's bytes are
                self.free.append(int(ids[k]))
        super().submit(slot, n)
        self._keep(slot, n)

    def _keep(self, slot, n):
        s = self.slots[slot]
        _, ver, st = s["res"]
        ids = np.full(n, -1, np.int32)
        for k in range(n):
            if st[k] == TOO_FEW_SHARDS_PRESENT and ver[k].any() and self.free:
                e = self.free.pop()
                self.pool[e] = np.where(ver[k][:, None] != 0, s["chunks"][k], 0)
                ids[k] = e
        self.ids[slot] = ids

    def carry_ids(self, slot, n):
        return self.ids[slot][:n]

    def carry_release(self, e):
        self.released.append(e)
        self.pool.pop(e)
        self.free.append(e)


@pytest.mark.parametrize("cap", [None, 1])
def test_read_repair_stream_carries_verified_chunks(cap):
    """CARRY: a retried part's verified chunks come from the device pool, so the reader fetches
    only the new chunks; the parts decode exactly as without carry, and an undecodable part's
    entry is released.  cap=1: the pool fills, and parts without an entry are re-sent as before."""
    d, p, L, P, depth, n = 4, 3, 96, 5, 3, 41
    chunks, dig = _store(n, d, p, L, 9)
    rng = np.random.default_rng(5)
    fetched = []

    def fetch(slot_chunks, rows):
        for k, part, flags in rows:
            fetched.append((part, flags.copy()))
            for j in np.flatnonzero(flags):
                slot_chunks[k, j] = chunks[part, j]
                if flags[j] == 1 and (rng.random() < 0.2 or part == 7):  # part 7: never decodes
                    slot_chunks[k, j, rng.integers(L)] ^= 0x5A

    fp = FakeCarryPipeline(d, p, L, P, depth, cap=cap)
    got = {}
    s = ReadRepairStream(fp, fetch, lambda ids: dig[ids], seed=4,
                         on_part=lambda slot, nb, k, part, tries: got.__setitem__(
                             part, fp.slots[slot]["res"][0][k].copy())).run(0, n)
    assert s.parts + s.undecodable_parts == n and 7 in s.undecodable
    for part, out in got.items():
        assert np.array_equal(out, chunks[part, :d]), part
    assert s.carried_chunks > 0
    if cap is None:
        # nothing verified is fetched twice: every fetch of a part is of chunks not fetched before
        seen = {}
        for part, flags in fetched:
            new = set(np.flatnonzero(flags))
            assert not new & seen.get(part, set()), part
            assert PRESENT_VERIFIED not in flags
            seen.setdefault(part, set()).update(new)
    assert not fp.pool or fp.released  # entries are used or released, never left behind
    assert sorted(fp.free) == list(range(fp.cap))


def test_read_repair_stream_last_retries_go_out_together():
    """After the last new part, the retries of the batches still in flight wait for all of them
    and go out as one batch (each retry round costs one SHA-256 chain whatever its size): every
    retry-only batch is submitted with nothing else in flight, and the parts still decode."""
    d, p, L, P, depth, n = 4, 3, 64, 6, 4, 60
    chunks, dig = _store(n, d, p, L, 21)
    rng = np.random.default_rng(8)

    class Counting(FakeReadPipeline):
        def __init__(self, *a):
            super().__init__(*a)
            self.out = 0
            self.log = []  # (rows, batches in flight when submitted)

        def submit(self, slot, n):
            self.log.append((self.slots[slot]["present"][:n].copy(), self.out))
            self.out += 1
            super().submit(slot, n)

        def wait(self, slot):
            self.out -= 1
            return super().wait(slot)

    def fetch(slot_chunks, rows):
        for k, part, flags in rows:
            for j in np.flatnonzero(flags):
                slot_chunks[k, j] = chunks[part, j]
                if flags[j] == 1 and rng.random() < 0.15:
                    slot_chunks[k, j, rng.integers(L)] ^= 0x5A

    fp = Counting(d, p, L, P, depth)
    got = {}
    s = ReadRepairStream(fp, fetch, lambda ids: dig[ids], seed=2,
                         on_part=lambda slot, nb, k, part, tries: got.__setitem__(
                             part, fp.slots[slot]["res"][0][k].copy())).run(0, n)
    assert s.parts + s.undecodable_parts == n
    assert all(np.array_equal(out, chunks[part, :d]) for part, out in got.items())
    last_new = max(i for i, (rows, _) in enumerate(fp.log)
                   if any(not (r == PRESENT_VERIFIED).any() for r in rows))
    tail = fp.log[last_new + 1:]
    assert tail and s.retry_batches == len(tail)
    assert all(busy == 0 for _, busy in tail)
    # the retries of the last `depth` batches went out together: fewer tail batches than that
    assert len(tail) < depth
