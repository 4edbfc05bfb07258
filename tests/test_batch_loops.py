"""The batched write / read / verify / resilver loops (chunky_ec.batchwriter / batchreader /
batchcheck: the executed twins of the Rust crate's batch::BatchWriter / BatchReader / FileReader /
BatchChecker) on the CPU, with the scheduler and the page-locked buffers replaced by stand-ins that
keep the C-ABI's contract (cec_multi_encode_hash / _read / _verify / _resilver: asynchronous jobs,
per-part status, CEC_PRESENT_VERIFIED chunks used but not hashed) and compute with the oracle and
hashlib.  Checks the loop logic itself -- part cut (writer.rs:172-194), file order across windows,
the short last part, read retries that walk a chunk's locations before drawing another chunk
(file_part.rs:92-107), every location hashed by verify / resilver (:236-243, :277-289), failures,
and that no job is left in flight -- in the CPU suite; tests/test_gpu_batch*.py run the same loops
on the real engine."""
import hashlib
import io
import itertools

import numpy as np
import pytest

import oracle
from chunky_ec import OK, PRESENT_VERIFIED, TOO_FEW_SHARDS_PRESENT, EncodedPart, Error, Sha256Hash
from _stores import Locations
import chunky_ec.batchcheck as bc
import chunky_ec.batchreader as br
import chunky_ec.batchwriter as bw

D, P, L = 3, 2, 512
T = D + P
CAP = D * L


class FakeHostBuffer:
    def __init__(self, nbytes, device=-1):
        self.array = np.zeros(nbytes, np.uint8)
        self.ptr = self.array.ctypes.data
        self.nbytes = nbytes

    def view(self, *shape):
        return self.array.reshape(*shape)


def _arr(b):
    return b.array if isinstance(b, FakeHostBuffer) else b


class FakeMulti:
    """cec_multi's job contract, computed with the oracle; `live` = jobs not yet waited for.
    Carry (cec_multi_read_carry): a part reported TooFewShardsPresent with a verified chunk gets
    an id whose entry keeps its verified chunks; a retry given the id takes its
    PRESENT_VERIFIED chunks from the entry (the caller's buffer is not read for them) and is
    refused unless the id is held and was kept for that part.  `uploaded` counts the chunks a
    read read from the caller's buffer."""
    ids = itertools.count(1)
    WRITE, READ = 1, 2

    def __init__(self, codec, chunk_len, parts_per_batch, depth, devices, kinds=3):
        self.d, self.p = codec.data_shard_count(), codec.parity_shard_count()
        self.t, self.L = self.d + self.p, chunk_len
        self.live = set()
        self.kinds = kinds
        self.pool = {}  # carry id -> (kept mask, expected digests, chunk bytes)
        self.next_carry = itertools.count(0)
        self.uploaded = self.carried = 0
        self.events = []  # ("read", n, retry?) per read job, in submission order

    def carry_release(self, cid):
        del self.pool[int(cid)]

    def query(self, job):
        assert job in self.live  # a job not submitted or already waited for is refused
        return True  # the oracle computed it at submission

    def _job(self):
        j = next(self.ids)
        self.live.add(j)
        return j

    def encode_hash(self, data, n, parity, digests):
        d, p, t, L = self.d, self.p, self.t, self.L
        src = _arr(data)[:n * d * L].reshape(n, d, L)
        par = _arr(parity)[:n * p * L].reshape(n, p, L)
        dig = _arr(digests)[:n * t * 32].reshape(n, t, 32)
        for k in range(n):
            st, pp = oracle.encode_sep(d, p, list(src[k]))
            assert st == 0
            par[k] = np.stack(pp)
            for i, c in enumerate(list(src[k]) + list(pp)):
                dig[k, i] = np.frombuffer(hashlib.sha256(c.tobytes()).digest(), np.uint8)
        return self._job()

    def read(self, chunks, present, expected, n, data, verified, status, rebuilt_only=False,
             carry_in=None, carry_out=None, ahead=False):
        assert self.kinds & self.READ
        assert ahead == (carry_in is not None)  # the readers' retry rounds, and only they
        self.events.append(("read", n, carry_in is not None))
        d, t, L = self.d, self.t, self.L
        ch = _arr(chunks)[:n * t * L].reshape(n, t, L).copy()
        pres = np.asarray(present).reshape(-1, t)
        exp = np.asarray(expected).reshape(-1, t, 32)
        out = _arr(data)[:n * d * L].reshape(n, d, L)
        ver = np.asarray(verified).reshape(-1, t)
        st = np.asarray(status)
        # REBUILT_ONLY: only rebuilt data chunks land in `data`; ptrs[k*d + j] says where each
        # data chunk is (a loaded one where the caller's buffer holds it)
        ptrs = [None] * (n * d) if rebuilt_only else None
        base_ch, base_out = _arr(chunks).ctypes.data, _arr(data).ctypes.data
        for k in range(n):
            cid = -1 if carry_in is None else int(carry_in[k])
            if cid >= 0:  # the entry replaces the part's verified chunks
                mask, want, kept = self.pool.pop(cid)
                assert np.array_equal(want, exp[k]), "carry id of another part"
                assert all(mask[i] for i in range(t) if pres[k, i] == PRESENT_VERIFIED)
                for i in range(t):
                    if pres[k, i] == PRESENT_VERIFIED:
                        ch[k, i] = kept[i]
                        self.carried += 1
            self.uploaded += sum(1 for i in range(t)
                                 if pres[k, i] and not (cid >= 0 and pres[k, i] == PRESENT_VERIFIED))
            if carry_out is not None:
                carry_out[k] = -1
            for i in range(t):
                if pres[k, i] == PRESENT_VERIFIED:
                    ver[k, i] = 1
                elif pres[k, i]:
                    ver[k, i] = hashlib.sha256(ch[k, i].tobytes()).digest() == exp[k, i].tobytes()
                else:
                    ver[k, i] = 0
            if ver[k].sum() < d:
                st[k] = TOO_FEW_SHARDS_PRESENT
                if carry_out is not None and ver[k].any():
                    c = next(self.next_carry)
                    self.pool[c] = (ver[k].copy(), exp[k].copy(), ch[k].copy())
                    carry_out[k] = c
                continue
            code, rec = oracle.reconstruct(d, self.p, [ch[k, i].copy() if ver[k, i] else None
                                                       for i in range(t)], data_only=True)
            assert code == 0
            redone = any(pres[k, i] and not ver[k, i] for i in range(t))
            for j in range(d):
                in_place = (rebuilt_only and not redone and pres[k, j]
                            and not (cid >= 0 and pres[k, j] == PRESENT_VERIFIED))
                if in_place:
                    ptrs[k * d + j] = base_ch + (k * t + j) * L
                else:
                    out[k, j] = rec[j]
                    if rebuilt_only:
                        ptrs[k * d + j] = base_out + (k * d + j) * L
            st[k] = OK
        return self._job(), ptrs

    def _verify_flags(self, ch, pres, exp, ver, n):
        for k in range(n):
            for i in range(self.t):
                if pres[k, i] == PRESENT_VERIFIED:
                    ver[k, i] = 1
                elif pres[k, i]:
                    ver[k, i] = hashlib.sha256(ch[k, i].tobytes()).digest() == exp[k, i].tobytes()
                else:
                    ver[k, i] = 0

    def verify(self, chunks, present, expected, n, verified):
        t, L = self.t, self.L
        self._verify_flags(_arr(chunks)[:n * t * L].reshape(n, t, L),
                           np.asarray(present).reshape(-1, t), np.asarray(expected).reshape(-1, t, 32),
                           np.asarray(verified).reshape(-1, t), n)
        return self._job()

    def resilver(self, chunks, present, expected, n, rebuilt, verified, status):
        d, t, L = self.d, self.t, self.L
        ch = _arr(chunks)[:n * t * L].reshape(n, t, L)
        out = _arr(rebuilt)[:n * t * L].reshape(n, t, L)
        ver = np.asarray(verified).reshape(-1, t)
        st = np.asarray(status)
        self._verify_flags(ch, np.asarray(present).reshape(-1, t),
                           np.asarray(expected).reshape(-1, t, 32), ver, n)
        for k in range(n):
            if ver[k].sum() < d:
                st[k] = TOO_FEW_SHARDS_PRESENT
                continue
            code, rec = oracle.reconstruct(d, self.p, [ch[k, i].copy() if ver[k, i] else None
                                                       for i in range(t)], data_only=False)
            assert code == 0
            for i in range(t):
                if not ver[k, i]:
                    out[k, i] = rec[i]
            st[k] = OK
        return self._job(), None

    def wait(self, job):
        self.live.remove(job)


def _oracle_part_encode(codec, buf, length):
    cs, par, dig = oracle.part_encode(codec.data_shard_count(), codec.parity_shard_count(),
                                      np.frombuffer(bytes(buf), np.uint8), length)
    return EncodedPart(cs, [x.tobytes() for x in par], [Sha256Hash(x.tobytes()) for x in dig])


class _HashlibSha:
    """Sha256Hash.from_bufs on the CPU (read_part's per-call hashing)."""

    def __init__(self, digest):
        self.digest = digest

    @classmethod
    def from_bufs(cls, bufs):
        return [cls(hashlib.sha256(bytes(b)).digest()) for b in bufs]


class _OracleCodec:
    """ReedSolomon's per-call reconstruct_data (read_part) on the CPU."""

    def __init__(self, d, p):
        self.d, self.p = d, p

    def data_shard_count(self):
        return self.d

    def total_shard_count(self):
        return self.d + self.p

    def parity_shard_count(self):
        return self.p

    def reconstruct_data(self, shards):
        code, rec = oracle.reconstruct(self.d, self.p, [None if s is None else
                                                        np.frombuffer(bytes(s), np.uint8)
                                                        for s in shards], data_only=True)
        assert code == 0
        for i in range(self.d):
            if shards[i] is None:
                shards[i] = bytearray(rec[i].tobytes())


@pytest.fixture
def fakes(monkeypatch):
    for mod in (bw, br, bc):
        monkeypatch.setattr(mod, "Multi", FakeMulti)
        monkeypatch.setattr(mod, "HostBuffer", FakeHostBuffer)
    monkeypatch.setattr(bw, "part_encode", _oracle_part_encode)
    monkeypatch.setattr(br, "Sha256Hash", _HashlibSha)
    for mod in (bw, br, bc):
        monkeypatch.setattr(mod, "ReedSolomon", _OracleCodec)


def _expected_part(file_bytes, k):
    part = file_bytes[k * CAP:(k + 1) * CAP]
    n = len(part)
    Lk = (n + D - 1) // D
    buf = np.zeros(D * Lk, np.uint8)
    buf[:n] = np.frombuffer(part, np.uint8)
    data = [buf[j * Lk:(j + 1) * Lk] for j in range(D)]
    st, par = oracle.encode_sep(D, P, data)
    chunks = [x.tobytes() for x in data] + [x.tobytes() for x in par]
    return n, Lk, chunks, [hashlib.sha256(c).digest() for c in chunks]


class Trickle(io.RawIOBase):
    def __init__(self, data, step):
        self.src, self.pos, self.step = data, 0, step

    def readable(self):
        return True

    def readinto(self, b):
        n = min(len(b), self.step, len(self.src) - self.pos)
        b[:n] = self.src[self.pos:self.pos + n]
        self.pos += n
        return n


def test_batch_writer_loop(fakes):
    w = bw.BatchWriter(D, P, L, 2, 2, [0])
    W = w.window
    rng = np.random.default_rng(1)
    for n in (0, 1, CAP - 1, CAP, CAP + 1, W * CAP, W * CAP + 5, 3 * W * CAP - 1, 3 * W * CAP):
        fb = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        parts = []
        total = w.write(Trickle(fb, 100) if n % 2 else io.BytesIO(fb),
                        lambda p: parts.append((p.index, p.length, p.chunksize, p.digests,
                                                [bytes(c) for c in p.chunks])))
        assert total == n and w.multi.live == set()
        assert [p[0] for p in parts] == list(range((n + CAP - 1) // CAP))
        for idx, length, cs, dig, chunks in parts:
            want = _expected_part(fb, idx)
            assert (length, cs, chunks, dig) == (want[0], want[1], want[2], want[3]), (n, idx)


def test_batch_writer_sink_error_drains(fakes):
    w = bw.BatchWriter(D, P, L, 2, 2, [0])
    fb = np.random.default_rng(2).integers(0, 256, 4 * w.window * CAP, dtype=np.uint8).tobytes()

    def sink(p):
        if p.index == w.window + 1:
            raise KeyError("full")
    with pytest.raises(KeyError):
        w.write(io.BytesIO(fb), sink)
    assert w.multi.live == set()  # the window in flight was waited for


def _store(n, seed, L=L):
    rng = np.random.default_rng(seed)
    chunks = np.zeros((n, T, L), np.uint8)
    dig = np.zeros((n, T, 32), np.uint8)
    for k in range(n):
        data = rng.integers(0, 256, size=(D, L), dtype=np.uint8)
        st, par = oracle.encode_sep(D, P, list(data))
        chunks[k, :D], chunks[k, D:] = data, np.stack(par)
        for i in range(T):
            dig[k, i] = np.frombuffer(hashlib.sha256(chunks[k, i].tobytes()).digest(), np.uint8)
    return chunks, dig


def test_batch_reader_loop(fakes):
    n = 17
    chunks, dig = _store(n, 3)
    st = Locations(chunks)
    # part 6: chunk 0 missing; part 9: chunk 1 damaged; part 12: chunks 0 and 2 damaged (two
    # replacements, taken from the parity chunks); part 16 (the last, in a short window): chunk 2
    st.set(6, 0, "gone")
    for k, i in ((9, 1), (12, 0), (12, 2), (16, 2)):
        st.set(k, i, "bad")
    r = br.BatchReader(D, P, L, 2, 2, [0, 0])
    got = []
    r.read(n, st.fetch, lambda k: dig[k], lambda k, data: got.append((k, b"".join(map(bytes, data)))))
    assert [k for k, _ in got] == list(range(n))
    assert all(b == chunks[k, :D].tobytes() for k, b in got)
    assert r.retries == 3 and r.multi.live == set()
    # every retried part's verified chunks stayed with the scheduler (carry): the retries sent
    # only their new chunks (9: 1, 12: 2, 16: 1) and no carry entry is left
    assert r.carried_parts == 3 and r.multi.carried == 2 + 1 + 2 and r.multi.pool == {}
    assert r.multi.uploaded == n * D + 1 + 2 + 1
    # part 12: its damaged chunks have no further location (fetch from 1 finds none), then the
    # two parity chunks are drawn
    assert [c for c in st.calls if c[0] == 12] == [(12, i, 0) for i in range(D)] + \
        [(12, 0, 1), (12, 2, 1), (12, 3, 0), (12, 4, 0)]
    # part 6: chunk 0 has no readable location: never asked again
    assert [c for c in st.calls if c[0] == 6] == [(6, 0, 0), (6, 1, 0), (6, 2, 0), (6, 3, 0)]


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_batch_reader_walks_a_chunks_locations_first(fakes, devices):
    """p + 1 chunks per part listed [bad, good] (what resilver leaves when it appends a rebuilt
    copy, file_part.rs:346): too few first copies verify, but each chunk's second location does.
    The reference reads it (file_part.rs:100-107); so must the batched loop, re-fetching the same
    chunk's next location before it draws another chunk."""
    n = 9
    chunks, dig = _store(n, 8)
    st = Locations(chunks)
    for k in range(n):
        for i in range(P + 1):
            st.set(k, (k + i) % T, "bad", "good")
    st.set(4, 3, "gone", "short", "bad", "good")  # unreadable, wrong size, bad, then good
    r = br.BatchReader(D, P, L, 2, 2, devices)
    got = []
    r.read(n, st.fetch, lambda k: dig[k], lambda k, data: got.append((k, b"".join(map(bytes, data)))))
    assert [k for k, _ in got] == list(range(n))
    assert all(b == chunks[k, :D].tobytes() for k, b in got)
    # part 0 (chunks 0, 1, 2 listed [bad, good]): one retry, on the same three chunks' location 1
    assert [c for c in st.calls if c[0] == 0] == [(0, 0, 0), (0, 1, 0), (0, 2, 0),
                                                  (0, 0, 1), (0, 1, 1), (0, 2, 1)]
    assert r.multi.live == set()


def test_batch_reader_out_of_chunks(fakes):
    chunks, dig = _store(9, 4)
    st = Locations(chunks)
    for i in (0, 3):
        st.set(5, i, "bad")
    st.set(5, 4, "bad", "gone", "bad")  # 2 good chunks < d = 3, whatever the locations hold
    r = br.BatchReader(D, P, L, 2, 2, [0])
    got = []
    with pytest.raises(Exception) as e:
        r.read(9, st.fetch, lambda k: dig[k], lambda k, data: got.append(k))
    assert getattr(e.value, "code", None) == TOO_FEW_SHARDS_PRESENT
    assert got == [0, 1, 2, 3] and r.multi.live == set()
    assert r.multi.pool == {}  # the failed part's carry id went back


def _file(nbytes, seed, d=D, p=P, chunk=L):
    """A file cut as writer.rs:172-194 / file_part.rs:150-158 does: (shapes, chunks per part,
    digests per part, the file bytes)."""
    fb = np.random.default_rng(seed).integers(0, 256, nbytes, dtype=np.uint8).tobytes()
    cap = d * chunk
    shapes, parts, digs = [], [], []
    for off in range(0, nbytes, cap):
        piece = fb[off:off + cap]
        Lk = -(-len(piece) // d)
        buf = np.zeros(d * Lk, np.uint8)
        buf[:len(piece)] = np.frombuffer(piece, np.uint8)
        data = [buf[j * Lk:(j + 1) * Lk] for j in range(d)]
        st, par = oracle.encode_sep(d, p, data)
        cs = [c.tobytes() for c in data] + [c.tobytes() for c in par]
        shapes.append((d, p, Lk))
        parts.append(cs)
        digs.append(np.array([np.frombuffer(hashlib.sha256(c).digest(), np.uint8) for c in cs]))
    return shapes, parts, digs, fb


@pytest.mark.parametrize("extra", [0, 1, 700])
def test_file_reader_short_last_part(fakes, extra):
    """The short last part has chunk size ceil(len / d) (file_part.rs:152): FileReader reads it
    through read_part instead of the full-size BatchReader (which would drop its chunks as the
    wrong size and fail the read), with its own damaged chunk walked to its second location."""
    shapes, parts, digs, fb = _file(7 * D * L + extra, 11)
    copies = {(k, i): [c] for k, cs in enumerate(parts) for i, c in enumerate(cs)}
    last = len(parts) - 1
    if extra:
        good = parts[last][1]
        copies[(last, 1)] = [bytes([good[0] ^ 1]) + good[1:], good]  # [bad, good]
        copies[(last, 0)] = [None]
    calls = []

    def fetch(k, i, start):
        calls.append((k, i, start))
        locs = copies[(k, i)]
        for j in range(start, len(locs)):
            if locs[j] is not None:
                return j, locs[j]
        return None
    reader = br.FileReader(2, 2, [0])
    out = bytearray()
    seen = []
    reader.read(shapes, fetch, lambda k: digs[k],
                lambda k, data: (seen.append(k), out.extend(b"".join(map(bytes, data)))))
    assert seen == list(range(len(parts)))
    assert bytes(out[:len(fb)]) == fb  # FileReference::length truncates the padding
    assert list(reader.readers) == [(D, P, L)]
    # a second file of the same shape reuses the kept reader (its pinned windows)
    keep = reader.readers[(D, P, L)]
    reader.read(shapes, fetch, lambda k: digs[k], lambda k, data: None)
    assert reader.readers[(D, P, L)] is keep


def test_checker_verify_hashes_every_location(fakes):
    n = 7
    chunks, dig = _store(n, 12)
    st = Locations(chunks)
    st.set(1, 0, "bad", "good")
    st.set(2, 4, "gone", "good", "bad")
    st.set(3, 2, "short")
    st.set(5, 1, "gone")
    st.set(6, 3)  # no locations at all
    c = bc.BatchChecker(D, P, L, 2, 2, [0])
    got = {}
    c.verify(n, st.read_all, lambda k: dig[k], lambda k, part: got.__setitem__(k, part))
    assert sorted(got) == list(range(n)) and c.multi.live == set()
    assert got[0].locations == [[True]] * T
    assert got[1].locations[0] == [False, True] and got[1].healthy_chunks() == T
    assert got[2].locations[4] == [None, True, False]
    assert got[3].locations[2] == [False] and got[3].healthy_chunks() == T - 1
    assert got[5].locations[1] == [None] and got[5].unavailable_locations() == 1
    assert got[6].locations[3] == [] and got[6].healthy_chunks() == T - 1
    assert sum(p.invalid_locations() for p in got.values()) == 3


def test_checker_resilver_rebuilds_only_chunks_without_a_valid_copy(fakes):
    n = 9
    chunks, dig = _store(n, 13)
    st = Locations(chunks)
    st.set(0, 0, "gone")                  # one location, unreadable: rebuilt
    st.set(0, D, "bad")                   # one location, bad: rebuilt
    st.set(2, 1, "bad", "good")           # a valid second copy: healthy, not rebuilt
    st.set(2, 4, "bad", "gone")           # no valid copy among two: rebuilt
    st.set(4, 2, "short", "bad", "good")
    for i in range(P + 1):                # too few chunks: write_error, the others go on
        st.set(7, i, "bad")
    c = bc.BatchChecker(D, P, L, 2, 2, [0])
    got = {}
    c.resilver(n, st.read_all, lambda k: dig[k],
               lambda k, part: got.__setitem__(k, (part, {i: bytes(b) for i, b in
                                                          part.rebuilt.items()})))
    assert sorted(got) == list(range(n)) and c.multi.live == set()
    assert sorted(got[0][1]) == [0, D] and got[0][0].locations[D] == [False]
    assert sorted(got[2][1]) == [4] and got[2][0].locations[1] == [False, True]
    assert got[4][1] == {} and got[4][0].locations[2] == [False, False, True]
    for k, (part, rebuilt) in got.items():
        for i, b in rebuilt.items():
            assert b == chunks[k, i].tobytes(), (k, i)
    assert got[7][0].error == TOO_FEW_SHARDS_PRESENT and got[7][1] == {}
    assert all(got[k][0].error is None for k in got if k != 7)
    assert c.extra_passes == 2  # windows holding parts 2 and 4 (multi-location chunks)


def test_batch_reader_retry_overlaps_the_next_window(fakes):
    """A window's failed parts go out again (their first retry round) as soon as its job is
    done (Multi.query; the fake's jobs are done at once): before the next window is loaded, so
    the retry runs beside that loading instead of stalling the loop; the parts still reach the
    sink in file order."""
    n = 4 * 3
    chunks, dig = _store(n, 12)
    st = Locations(chunks)
    st.set(1, 0, "bad")  # window 0 (parts 0-3): part 1 retries
    r = br.BatchReader(D, P, L, 4, 2, [0])
    order = []
    r.read(n, st.fetch, lambda k: dig[k], lambda k, data: order.append(("emit", k)))
    assert [k for _, k in order] == list(range(n))
    ev = r.multi.events
    # window 0, its retry, then windows 1 and 2
    assert ev[:4] == [("read", 4, False), ("read", 1, True), ("read", 4, False),
                      ("read", 4, False)], ev
    assert r.retries == 1 and r.carried_parts == 1 and r.multi.pool == {}


def test_batch_reader_checks_windows_as_soon_as_their_jobs_are_done(fakes):
    """At depth 4 the reader keeps 5 windows and checks each as soon as its job is done: window
    0's retry goes out before window 1 is loaded, four steps before window 0 is emitted (a retry
    round costs one SHA-256 chain whatever its size)."""
    n = 4 * 7
    chunks, dig = _store(n, 14)
    st = Locations(chunks)
    st.set(1, 0, "bad")   # window 0: part 1 retries
    st.set(13, 2, "bad")  # window 3: part 13 retries
    r = br.BatchReader(D, P, L, 4, 4, [0])
    assert r.R == 5
    order = []
    r.read(n, st.fetch, lambda k: dig[k], lambda k, data: order.append(k))
    assert order == list(range(n))
    ev = r.multi.events
    assert ev == [("read", 4, False), ("read", 1, True)] + [("read", 4, False)] * 3 \
        + [("read", 1, True)] + [("read", 4, False)] * 3, ev
    assert r.retries == 2 and r.multi.pool == {}


def test_batch_reader_retries_of_the_last_windows_go_out_before_any_is_emitted(fakes):
    """Each window's retry goes out as soon as its job is done, so those of the last windows are
    all in flight before the first of them is emitted (not one per emitted window)."""
    n = 4 * 5
    chunks, dig = _store(n, 15)
    st = Locations(chunks)
    for k in (9, 13, 17):  # windows 2, 3 and 4
        st.set(k, 0, "bad")
    r = br.BatchReader(D, P, L, 4, 4, [0])
    order = []
    r.read(n, st.fetch, lambda k: dig[k], lambda k, data: order.append(k))
    assert order == list(range(n))
    # each of windows 2-4 is followed by its retry; all five are submitted before window 0 is
    # emitted (5 window buffers)
    assert r.multi.events == [("read", 4, False)] * 3 + [("read", 1, True), ("read", 4, False)] * 2 \
        + [("read", 1, True)], r.multi.events


class _LazyFakeMulti(FakeMulti):
    """FakeMulti whose jobs report done only after a seeded number of queries (wait always
    completes them): the polling read loop sees windows and retry rounds finish out of order."""
    rng = np.random.default_rng(0)

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.polls = {}

    def query(self, job):
        assert job in self.live
        left = self.polls.setdefault(job, int(self.rng.integers(0, 6)))
        self.polls[job] = left - 1
        return left <= 0


@pytest.mark.parametrize("seed", range(12))
def test_batch_reader_polling_loop_fuzz(fakes, monkeypatch, seed):
    """Random location mixes (good, bad, unreadable, short copies; several per chunk), random
    window size and depth, jobs finishing after random numbers of polls: every part comes out in
    file order as stored, a part with fewer than d good chunks fails the read with
    TooFewShardsPresent (the parts before it out), and afterwards no job is left unwaited and no
    carry id held."""
    monkeypatch.setattr(br, "Multi", _LazyFakeMulti)
    _LazyFakeMulti.rng = np.random.default_rng(1000 + seed)
    rng = np.random.default_rng(seed)
    n = int(rng.integers(5, 40))
    chunks, dig = _store(n, 50 + seed)
    st = Locations(chunks)
    good = {}
    for k in range(n):
        good[k] = 0
        for i in range(T):
            u = rng.random()
            spec = (["good"] if u < 0.7 else ["bad", "good"] if u < 0.8 else
                    ["gone", "short", "good"] if u < 0.86 else ["bad", "bad"] if u < 0.93 else
                    ["gone"])
            st.set(k, i, *spec)
            good[k] += "good" in spec
    ppb, depth = int(rng.integers(1, 5)), int(rng.integers(1, 6))
    r = br.BatchReader(D, P, L, ppb, depth, [0], carry=bool(rng.integers(0, 2)))
    got = []
    short = [k for k in range(n) if good[k] < D]
    try:
        r.read(n, st.fetch, lambda k: dig[k],
               lambda k, data: got.append((k, b"".join(bytes(x) for x in data))))
        err = None
    except Error as e:
        err = e.code
    assert [k for k, _ in got] == list(range(len(got)))
    for k, b in got:
        assert b == chunks[k, :D].tobytes(), (seed, k)
    if short:
        assert err == TOO_FEW_SHARDS_PRESENT and len(got) <= short[0], (seed, short, len(got))
    else:
        assert err is None and len(got) == n, seed
    assert r.multi.live == set() and r.multi.pool == {}, seed


@pytest.mark.parametrize("seed", range(10))
def test_batch_checker_fuzz(fakes, monkeypatch, seed):
    """BatchChecker verify and resilver over random location mixes (one or several copies per
    chunk: good, bad, short, unreadable; chunks with no location), random window size, depth and
    shard list, against a model of file_part.rs:228-390: every location's result (valid /
    invalid / unavailable), and resilver rebuilding exactly the chunks with no valid copy, with the
    stored bytes, or TooFewShardsPresent for a part with fewer than d of them; no job left."""
    monkeypatch.setattr(bc, "Multi", _LazyFakeMulti)
    _LazyFakeMulti.rng = np.random.default_rng(2000 + seed)
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(3, 30))
    chunks, dig = _store(n, 70 + seed)
    st = Locations(chunks)
    want = {}
    kinds = ["good", "bad", "short", "gone"]
    res = {"good": True, "bad": False, "short": False, "gone": None}
    for k in range(n):
        for i in range(T):
            if rng.random() < 0.6:
                spec = ["good"]
            else:
                spec = [kinds[int(x)] for x in rng.choice(4, int(rng.integers(0, 4)), p=[.35, .3, .1, .25])]
            st.set(k, i, *spec)
            want[(k, i)] = [res[s] for s in spec]
    ppb, depth = int(rng.integers(1, 5)), int(rng.integers(1, 6))
    devices = [0] if rng.integers(0, 2) else [0, 0]
    c = bc.BatchChecker(D, P, L, ppb, depth, devices)
    got = {}
    c.verify(n, st.read_all, lambda k: dig[k], lambda k, part: got.__setitem__(k, part))
    assert sorted(got) == list(range(n)) and c.multi.live == set()
    for k in range(n):
        assert got[k].locations == [want[(k, i)] for i in range(T)], (seed, k)
    fixed = {}
    c.resilver(n, st.read_all, lambda k: dig[k],
               lambda k, part: fixed.__setitem__(k, (part, {i: bytes(b) for i, b in
                                                            part.rebuilt.items()})))
    assert sorted(fixed) == list(range(n)) and c.multi.live == set()
    for k in range(n):
        part, rebuilt = fixed[k]
        assert part.locations == [want[(k, i)] for i in range(T)], (seed, k)
        lost = [i for i in range(T) if True not in want[(k, i)]]
        if T - len(lost) < D:
            assert part.error == TOO_FEW_SHARDS_PRESENT and rebuilt == {}, (seed, k)
        else:
            assert part.error is None and sorted(rebuilt) == lost, (seed, k)
            assert all(rebuilt[i] == chunks[k, i].tobytes() for i in lost), (seed, k)


@pytest.mark.parametrize("seed", range(8))
def test_batch_reader_sink_error_leaves_nothing(fakes, monkeypatch, seed):
    """A sink that raises part way through a damaged read (jobs finishing out of order): the
    error reaches the caller, every job is waited for, every carry id given back, and the reader
    then reads the same store whole."""
    monkeypatch.setattr(br, "Multi", _LazyFakeMulti)
    _LazyFakeMulti.rng = np.random.default_rng(3000 + seed)
    rng = np.random.default_rng(200 + seed)
    n = int(rng.integers(8, 30))
    chunks, dig = _store(n, 90 + seed)
    st = Locations(chunks)
    for k in range(n):
        for i in range(T):
            if rng.random() < 0.15:
                st.set(k, i, "bad", "good")
    r = br.BatchReader(D, P, L, int(rng.integers(1, 4)), int(rng.integers(1, 5)), [0])
    stop = int(rng.integers(0, n))

    def sink(k, data):
        if k == stop:
            raise KeyError("sink closed")
    with pytest.raises(KeyError):
        r.read(n, st.fetch, lambda k: dig[k], sink)
    assert r.multi.live == set() and r.multi.pool == {}, seed
    got = []
    r.read(n, st.fetch, lambda k: dig[k],
           lambda k, data: got.append((k, b"".join(bytes(x) for x in data))))
    assert [k for k, _ in got] == list(range(n))
    assert all(b == chunks[k, :D].tobytes() for k, b in got)
    assert r.multi.live == set() and r.multi.pool == {}, seed


@pytest.mark.parametrize("seed", range(6))
def test_file_reader_range_reads(fakes, seed):
    """FileReader.read_range (FileReadBuilder::seek / take, reader.rs:22-173; the gateway's Range
    reads): the range's bytes of a file with a short last part and a [bad, good] chunk, read only
    from the parts that hold the range; range_len as reader.rs:129-138."""
    rng = np.random.default_rng(seed)
    shapes, parts, digs, fb = _file(9 * D * L + int(rng.integers(1, D * L)), 30 + seed)
    copies = {(k, i): [c] for k, cs in enumerate(parts) for i, c in enumerate(cs)}
    good = parts[3][0]
    copies[(3, 0)] = [bytes([good[0] ^ 4]) + good[1:], good]
    calls = []

    def fetch(k, i, start):
        calls.append(k)
        locs = copies[(k, i)]
        for j in range(start, len(locs)):
            if locs[j] is not None:
                return j, locs[j]
        return None
    reader = br.FileReader(2, 2, [0])
    starts = np.cumsum([0] + [d * Lk for d, _, Lk in shapes])
    n = len(fb)
    for _ in range(8):
        seek = int(starts[rng.integers(0, len(starts))]) if rng.random() < 0.3 else int(rng.integers(0, n + 3))
        take = 0 if rng.random() < 0.3 else int(rng.integers(0, n + 3))
        want = fb[seek:] if take == 0 else fb[seek:seek + take]
        assert br.range_len(n, seek, take) == len(want)
        calls.clear()
        out, seen = bytearray(), []
        got = reader.read_range(shapes, n, seek, take, fetch, lambda k: digs[k],
                                lambda k, pieces: (seen.append(k),
                                                   [out.extend(bytes(x)) for x in pieces]))
        assert bytes(out) == want and got == len(want), (seek, take)
        assert seen == sorted(set(seen))
        # only the parts holding the range were read
        lo = int(np.searchsorted(starts, seek, side="right")) - 1
        hi = int(np.searchsorted(starts, seek + len(want), side="left"))
        assert set(calls) <= set(range(lo, max(hi, lo + 1))), (seek, take, sorted(set(calls)))
        assert not want or seen[0] == lo


def test_file_reader_range_read_fails_only_inside_the_range(fakes):
    """A part without d good chunks fails a range read that reaches into it (TooFewShardsPresent,
    file_part.rs:92-107) and not one that ends before it or starts after it: the parts outside
    the range are not read."""
    shapes, parts, digs, fb = _file(8 * D * L, 61)
    copies = {(k, i): [c] for k, cs in enumerate(parts) for i, c in enumerate(cs)}
    for i in range(P + 1):  # part 4: P + 1 chunks lost
        copies[(4, i)] = [None]

    def fetch(k, i, start):
        locs = copies[(k, i)]
        for j in range(start, len(locs)):
            if locs[j] is not None:
                return j, locs[j]
        return None
    reader = br.FileReader(2, 2, [0])
    part, n = D * L, len(fb)
    for seek, take, fails in ((0, 4 * part, False), (5 * part, 0, False), (4 * part - 1, 1, False),
                              (4 * part - 1, 2, True), (3 * part, 2 * part, True), (0, 0, True)):
        out = bytearray()
        try:
            reader.read_range(shapes, n, seek, take, fetch, lambda k: digs[k],
                              lambda k, pieces: [out.extend(bytes(x)) for x in pieces])
            err = None
        except Error as e:
            err = e.code
        if fails:
            assert err == TOO_FEW_SHARDS_PRESENT, (seek, take)
        else:
            want = fb[seek:] if take == 0 else fb[seek:seek + take]
            assert err is None and bytes(out) == want, (seek, take)
