"""The batched write / read loops (chunky_ec.batchwriter / batchreader: the executed twins of the
Rust crate's batch::BatchWriter / BatchReader) on the CPU, with the scheduler and the page-locked
buffers replaced by stand-ins that keep the C-ABI's contract (cec_multi_encode_hash / _read:
asynchronous jobs, per-part status, CEC_PRESENT_VERIFIED chunks used but not hashed) and compute
with the oracle and hashlib.  Checks the loop logic itself -- part cut (writer.rs:172-194), file
order across windows, the short last part, read retries (file_part.rs:92-107), failures, and
that no job is left in flight -- in the CPU suite; tests/test_gpu_batchwriter.py and
tests/test_gpu_batchreader.py run the same loops on the real engine."""
import hashlib
import io
import itertools

import numpy as np
import pytest

import oracle
from chunky_ec import OK, PRESENT_VERIFIED, TOO_FEW_SHARDS_PRESENT, EncodedPart, Sha256Hash
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
    """cec_multi's job contract, computed with the oracle; `live` = jobs not yet waited for."""
    ids = itertools.count(1)

    def __init__(self, codec, chunk_len, parts_per_batch, depth, devices):
        self.d, self.p = codec.data_shard_count(), codec.parity_shard_count()
        self.t, self.L = self.d + self.p, chunk_len
        self.live = set()

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

    def read(self, chunks, present, expected, n, data, verified, status, rebuilt_only=False):
        d, t, L = self.d, self.t, self.L
        ch = _arr(chunks)[:n * t * L].reshape(n, t, L)
        pres = np.asarray(present).reshape(-1, t)
        exp = np.asarray(expected).reshape(-1, t, 32)
        out = _arr(data)[:n * d * L].reshape(n, d, L)
        ver = np.asarray(verified).reshape(-1, t)
        st = np.asarray(status)
        for k in range(n):
            for i in range(t):
                if pres[k, i] == PRESENT_VERIFIED:
                    ver[k, i] = 1
                elif pres[k, i]:
                    ver[k, i] = hashlib.sha256(ch[k, i].tobytes()).digest() == exp[k, i].tobytes()
                else:
                    ver[k, i] = 0
            if ver[k].sum() < d:
                st[k] = TOO_FEW_SHARDS_PRESENT
                continue
            code, rec = oracle.reconstruct(d, self.p, [ch[k, i].copy() if ver[k, i] else None
                                                       for i in range(t)], data_only=True)
            assert code == 0
            out[k] = np.stack(rec[:d])
            st[k] = OK
        return self._job(), None

    def wait(self, job):
        self.live.remove(job)


def _oracle_part_encode(codec, buf, length):
    cs, par, dig = oracle.part_encode(codec.data_shard_count(), codec.parity_shard_count(),
                                      np.frombuffer(bytes(buf), np.uint8), length)
    return EncodedPart(cs, [x.tobytes() for x in par], [Sha256Hash(x.tobytes()) for x in dig])


@pytest.fixture
def fakes(monkeypatch):
    for mod in (bw, br):
        monkeypatch.setattr(mod, "Multi", FakeMulti)
        monkeypatch.setattr(mod, "HostBuffer", FakeHostBuffer)
    monkeypatch.setattr(bw, "part_encode", _oracle_part_encode)


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


def _store(n, seed):
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


def _fetcher(chunks, missing=(), damaged=()):
    calls = []

    def fetch(part, i):
        calls.append((part, i))
        if (part, i) in missing:
            return None
        b = chunks[part, i].copy()
        if (part, i) in damaged:
            b[3] ^= 1
        return b.tobytes()
    return fetch, calls


def test_batch_reader_loop(fakes):
    n = 17
    chunks, dig = _store(n, 3)
    # part 6: chunk 0 missing; part 9: chunk 1 damaged; part 12: chunks 0 and 2 damaged (two
    # replacements, taken from the parity chunks); part 16 (the last, in a short window): chunk 2
    fetch, calls = _fetcher(chunks, missing={(6, 0)}, damaged={(9, 1), (12, 0), (12, 2), (16, 2)})
    r = br.BatchReader(D, P, L, 2, 2, [0, 0])
    got = []
    r.read(n, fetch, lambda k: dig[k], lambda k, data: got.append((k, b"".join(map(bytes, data)))))
    assert [k for k, _ in got] == list(range(n))
    assert all(b == chunks[k, :D].tobytes() for k, b in got)
    assert r.retries == 3 and r.multi.live == set()
    assert [c for c in calls if c[0] == 12] == [(12, i) for i in range(T)]
    assert [c for c in calls if c[0] == 6] == [(6, 0), (6, 1), (6, 2), (6, 3)]


def test_batch_reader_out_of_chunks(fakes):
    chunks, dig = _store(9, 4)
    fetch, _ = _fetcher(chunks, damaged={(5, 0), (5, 3), (5, 4)})  # 2 good < d = 3
    r = br.BatchReader(D, P, L, 2, 2, [0])
    got = []
    with pytest.raises(Exception) as e:
        r.read(9, fetch, lambda k: dig[k], lambda k, data: got.append(k))
    assert getattr(e.value, "code", None) == TOO_FEW_SHARDS_PRESENT
    assert got == [0, 1, 2, 3] and r.multi.live == set()
