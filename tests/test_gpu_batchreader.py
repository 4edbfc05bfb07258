"""chunky_ec.batchreader.BatchReader (the executed twin of the Rust crate's batch::BatchReader and
the C++ FileReference::read_run / retry) on the GPU: parts come out in file order with their
stored data chunks, with chunks missing from storage, chunks served damaged (rejected by the
SHA-256 verification and replaced, file_part.rs:92-107), over one and two scheduler shards; a part
that runs out of good chunks fails the read with TooFewShardsPresent."""
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

import chunky_ec as ce  # noqa: E402
import oracle  # noqa: E402
from chunky_ec.batchreader import BatchReader  # noqa: E402

D, P, L = 4, 2, 4096
T = D + P


def _store(n, seed):
    rng = np.random.default_rng(seed)
    chunks = np.zeros((n, T, L), np.uint8)
    dig = np.zeros((n, T, 32), np.uint8)
    for k in range(n):
        data = rng.integers(0, 256, size=(D, L), dtype=np.uint8)
        st, par = oracle.encode_sep(D, P, list(data))
        assert st == 0
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
            b[17] ^= 0x40
        return b.tobytes()
    return fetch, calls


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_batch_reader_in_order_with_missing_and_damaged_chunks(devices):
    n = 23
    chunks, dig = _store(n, 5)
    missing = {(3, 0), (4, 0), (4, 1), (11, 2)}
    damaged = {(5, 1), (8, 0), (8, 3), (16, 2), (22, 0)}
    fetch, calls = _fetcher(chunks, missing, damaged)
    r = BatchReader(D, P, L, 3, 2, devices)
    got = []
    r.read(n, fetch, lambda k: dig[k], lambda k, data: got.append((k, b"".join(bytes(x)
                                                                                  for x in data))))
    assert [k for k, _ in got] == list(range(n))
    for k, b in got:
        assert b == chunks[k, :D].tobytes(), k
    # every part with a damaged chunk was resubmitted once; an intact part loaded exactly its d
    # data chunks; part 8 (chunks 0 and 3 damaged) took the two parity chunks on its retry
    assert r.retries == 4
    assert [c for c in calls if c[0] == 0] == [(0, i) for i in range(D)]
    assert [c for c in calls if c[0] == 8] == [(8, i) for i in range(T)]


def test_batch_reader_part_out_of_chunks_fails_the_read():
    n = 7
    chunks, dig = _store(n, 6)
    damaged = {(4, 0), (4, 2), (4, 5)}  # 3 of 6 bad: 3 good < d = 4
    fetch, _ = _fetcher(chunks, damaged=damaged)
    r = BatchReader(D, P, L, 2, 2, [0])
    got = []
    with pytest.raises(ce.Error) as e:
        r.read(n, fetch, lambda k: dig[k], lambda k, data: got.append(k))
    assert e.value.code == ce.TOO_FEW_SHARDS_PRESENT
    assert got == [0, 1, 2, 3]  # the windows before the failing one were handed out, in order
    # the reader is reusable after the failure (no job left in flight on its windows)
    fetch, _ = _fetcher(chunks)
    got = []
    r.read(n, fetch, lambda k: dig[k], lambda k, data: got.append(k))
    assert got == list(range(n))
