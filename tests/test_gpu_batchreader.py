"""chunky_ec.batchreader (the executed twin of the Rust crate's batch::BatchReader / read_part /
FileReader and of the C++ FileReference::read_run / retry_start / retry_collect) on the GPU: parts come out in file
order with their stored data chunks, with chunks missing from storage, chunks served damaged
(rejected by the SHA-256 verification and replaced, file_part.rs:92-107), chunks listed with a bad
copy before a good one (the next location of the same chunk is read before another chunk is
drawn, file_part.rs:100-107), a short last part, over one and two scheduler shards; a part that
runs out of good copies fails the read with TooFewShardsPresent."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

import chunky_ec as ce  # noqa: E402
import oracle  # noqa: E402
from _stores import Locations, make_parts  # noqa: E402
from chunky_ec.batchreader import BatchReader, FileReader  # noqa: E402

D, P, L = 4, 2, 4096
T = D + P


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_batch_reader_in_order_with_missing_and_damaged_chunks(devices):
    n = 23
    chunks, dig = make_parts(n, D, P, L, 5)
    st = Locations(chunks)
    for k, i in ((3, 0), (4, 0), (4, 1), (11, 2)):
        st.set(k, i, "gone")
    for k, i in ((5, 1), (8, 0), (8, 3), (16, 2), (22, 0)):
        st.set(k, i, "bad")
    r = BatchReader(D, P, L, 3, 2, devices)
    got = []
    r.read(n, st.fetch, lambda k: dig[k],
           lambda k, data: got.append((k, b"".join(bytes(x) for x in data))))
    assert [k for k, _ in got] == list(range(n))
    for k, b in got:
        assert b == chunks[k, :D].tobytes(), k
    # every part with a damaged chunk was resubmitted once; an intact part loaded exactly its d
    # data chunks; part 8 (chunks 0 and 3 damaged, no second copy) took the two parity chunks on
    # its retry
    assert r.retries == 4
    assert [c for c in st.calls if c[0] == 0] == [(0, i, 0) for i in range(D)]
    assert [c for c in st.calls if c[0] == 8] == [(8, i, 0) for i in range(D)] + \
        [(8, 0, 1), (8, 3, 1), (8, 4, 0), (8, 5, 0)]


@pytest.mark.parametrize("d,p,L", [(3, 2, 65536), (10, 4, 16384)])
@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_batch_reader_reads_chunks_listed_bad_then_good(d, p, L, devices):
    """RS(3,2) and RS(10,4) stores where p + 1 chunks of every part are listed [bad, good] -- a
    store a resilver has touched (file_part.rs:346 appends the rebuilt copy's location): fewer
    than d first copies verify, so only a reader that walks each chunk's locations decodes it.
    Every part must come back bit-exact with the oracle's data."""
    n = 11
    chunks, dig = make_parts(n, d, p, L, 40 + d)
    st = Locations(chunks)
    t = d + p
    for k in range(n):
        for i in range(p + 1):
            st.set(k, (k + 3 * i) % t, "bad", "good")
    st.set(2, 0, "gone", "short", "bad", "good")
    r = BatchReader(d, p, L, 4, 2, devices)
    got = []
    r.read(n, st.fetch, lambda k: dig[k],
           lambda k, data: got.append((k, b"".join(bytes(x) for x in data))))
    assert [k for k, _ in got] == list(range(n))
    for k, b in got:
        assert b == chunks[k, :d].tobytes(), k
    for k in range(n):
        # the bad copies were followed by their chunk's next location
        bad = {(k + 3 * i) % t for i in range(p + 1)}
        loaded = [i for (kk, i, s) in st.calls if kk == k and s == 0]
        for i in bad & set(loaded):
            assert (k, i, 1) in st.calls or (k == 2 and i == 0), (k, i)


def test_batch_reader_part_out_of_chunks_fails_the_read():
    n = 7
    chunks, dig = make_parts(n, D, P, L, 6)
    st = Locations(chunks)
    st.set(4, 0, "bad", "bad")
    st.set(4, 2, "gone", "bad")
    st.set(4, 5, "bad")  # 3 of 6 chunks without a good copy: 3 good < d = 4
    r = BatchReader(D, P, L, 2, 2, [0])
    got = []
    with pytest.raises(ce.Error) as e:
        r.read(n, st.fetch, lambda k: dig[k], lambda k, data: got.append(k))
    assert e.value.code == ce.TOO_FEW_SHARDS_PRESENT
    assert got == [0, 1, 2, 3]  # the windows before the failing one were handed out, in order
    # the reader is reusable after the failure (no job left in flight on its windows)
    st = Locations(chunks)
    got = []
    r.read(n, st.fetch, lambda k: dig[k], lambda k, data: got.append(k))
    assert got == list(range(n))


def test_file_reader_with_short_last_part():
    """A file whose last part is short (chunk size ceil(len / d), file_part.rs:152): FileReader
    reads the full parts through a BatchReader and the last one through read_part (per-call
    engine calls), its first data chunk listed [bad, good]."""
    import hashlib
    d, p, chunk = 3, 2, 8192
    rng = np.random.default_rng(21)
    fb = rng.integers(0, 256, 9 * d * chunk + 1001, dtype=np.uint8).tobytes()
    shapes, copies, digs = [], {}, []
    for k, off in enumerate(range(0, len(fb), d * chunk)):
        piece = fb[off:off + d * chunk]
        Lk = -(-len(piece) // d)
        buf = np.zeros(d * Lk, np.uint8)
        buf[:len(piece)] = np.frombuffer(piece, np.uint8)
        data = [buf[j * Lk:(j + 1) * Lk] for j in range(d)]
        st, par = oracle.encode_sep(d, p, data)
        cs = [c.tobytes() for c in data] + [c.tobytes() for c in par]
        for i, c in enumerate(cs):
            copies[(k, i)] = [c]
        shapes.append((d, p, Lk))
        digs.append(np.array([np.frombuffer(hashlib.sha256(c).digest(), np.uint8) for c in cs]))
    last = len(shapes) - 1
    good = copies[(last, 0)][0]
    copies[(last, 0)] = [bytes([good[0] ^ 0x10]) + good[1:], good]

    def fetch(k, i, start):
        locs = copies[(k, i)]
        for j in range(start, len(locs)):
            if locs[j] is not None:
                return j, locs[j]
        return None
    out = bytearray()
    FileReader(4, 2, [0]).read(shapes, fetch, lambda k: digs[k],
                               lambda k, data: out.extend(b"".join(bytes(x) for x in data)))
    assert bytes(out[:len(fb)]) == fb


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_batch_readers_in_two_threads_with_random_damage(devices):
    """The polling read loop under load: two BatchReaders (depth 4: five windows each, every
    window polled, retry rounds as AHEAD jobs on the scheduler's priority slots, windows bringing
    down only rebuilt chunks) read two stores with random damage at once from two threads.
    Locations are random mixes of good, bad, unreadable and short copies, some chunks with
    several; every part must come out as stored, in order, and a part left without d good
    chunks must fail its reader with TooFewShardsPresent."""
    import threading

    d, p, Lc, n = 6, 3, 8192, 96
    t = d + p
    results, errors = {}, {}

    def store(seed):
        chunks, dig = make_parts(n, d, p, Lc, seed)
        rng = np.random.default_rng(seed)
        st = Locations(chunks)
        good = {}
        for k in range(n):
            good[k] = 0
            for i in range(t):
                u = rng.random()
                if u < 0.75:
                    spec = ["good"]
                elif u < 0.85:
                    spec = ["bad", "good"]
                elif u < 0.9:
                    spec = ["gone", "short", "good"]
                elif u < 0.95:
                    spec = ["bad"]
                else:
                    spec = ["gone"]
                st.set(k, i, *spec)
                good[k] += "good" in spec
        return chunks, dig, st, good

    def run(name, seed):
        chunks, dig, st, good = store(seed)
        r = BatchReader(d, p, Lc, 4, 4, devices)
        got = []
        try:
            r.read(n, st.fetch, lambda k: dig[k],
                   lambda k, data: got.append((k, b"".join(bytes(x) for x in data))))
            errors[name] = None
        except ce.Error as e:
            errors[name] = e.code
        results[name] = (chunks, good, got, r)

    threads = [threading.Thread(target=run, args=(f"r{s}", 70 + s)) for s in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    for name, (chunks, good, got, r) in results.items():
        short = [k for k in range(n) if good[k] < d]
        # file order, stored bytes, up to the first part that cannot be decoded
        assert [k for k, _ in got] == list(range(len(got)))
        for k, b in got:
            assert b == chunks[k, :d].tobytes(), (name, k)
        if short:
            assert errors[name] == ce.TOO_FEW_SHARDS_PRESENT and len(got) <= short[0], name
        else:
            assert errors[name] is None and len(got) == n, name
        assert all(r.multi.stats(g)["carry_held"] == 0 for g in range(len(devices))), name


def test_failed_read_leaves_no_job_or_carry_id_behind():
    """A part that runs out of copies fails the read while other windows' retry rounds are in
    flight: the reader waits for every job it queued, gives every carry id back (none held), and
    the same reader then reads another file correctly."""
    d, p, Lc, n = 4, 2, 8192, 40
    chunks, dig = make_parts(n, d, p, Lc, 98)
    st = Locations(chunks)
    for k in (2, 9, 13, 21, 30):  # retried parts in several windows (4 parts per window)
        st.set(k, 1, "bad", "good")
    for i in range(p + 1):  # part 17: p + 1 chunks with no good copy
        st.set(17, i, "bad")
    r = BatchReader(d, p, Lc, 4, 4, [0])
    got = []
    with pytest.raises(ce.Error) as e:
        r.read(n, st.fetch, lambda k: dig[k], lambda k, data: got.append(k))
    assert e.value.code == ce.TOO_FEW_SHARDS_PRESENT
    assert got == list(range(len(got))) and len(got) <= 17
    assert r.multi.stats(0)["carry_held"] == 0
    good = Locations(chunks)
    out = {}
    r.read(n, good.fetch, lambda k: dig[k],
           lambda k, data: out.__setitem__(k, b"".join(bytes(x) for x in data)))
    assert all(out[k] == chunks[k, :d].tobytes() for k in range(n))
    assert r.multi.stats(0)["carry_held"] == 0


def test_file_reader_range_reads():
    """FileReader.read_range (FileReadBuilder::seek / take, reader.rs:22-173) on the GPU: the
    gateway's Range / Prefix / Suffix reads of an RS(3,2) file with a short last part and a lost
    chunk in every part return the range's bytes, reading only the parts that hold it."""
    import hashlib
    d, p, chunk = 3, 2, 8192
    rng = np.random.default_rng(23)
    fb = rng.integers(0, 256, 11 * d * chunk + 777, dtype=np.uint8).tobytes()
    shapes, copies, digs = [], {}, []
    for k, off in enumerate(range(0, len(fb), d * chunk)):
        piece = fb[off:off + d * chunk]
        Lk = -(-len(piece) // d)
        buf = np.zeros(d * Lk, np.uint8)
        buf[:len(piece)] = np.frombuffer(piece, np.uint8)
        data = [buf[j * Lk:(j + 1) * Lk] for j in range(d)]
        st, par = oracle.encode_sep(d, p, data)
        cs = [c.tobytes() for c in data] + [c.tobytes() for c in par]
        for i, c in enumerate(cs):
            copies[(k, i)] = [None] if i == k % d else [c]
        shapes.append((d, p, Lk))
        digs.append(np.array([np.frombuffer(hashlib.sha256(c).digest(), np.uint8) for c in cs]))
    read = set()

    def fetch(k, i, start):
        read.add(k)
        locs = copies[(k, i)]
        for j in range(start, len(locs)):
            if locs[j] is not None:
                return j, locs[j]
        return None
    n, part = len(fb), d * chunk
    reader = FileReader(2, 2, [0])
    for seek, take in ((0, 0), (0, 10), (part - 1, 2), (part, part), (5 * part + 7, 0),
                       (n - 777, 0), (n - 1, 0), (n - 100, 1000), (n, 0), (12345, 3 * part)):
        want = fb[seek:] if take == 0 else fb[seek:seek + take]
        read.clear()
        out = bytearray()
        reader.read_range(shapes, n, seek, take, fetch, lambda k: digs[k],
                          lambda k, pieces: [out.extend(bytes(x)) for x in pieces])
        assert bytes(out) == want, (seek, take)
        if want:
            assert read == set(range(seek // part, (seek + len(want) - 1) // part + 1)), (seek, take)
        else:
            assert not read
