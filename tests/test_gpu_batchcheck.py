"""chunky_ec.batchcheck.BatchChecker (the executed twin of the Rust crate's batch::BatchChecker and
of the C++ FileReference::verify / resilver batched paths) on the GPU: every location of every
chunk hashed (file_part.rs:236-243, :277-289), exactly the bad locations reported invalid and the
unreadable ones unavailable, only the chunks with no valid copy rebuilt (data and parity, checked
against the oracle), and the rebuilt copies' locations APPENDED to the chunks' lists
(file_part.rs:346) -- after which verify is ideal and the batched reader reads the store back
bit-exact.  The tests/cluster.rs:145-231 scenario (delete one data + one parity chunk per part,
verify, resilver, verify ideal) in location terms, on RS(3,2) and RS(10,4)."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

import chunky_ec as ce  # noqa: E402
from _stores import Locations, make_parts  # noqa: E402
from chunky_ec.batchcheck import BatchChecker  # noqa: E402
from chunky_ec.batchreader import BatchReader  # noqa: E402


def _verify(checker, n, st, dig):
    got = {}
    checker.verify(n, st.read_all, lambda k: dig[k], lambda k, part: got.__setitem__(k, part))
    assert sorted(got) == list(range(n))
    return got


@pytest.mark.parametrize("d,p,L", [(3, 2, 65536), (10, 4, 16384)])
@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_verify_marks_exactly_the_bad_locations(d, p, L, devices):
    n = 10
    t = d + p
    chunks, dig = make_parts(n, d, p, L, 60 + d)
    st = Locations(chunks)
    bad, gone = set(), set()
    for k in range(n):
        for i in range(p + 1):  # p + 1 chunks per part listed [bad, good]
            c = (k + 2 * i) % t
            st.set(k, c, "bad", "good")
            bad.add((k, c, 0))
    st.set(3, 1, "gone", "bad", "good", "bad")
    bad -= {(3, 1, 0)}
    bad |= {(3, 1, 1), (3, 1, 3)}
    gone.add((3, 1, 0))
    c = BatchChecker(d, p, L, 4, 2, devices)
    got = _verify(c, n, st, dig)
    for k in range(n):
        for i in range(t):
            for j, r in enumerate(got[k].locations[i]):
                want = None if (k, i, j) in gone else ((k, i, j) not in bad)
                assert r is want, (k, i, j, r)
        assert got[k].healthy_chunks() == t  # every chunk has a valid copy: the part is Valid
    assert sum(g.invalid_locations() for g in got.values()) == len(bad)
    assert sum(g.unavailable_locations() for g in got.values()) == 1


@pytest.mark.parametrize("d,p,L", [(3, 2, 65536), (10, 4, 16384)])
def test_resilver_appends_and_the_store_reads_back(d, p, L):
    """tests/cluster.rs:145-231 with locations: delete data[0] and parity[0] of every part (their
    only location), flip a byte of another chunk's first copy where a second good copy exists, and
    give one part too few chunks (its write_error is reported, the others are resilvered)."""
    n = 13
    t = d + p
    chunks, dig = make_parts(n, d, p, L, 70 + d)
    st = Locations(chunks)
    for k in range(n):
        if k != 8:
            st.set(k, 0, "gone")
        st.set(k, d, "gone")
    st.set(5, 1, "bad", "good")  # healthy: must not be rewritten
    st.set(8, 2, "bad")          # its only copy is bad (data[0] kept): rebuilt, location appended
    lost = 9
    for i in range(1, p):        # part 9: p + 1 chunks gone, no rebuild possible
        st.set(lost, d + i, "gone")
    checker = BatchChecker(d, p, L, 4, 2, [0, 0])
    before = _verify(checker, n, st, dig)
    unavailable = sum(g.unavailable_locations() for g in before.values())
    assert unavailable == 2 * n - 1 + (p - 1)
    assert all(before[k].healthy_chunks() == t - 2 for k in range(n) if k not in (8, lost))

    new_locations = []

    def sink(k, part):
        if part.error is not None:
            assert k == lost and part.error == ce.TOO_FEW_SHARDS_PRESENT and not part.rebuilt
            return
        for i, blob in part.rebuilt.items():
            assert bytes(blob) == chunks[k, i].tobytes(), (k, i)  # data and parity, as the oracle
            new_locations.append((k, i, st.append(k, i, blob)))
    checker.resilver(n, st.read_all, lambda k: dig[k], sink)
    rebuilt = sorted((k, i) for k, i, _ in new_locations)
    want = sorted([(k, 0) for k in range(n) if k not in (8, lost)] +
                  [(k, d) for k in range(n) if k != lost] + [(8, 2)])
    assert rebuilt == want
    # appended, not overwritten: the bad / unreadable first locations are still listed
    for k, i, j in new_locations:
        assert j == len(st.locs(k, i)) - 1 and j >= 1
    assert st.locs(5, 1)[0] != chunks[5, 1].tobytes() and len(st.locs(5, 1)) == 2

    after = _verify(checker, n, st, dig)
    for k in range(n):
        if k != lost:
            assert after[k].healthy_chunks() == t, k  # verify is ideal again (cluster.rs:186)
    # and the batched reader reads the repaired parts back through their [bad, good] lists
    ok = [k for k in range(n) if k != lost]
    r = BatchReader(d, p, L, 4, 2, [0])
    got = []
    r.read(len(ok), lambda q, i, s: st.fetch(ok[q], i, s), lambda q: dig[ok[q]],
           lambda q, data: got.append(b"".join(bytes(x) for x in data)))
    assert got == [chunks[k, :d].tobytes() for k in ok]
