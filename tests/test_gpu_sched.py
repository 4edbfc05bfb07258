"""The scheduler's pipelines and carry on the GPU (round-6 verdict items 2 and 3):

* every cec_multi shard makes its pipelines ONCE, in cec_multi_new; verify, resilver and read
  jobs (FilePart::verify / resilver / read_with_context on the same parts, file_part.rs:73-390)
  pick their mode per submit on the same read pipeline, so no stream or device buffer is made
  while another shard's batches run (the round-5 deadlock);
* one read pipeline serves every mode per submit (cec_read_pipeline_submit_ex), results against
  the oracle;
* read retries through the scheduler keep their verified chunks on the GPU (cec_multi_read_carry:
  file_part.rs:92-107 keeps them in memory), so fewer chunks go up than without carry, and the
  parts still come back bit-exact;
* a carry id is accepted only for the part it was kept for (same digests, its verified chunks
  among the kept ones), and entries nobody claimed go back when their slot is reused."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

import chunky_ec as ce  # noqa: E402
import oracle  # noqa: E402
from _stores import Locations, make_parts  # noqa: E402
from chunky_ec.batchcheck import FileChecker  # noqa: E402
from chunky_ec.batchreader import BatchReader  # noqa: E402


def _made():
    return int(ce._lib.cec_pipelines_made())


def test_scheduler_makes_its_pipelines_once_across_verify_resilver_read():
    """[0, 0] shards: one read pipeline each, made in cec_multi_new; a verify, a resilver, a read
    with damaged chunks and another verify make none (cec_pipelines_made and the shards' own
    counters), and every job's results match the oracle."""
    d, p, L, n = 4, 2, 8192, 24
    t = d + p
    chunks, dig = make_parts(n, d, p, L, 90)
    m0 = _made()
    m = ce.Multi(ce.ReedSolomon(d, p), L, 4, 2, [0, 0], kinds=ce.Multi.READ)
    assert _made() - m0 == 2
    assert [m.stats(g)["pipelines_made"] for g in range(2)] == [1, 1]
    rng = np.random.default_rng(5)
    for rnd in range(2):
        # verify: every chunk loaded, a few damaged
        ch = chunks.copy()
        bad = {(int(k), int(i)) for k, i in zip(rng.integers(0, n, 6), rng.integers(0, t, 6))}
        for k, i in bad:
            ch[k, i, 7] ^= 0x40
        pres = np.ones((n, t), np.uint8)
        ver = np.zeros((n, t), np.uint8)
        m.verify_sync(ch, pres, dig, n, ver)
        want = np.ones((n, t), np.uint8)
        for k, i in bad:
            want[k, i] = 0
        assert np.array_equal(ver, want)
        # resilver: chunk 0 and d of every part missing, the damaged ones fail verification
        pres[:, 0] = pres[:, d] = 0
        rebuilt = np.zeros((n, t, L), np.uint8)
        st = np.zeros(n, np.int32)
        m.resilver_sync(ch, pres, dig, n, rebuilt, ver, st)
        for k in range(n):
            lost = {0, d} | {i for kk, i in bad if kk == k}
            if t - len(lost) < d:
                assert st[k] == ce.TOO_FEW_SHARDS_PRESENT
                continue
            assert st[k] == ce.OK, k
            for i in lost:
                assert np.array_equal(rebuilt[k, i], chunks[k, i]), (k, i)
        # read: d random chunks per part (the damaged copies among them fail, TooFew or decoded)
        pres = np.zeros((n, t), np.uint8)
        for k in range(n):
            pres[k, rng.permutation(t)[:d]] = 1
        out = np.zeros((n, d, L), np.uint8)
        st[:] = 0
        m.read_sync(ch, pres, dig, n, out, ver, st)
        for k in range(n):
            hit = any(pres[k, i] for kk, i in bad if kk == k)
            assert st[k] == (ce.TOO_FEW_SHARDS_PRESENT if hit else ce.OK), k
            if not hit:
                assert np.array_equal(out[k], chunks[k, :d]), k
    assert _made() - m0 == 2
    assert [m.stats(g)["pipelines_made"] for g in range(2)] == [1, 1]
    # a job of a kind the scheduler was not made for is refused
    with pytest.raises(ce.Error):
        m.encode_hash(np.zeros((1, d, L), np.uint8), 1, np.zeros((1, p, L), np.uint8),
                      np.zeros((1, t, 32), np.uint8))


def test_file_checker_verify_resilver_then_read_make_no_pipeline():
    """FileChecker verify -> resilver (then verify again) over [0, 0]: the one checker's
    scheduler made one read pipeline per shard, at its creation, and the jobs made none; the
    resilvered store then reads back bit-exact through a BatchReader."""
    d, p, L, n = 3, 2, 16384, 12
    chunks, dig = make_parts(n, d, p, L, 91)
    st = Locations(chunks)
    for k in range(n):
        st.set(k, 0, "gone")
        st.set(k, d, "bad", "good")
    fc = FileChecker(4, 2, [0, 0])
    shapes = [(d, p, L)] * n
    m0 = _made()
    reports = {}
    fc.verify(shapes, st.read_all, lambda k: dig[k], lambda k, r: reports.__setitem__(k, r))
    assert _made() - m0 == 2  # the checker's scheduler: one read pipeline per shard
    def rebuilt(k, part):  # resilver's write-back: the rebuilt copy's location is appended
        assert part.error is None
        for i, blob in part.rebuilt.items():
            assert bytes(blob) == chunks[k, i].tobytes(), (k, i)
            st.append(k, i, blob)
    fc.resilver(shapes, st.read_all, lambda k: dig[k], rebuilt)
    fc.verify(shapes, st.read_all, lambda k: dig[k], lambda k, r: reports.__setitem__(k, r))
    assert _made() - m0 == 2
    assert all(r.healthy_chunks() == d + p for r in reports.values())
    r = BatchReader(d, p, L, 4, 2, [0, 0])
    got = {}
    r.read(n, st.fetch, lambda k: dig[k], lambda k, data: got.__setitem__(k, b"".join(map(bytes, data))))
    assert all(got[k] == chunks[k, :d].tobytes() for k in range(n))


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_scheduler_read_retries_keep_verified_chunks_on_the_gpu(devices):
    """Damaged first copies (listed [bad, good]) on RS(10,4): every retried part's verified chunks
    stay on its shard's GPU, so the retries send only their new chunks -- fewer chunks go up than
    with carry off -- and both read the stored bytes; no carry entry is left held."""
    d, p, L, n = 10, 4, 16384, 40
    chunks, dig = make_parts(n, d, p, L, 92)
    ups = {}
    for carry in (True, False):
        st = Locations(chunks)
        for k in range(0, n, 3):
            st.set(k, (k // 3) % d, "bad", "good")
        r = BatchReader(d, p, L, 8, 2, devices, carry=carry)
        got = {}
        r.read(n, st.fetch, lambda k: dig[k],
               lambda k, data: got.__setitem__(k, b"".join(map(bytes, data))))
        assert all(got[k] == chunks[k, :d].tobytes() for k in range(n))
        stats = [r.multi.stats(g) for g in range(len(devices))]
        ups[carry] = sum(s["chunks_uploaded"] for s in stats)
        retried = len(range(0, n, 3))
        assert r.retries == retried
        if carry:
            assert r.carried_parts == retried
            assert sum(s["chunks_carried"] for s in stats) == retried * (d - 1)
        else:
            assert sum(s["chunks_carried"] for s in stats) == 0
        assert all(s["carry_held"] == 0 for s in stats)
    # each retry sends 1 chunk with carry, d (its d - 1 verified + 1 new) without
    assert ups[False] - ups[True] == len(range(0, n, 3)) * (d - 1)


def test_scheduler_carry_id_refused_for_another_part():
    """cec_multi_read_carry: ids swapped between two parts fail the retry job
    (CEC_ERR_INVALID_ARGUMENT: the digests differ), and the ids stay usable for their own parts,
    which then decode to the stored bytes."""
    d, p, L, n = 4, 2, 4096, 2
    t = d + p
    chunks, dig = make_parts(n, d, p, L, 93)
    m = ce.Multi(ce.ReedSolomon(d, p), L, 4, 2, [0], kinds=ce.Multi.READ)
    ch = chunks.copy()
    pres = np.zeros((n, t), np.uint8)
    pres[:, :d] = 1
    ch[0, 1, 0] ^= 1
    ch[1, 2, 0] ^= 1
    out = np.zeros((n, d, L), np.uint8)
    ver = np.zeros((n, t), np.uint8)
    st = np.zeros(n, np.int32)
    cout = np.full(n, -1, np.int32)
    job, _ = m.read(ch, pres, dig, n, out, ver, st, carry_out=cout)
    m.wait(job)
    assert list(st) == [ce.TOO_FEW_SHARDS_PRESENT] * 2 and (cout >= 0).all()
    assert m.stats(0)["carry_held"] == 2
    # the retry: verified chunks from the GPU, one parity chunk fetched
    rpres = np.where(ver != 0, ce.PRESENT_VERIFIED, 0).astype(np.uint8)
    rch = np.zeros_like(ch)
    for k in range(n):
        rpres[k, d] = 1
        rch[k, d] = chunks[k, d]
    with pytest.raises(ce.MultiError) as e:
        job, _ = m.read(rch, rpres, dig, n, out, ver, st, carry_in=cout[::-1].copy())
        m.wait(job)
    assert e.value.code == ce.ERR_INVALID_ARGUMENT
    job, _ = m.read(rch, rpres, dig, n, out, ver, st, carry_in=cout)
    m.wait(job)
    assert list(st) == [ce.OK] * 2
    for k in range(n):
        assert np.array_equal(out[k], chunks[k, :d]), k
    assert m.stats(0)["carry_held"] == 0


def test_pipeline_carry_refuses_swapped_ids_and_wider_masks():
    """submit with a carry id checks that the id was kept for that part -- a
    swapped id (other digests) and a CEC_PRESENT_VERIFIED flag on a chunk the entry does not hold
    are refused before anything is queued; the right ids decode the parts."""
    d, p, L = 3, 2, 2048
    t = d + p
    chunks, dig = make_parts(2, d, p, L, 94)
    rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, 2, 2, ce.ReadPipeline.CARRY)
    slot, ch, pres, exp = rp.acquire()
    pres[:2] = 0
    for k in range(2):
        ch[k] = chunks[k]
        exp[k] = dig[k]
        pres[k, :d] = 1
    ch[0, 2, 1] ^= 1  # part 0 keeps chunks 0, 1
    ch[1, 0, 1] ^= 1  # part 1 keeps chunks 1, 2
    rp.submit(slot, 2)
    _, ver, st = rp.wait(slot)
    assert list(st) == [ce.TOO_FEW_SHARDS_PRESENT] * 2
    ids = rp.carry_ids(slot, 2)
    assert (ids >= 0).all() and rp.carry_held() == 2

    def retry(ids_, wide=False):
        slot, ch, pres, exp = rp.acquire()
        pres[:2] = 0
        for k in range(2):
            exp[k] = dig[k]
            pres[k, :d] = np.where(ver[k, :d] != 0, ce.PRESENT_VERIFIED, 0)
            pres[k, d] = 1
            ch[k, d] = chunks[k, d]
        if wide:  # part 0 claims chunk 2 verified too: its entry does not hold it
            pres[0, 2] = ce.PRESENT_VERIFIED
        rp.submit_carried(slot, 2, ids_)
        return slot

    for bad_ids, wide in ((ids[::-1].copy(), False), (ids, True)):
        with pytest.raises(ce.Error) as e:
            retry(bad_ids, wide)
        assert e.value.code == ce.ERR_INVALID_ARGUMENT
        assert rp.carry_held() == 2  # refused before anything was queued or consumed
    slot = retry(ids)
    _, _, st = rp.wait(slot)
    assert list(st) == [ce.OK] * 2 and rp.carry_held() == 0
    for k in range(2):
        assert rp.part_bytes(slot, 2, k) == chunks[k, :d].tobytes()


def test_pipeline_unclaimed_carry_entries_go_back():
    """entries of a batch whose ids nobody took (plain submits, no
    carry_ids call) go back when the slot is submitted again, so the pool never fills up with
    entries no caller holds: 50 rounds of all-failing batches keep getting ids."""
    d, p, L, P = 3, 2, 1024, 8
    chunks, dig = make_parts(P, d, p, L, 95)
    rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, P, 2, ce.ReadPipeline.CARRY)
    for rnd in range(50):
        slot, ch, pres, exp = rp.acquire()
        pres[:] = 0
        ch[:] = chunks
        exp[:] = dig
        pres[:, :d] = 1
        ch[:, 0, 0] ^= 1  # every part: chunk 0 bad -> TooFew, 2 chunks kept
        rp.submit(slot, P)
        _, _, st = rp.wait(slot)
        assert (st == ce.TOO_FEW_SHARDS_PRESENT).all()
        if rnd == 49:
            ids = rp.carry_ids(slot, P)
            assert (ids >= 0).all()
    assert rp.carry_held() == P
    for i in ids:
        rp.carry_release(int(i))
    assert rp.carry_held() == 0


@pytest.mark.parametrize("packed", [False, True])
def test_one_pipeline_serves_every_mode_per_submit(packed):
    """cec_read_pipeline_submit_ex on one CEC_PIPE_EXTERNAL | CEC_READ_CARRY pipeline: a verify,
    a resilver, a read and a REBUILT_ONLY read submit in turn on the same slots (what a
    scheduler shard does), each against the oracle / the stored chunks; a carried retry from a
    packed batch; a resilver into the slot's d-wide output is refused."""
    d, p, L, P = 4, 2, 4096 + 64, 6
    t = d + p
    chunks, dig = make_parts(P, d, p, L, 96)
    made = _made()
    rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, P, 2, ce.PIPE_EXTERNAL | ce.ReadPipeline.CARRY)
    rng = np.random.default_rng(8)

    def go(mode, pres, ch, out=None, ids=None):
        slot, _, _, _ = rp.acquire()
        if packed:
            sel = [ch[k, i] for k in range(P) for i in range(t)
                   if pres[k, i] and not (ids is not None and ids[k] >= 0 and
                                          pres[k, i] == ce.PRESENT_VERIFIED)]
            buf = np.ascontiguousarray(np.stack(sel)) if sel else np.zeros((1, L), np.uint8)
        else:
            buf = ch
        rp.submit_ex(slot, P, chunks=buf, present=pres, expected=dig, data=out, carry_ids=ids,
                     mode=mode, packed=packed)
        keep = (buf, out)
        res = rp.wait(slot)
        return slot, res, keep

    for rnd in range(3):
        ch = chunks.copy()
        ch[1, 2, 5] ^= 1
        # verify
        pres = np.ones((P, t), np.uint8)
        _, (_, ver, st), _ = go(ce.READ_VERIFY_ONLY, pres, ch)
        want = np.ones((P, t), np.uint8)
        want[1, 2] = 0
        assert np.array_equal(ver, want) and (st == ce.OK).all()
        # resilver: chunk 0 missing everywhere, part 1's chunk 2 bad
        pres[:, 0] = 0
        out = np.zeros((P, t, L), np.uint8)
        slot, (_, ver, st), keep = go(ce.READ_RESILVER, pres, ch, out)  # keep: ptrs into it
        assert (st == ce.OK).all()
        for k in range(P):
            for i in ([0, 2] if k == 1 else [0]):
                assert np.array_equal(out[k, i], chunks[k, i]), (k, i)
        ptrs = rp.data_chunks(slot, P, out_chunks=t)
        for k in range(P):
            for i in range(t):
                assert ctypes.string_at(int(ptrs[k, i]), L) == chunks[k, i].tobytes()
        # read: d random chunks; part 1 includes its bad chunk 2 -> TooFew with a carry id
        pres = np.zeros((P, t), np.uint8)
        for k in range(P):
            pres[k, rng.permutation(t)[:d]] = 1
        pres[1] = 0
        pres[1, :d] = 1
        out = np.zeros((P, d, L), np.uint8)
        slot, (_, ver, st), _ = go(0, pres, ch, out)
        for k in range(P):
            if k == 1:
                assert st[k] == ce.TOO_FEW_SHARDS_PRESENT
            else:
                assert st[k] == ce.OK and np.array_equal(out[k], chunks[k, :d]), k
        ids = rp.carry_ids(slot, P)
        assert ids[1] >= 0 and (np.delete(ids, 1) == -1).all()
        # REBUILT_ONLY retry of part 1 (its verified chunks from the pool) with all other parts
        # re-read: their loaded chunks stay where read
        rpres = pres.copy()
        rpres[1] = np.where(ver[1] != 0, ce.PRESENT_VERIFIED, 0)
        rpres[1, d] = 1
        rch = ch.copy()
        rch[1, :d] = 0x5A  # the caller need not hold the carried chunks
        out = np.zeros((P, d, L), np.uint8)
        slot, (_, ver, st), keep = go(ce.ReadPipeline.REBUILT_ONLY, rpres, rch, out, ids)
        assert (st == ce.OK).all()
        for k in range(P):
            assert rp.part_bytes(slot, P, k) == chunks[k, :d].tobytes(), k
        assert rp.carry_held() == 0
    # the slot's own output of an external pipeline does not exist: resilver needs data_out
    slot, _, _, _ = rp.acquire()
    with pytest.raises(ce.Error):
        rp.submit_ex(slot, P, chunks=chunks, present=np.ones((P, t), np.uint8), expected=dig,
                     mode=ce.READ_RESILVER)
    assert _made() - made == 1


def test_scheduler_releases_carry_ids_while_idle():
    """cec_multi_carry_release hands the ids to their shard's worker, which gives them back even
    when no read job follows (the worker wakes for them): the held count drops to 0."""
    import time
    d, p, L, n = 4, 2, 4096, 6
    t = d + p
    chunks, dig = make_parts(n, d, p, L, 97)
    m = ce.Multi(ce.ReedSolomon(d, p), L, 8, 2, [0, 0], kinds=ce.Multi.READ)
    ch = chunks.copy()
    ch[:, 0, 0] ^= 1  # every part: chunk 0 bad -> TooFewShardsPresent, 3 chunks kept
    pres = np.zeros((n, t), np.uint8)
    pres[:, :d] = 1
    out, ver = np.zeros((n, d, L), np.uint8), np.zeros((n, t), np.uint8)
    st, cout = np.zeros(n, np.int32), np.full(n, -1, np.int32)
    job, _ = m.read(ch, pres, dig, n, out, ver, st, carry_out=cout)
    m.wait(job)
    assert (st == ce.TOO_FEW_SHARDS_PRESENT).all() and (cout >= 0).all()
    assert {int(c) >> 20 for c in cout} == {0, 1}  # both shards kept some
    assert sum(m.stats(g)["carry_held"] for g in range(2)) == n
    for c in cout:
        m.carry_release(int(c))
    deadline = time.time() + 5
    while sum(m.stats(g)["carry_held"] for g in range(2)) and time.time() < deadline:
        time.sleep(0.01)
    assert sum(m.stats(g)["carry_held"] for g in range(2)) == 0
    with pytest.raises(ce.Error):
        m.carry_release(7 << 20)  # no shard 7


def test_ahead_job_overtakes_queued_jobs():
    """CEC_MULTI_AHEAD (a reader's retry round): a read job so flagged goes ahead of the queued
    jobs that have not started, so it is done while most of eight read jobs submitted before it
    are still to run; every job's parts are still the stored bytes, and an unknown flag bit is
    refused."""
    d, p, L, n, P = 4, 2, 1 << 18, 64, 16
    t = d + p
    chunks, dig = make_parts(n, d, p, L, 96)
    m = ce.Multi(ce.ReedSolomon(d, p), L, P, 2, [0], kinds=ce.Multi.READ)
    host = ce.HostBuffer(n * t * L, 0)  # page-locked: no staging copy in the timing
    host.view(n, t, L)[:] = chunks
    pres = np.zeros((n, t), np.uint8)
    pres[:, :d] = 1
    jobs, outs = [], []
    for _ in range(8):
        out = np.zeros((n, d, L), np.uint8)
        ver = np.zeros((n, t), np.uint8)
        st = np.zeros(n, np.int32)
        outs.append((out, ver, st))
        jobs.append(m.read(host.array, pres, dig, n, out, ver, st)[0])
    a_out = np.zeros((1, d, L), np.uint8)
    a_ver = np.zeros((1, t), np.uint8)
    a_st = np.zeros(1, np.int32)
    aj, _ = m.read(host.array[: t * L], pres[:1], dig[:1], 1, a_out, a_ver, a_st, ahead=True)
    m.wait(aj)
    done_then = m.stats(0)["parts"]
    for j in jobs:
        m.wait(j)
    assert done_then < 8 * n - n, done_then  # at least one whole earlier job still to run
    assert a_st[0] == ce.OK and np.array_equal(a_out[0], chunks[0, :d])
    for out, ver, st in outs:
        assert (st == ce.OK).all() and np.array_equal(out, chunks[:, :d])
    with pytest.raises(ce.MultiError):
        job = ctypes.c_uint64(0)
        code = ce._lib.cec_multi_read_carry(m._h, host.array.ctypes.data, pres.ctypes.data,
                                            dig.ctypes.data, 1, a_out.ctypes.data,
                                            a_ver.ctypes.data, a_st.ctypes.data_as(
                                                ctypes.POINTER(ctypes.c_int)), None, 128,
                                            None, None, ctypes.byref(job))
        if code != ce.OK:
            raise ce.MultiError(code)


def test_multi_query_never_blocks_and_tracks_the_job():
    """cec_multi_query: 0 while a job runs, 1 once it is done (wait then returns at once), and
    CEC_ERR_INVALID_ARGUMENT for a job already waited for or never submitted."""
    import time
    d, p, L, n = 4, 2, 1 << 18, 64
    t = d + p
    chunks, dig = make_parts(n, d, p, L, 97)
    m = ce.Multi(ce.ReedSolomon(d, p), L, 16, 2, [0], kinds=ce.Multi.READ)
    pres = np.zeros((n, t), np.uint8)
    pres[:, :d] = 1
    out = np.zeros((n, d, L), np.uint8)
    ver = np.zeros((n, t), np.uint8)
    st = np.zeros(n, np.int32)
    job, _ = m.read(chunks, pres, dig, n, out, ver, st)
    seen, t0 = [], time.perf_counter()
    while not m.query(job):
        seen.append(0)
        assert time.perf_counter() - t0 < 60
        time.sleep(1e-3)
    assert m.query(job)  # stays done until waited for
    m.wait(job)
    assert (st == ce.OK).all() and np.array_equal(out, chunks[:, :d])
    for bad in (job, job + 1000):
        with pytest.raises(ce.MultiError) as e:
            m.query(bad)
        assert e.value.code == ce.ERR_INVALID_ARGUMENT
