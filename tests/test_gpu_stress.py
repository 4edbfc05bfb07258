"""Ordering stress for the read / resilver paths: many small batches in flight (small chunks, so
kernels and copies finish in microseconds and any missing stream dependency shows up), parts
whose speculative decode must be redone (a corrupted loaded chunk), several scheduler jobs
queued at once.  Every returned byte is checked against the written data.

Round 2 found a race on this path (work queued behind a hipFreeAsync of the decode patterns did
not reliably wait for the decode): the C++ mirror's batched verify/resilver (a plain C++ process)
failed 4 of 4 runs until per-launch metadata moved to the event-recycled scratch pool
(DESIGN.md §4.9).  These Python cases, run against the old allocator in this (torch) process,
did not reproduce it (profiles/r2_fix/stress/); they stay as ordering coverage next to the
mirror case, which does.
"""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import chunky_ec as ce  # noqa: E402

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)


def _parts(d, p, L, n, seed):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (n, d, L), dtype=np.uint8)
    full = np.zeros((n, d + p, L), np.uint8)
    full[:, :d] = data
    dig = np.zeros((n, d + p, 32), np.uint8)
    for k in range(n):
        st, par = oracle.encode_sep(d, p, [data[k, j] for j in range(d)])
        assert st == 0
        for i in range(p):
            full[k, d + i] = par[i]
        for i in range(d + p):
            dig[k, i] = np.frombuffer(hashlib.sha256(full[k, i].tobytes()).digest(), np.uint8)
    return full, dig


def _damage(full, d, p, rng):
    """Erase chunk 0 and the first parity chunk of every part; corrupt data chunk 2 of every
    third part (its speculative decode is redone); the first d+1 stored chunks are loaded."""
    n, t, L = full.shape
    chunks = full.copy()
    present = np.zeros((n, t), np.uint8)
    bad = np.zeros((n, t), bool)
    for k in range(n):
        stored = [i for i in range(t) if i not in (0, d)]
        present[k, stored[: d + 1]] = 1
        if k % 3 == 1:
            chunks[k, 2, int(rng.integers(0, L))] ^= 0x41
            bad[k, 2] = True
    chunks[present == 0] = 0
    return chunks, present, bad


@pytest.mark.parametrize("devices", [[0], [0, 0]])
@pytest.mark.parametrize("L", [1024, 4096])
def test_many_small_jobs_read_and_resilver(devices, L):
    d, p, n, ppb, depth, jobs = 3, 3, 24, 4, 2, 6
    t = d + p
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, ppb, depth, devices)
    full, dig = _parts(d, p, L, n, L + len(devices))
    rng = np.random.default_rng(7)
    bufs = []
    for r in range(jobs):  # all queued before the first wait
        chunks, present, bad = _damage(full, d, p, rng)
        src = ce.HostBuffer(n * t * L)
        src.view(n, t, L)[:] = chunks
        if r % 2 == 0:
            out = ce.HostBuffer(n * d * L)
            ver, st = np.zeros((n, t), np.uint8), np.zeros(n, np.int32)
            job, _ = m.read(src, present, dig, n, out, ver, st)
            bufs.append(("read", job, out, ver, st, present, bad))
        else:
            out = ce.HostBuffer(n * t * L)
            ver, st = np.zeros((n, t), np.uint8), np.zeros(n, np.int32)
            job, _ = m.resilver(src, present, dig, n, out, ver, st)
            bufs.append(("resilver", job, out, ver, st, present, bad))
        bufs[-1] = bufs[-1] + (src,)
    for kind, job, out, ver, st, present, bad, _src in bufs:
        m.wait(job)
        assert (st == 0).all(), kind
        assert np.array_equal(ver.astype(bool), present.astype(bool) & ~bad), kind
        if kind == "read":
            assert np.array_equal(out.view(n, d, L), full[:, :d]), kind
        else:
            got = out.view(n, t, L)
            for k in range(n):
                for i in range(t):
                    if not ver[k, i]:
                        assert np.array_equal(got[k, i], full[k, i]), (kind, k, i)


@pytest.mark.parametrize("flags", [0, ce.ReadPipeline.REBUILT_ONLY, ce.READ_RESILVER])
def test_read_pipeline_small_batches_with_redo(flags):
    """Two slots, 80 batches of 4 parts with a redo part in most batches."""
    d, p, L, P, depth = 3, 3, 1024, 4, 2
    t = d + p
    rs = ce.ReedSolomon(d, p)
    rp = ce.ReadPipeline(rs, L, P, depth, flags)
    full, dig = _parts(d, p, L, 40, 99)
    rng = np.random.default_rng(3)
    pending = {}

    def check(slot, b):
        data, ver, st = rp.wait(slot)
        idx, present, bad = pending.pop(slot)
        assert (st == 0).all(), b
        assert np.array_equal(ver.astype(bool), present.astype(bool) & ~bad), b
        if flags == ce.READ_RESILVER:  # every chunk, verified where read or rebuilt
            ptrs = (ctypes.c_void_p * (P * t))()
            assert ce._lib.cec_read_pipeline_data_chunks(rp._h, slot, ptrs, len(ptrs)) == 0
            for q, k in enumerate(idx):
                for i in range(t):
                    assert ctypes.string_at(ptrs[q * t + i], L) == full[k, i].tobytes(), (b, q, i)
            return
        for q, k in enumerate(idx):
            assert rp.part_bytes(slot, P, q) == full[k, :d].tobytes(), (b, q)

    for b in range(80):
        slot, chunks, present, expected = rp.acquire()
        if slot in pending:
            check(slot, b)
        idx = [(4 * b + q) % 40 for q in range(P)]
        c, pr, bad = _damage(full[idx], d, p, rng)
        if b % 4 == 0:
            bad[:] = False  # a batch without redo
            c = full[idx].copy()
            c[pr == 0] = 0
        chunks[:] = c
        present[:] = pr
        expected[:] = dig[idx]
        rp.submit(slot, P)
        pending[slot] = (idx, pr.copy(), bad.copy())
    for slot in list(pending):
        check(slot, -1)
    rp.drain()


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_verify_resilver_verify_mode_switches(devices):
    """tests/cluster.rs's delete + resilver, batched the way FileReference::verify / resilver
    run it (windows of 8 parts through one scheduler, the read pipeline recreated at each mode
    switch): verify, resilver, verify again, read.  The exact sequence of the C++ mirror case
    that exposed the round-2 race."""
    d, p, L, n, ppb, depth = 3, 3, 1024, 11, 4, 2
    t = d + p
    W = ppb * depth * len(devices)
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, ppb, depth, devices)
    full, dig = _parts(d, p, L, n, 1234)
    store = full.copy()
    avail = np.ones((n, t), bool)
    avail[:, 0] = avail[:, d] = False
    for k in range(1, n, 3):
        store[k, 2, 7] ^= 0xFF

    def load():
        chunks = ce.HostBuffer(n * t * L)
        chunks.view(n, t, L)[:] = np.where(avail[:, :, None], store, 0)
        return chunks, avail.astype(np.uint8)

    def windows(fn):
        for at in range(0, n, W):
            fn(at, min(W, n - at))

    chunks, present = load()
    ver = np.zeros((n, t), np.uint8)
    windows(lambda at, c: m.verify_sync(chunks.view(n, t, L)[at:at + c], present[at:at + c].copy(),
                                        dig[at:at + c].copy(), c, ver[at:at + c]))
    want = avail.copy()
    want[1::3, 2] = False
    assert np.array_equal(ver.astype(bool), want)
    rebuilt = ce.HostBuffer(n * t * L)
    st = np.zeros(n, np.int32)
    ver2 = np.zeros((n, t), np.uint8)

    def res(at, c):
        out = ce.HostBuffer(c * t * L)
        v = np.zeros((c, t), np.uint8)
        s = np.zeros(c, np.int32)
        m.resilver_sync(chunks.view(n, t, L)[at:at + c], present[at:at + c].copy(),
                        dig[at:at + c].copy(), c, out, v, s)
        rebuilt.view(n, t, L)[at:at + c] = out.view(c, t, L)
        ver2[at:at + c] = v
        st[at:at + c] = s

    windows(res)
    assert (st == 0).all()
    for k in range(n):
        for i in range(t):
            if not ver2[k, i]:  # written back, as resilver does
                assert np.array_equal(rebuilt.view(n, t, L)[k, i], full[k, i]), (k, i)
                store[k, i] = rebuilt.view(n, t, L)[k, i]
                avail[k, i] = True
    chunks, present = load()
    ver3 = np.zeros((n, t), np.uint8)
    windows(lambda at, c: m.verify_sync(chunks.view(n, t, L)[at:at + c], present[at:at + c].copy(),
                                        dig[at:at + c].copy(), c, ver3[at:at + c]))
    assert ver3.all()


def test_concurrent_read_batches_on_many_streams():
    """16 host threads call cec_read_batch at once, each on its own stream (each read forks its
    speculative decode onto a pooled side stream and joins it back): many more streams than
    the process's hardware queues, cross-stream event waits in flight together.  Every read
    rebuilds its parts bit-exact and none waits forever (tools/stress_read_batch.py, the same
    at 48 threads)."""
    import os
    import sys
    import types
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tools"))
    import stress_read_batch as srb
    import threading
    errors = []
    args = types.SimpleNamespace(iters=5)
    ths = [threading.Thread(target=srb.worker, args=(i, args, errors)) for i in range(16)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths), "a read never finished"
    assert not errors, errors


def test_scheduler_jobs_from_many_threads():
    """8 host threads submit and wait for their own write jobs on ONE scheduler (two shards on
    cuda:0) at the same time, pageable and page-locked buffers mixed: every job gets its own
    parts' parity and digests (the scheduler's job queue and completion are shared)."""
    import threading
    d, p, L = 10, 4, 4096
    t = d + p
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, 4, 2, [0, 0])
    errors = []

    def worker(w):
        try:
            for it in range(4):
                n = 5 + (w + it) % 7
                data, dig_ref = _parts(d, p, L, n, 300 + 10 * w + it)
                if (w + it) % 2:
                    hb = [ce.HostBuffer(n * d * L), ce.HostBuffer(n * p * L),
                          ce.HostBuffer(n * t * 32)]
                    src, par, dg = hb[0].view(n, d, L), hb[1].view(n, p, L), hb[2].view(n, t, 32)
                    src[:] = data[:, :d]
                else:
                    src = np.ascontiguousarray(data[:, :d])
                    par = np.zeros((n, p, L), np.uint8)
                    dg = np.zeros((n, t, 32), np.uint8)
                m.wait(m.encode_hash(src, n, par, dg))
                assert np.array_equal(par, data[:, d:]), (w, it)
                assert np.array_equal(dg, dig_ref), (w, it)
        except Exception as e:  # noqa: BLE001
            errors.append(f"{w}: {e!r}")

    ths = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in ths), "a job never finished"
    assert not errors, errors


def test_mixed_workload_in_one_process():
    """Every tier at once in one process: a scheduler write stream (two shards on cuda:0), 24
    per-call part_encode callers, 6 threads of device-batch reads on their own streams and a
    read pipeline — each checked bit-exact, none left waiting."""
    import os
    import sys
    import threading
    import types
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tools"))
    import stress_read_batch as srb
    d, p, L = 10, 4, 8192
    t = d + p
    rs = ce.ReedSolomon(d, p)
    errors = []

    def guard(fn, name):
        def run():
            try:
                fn()
            except Exception as e:  # noqa: BLE001
                errors.append(f"{name}: {e!r}")
        return run

    def scheduler_stream():
        m = ce.Multi(rs, L, 4, 2, [0, 0])
        for it in range(6):
            n = 9 + it
            full, dig_ref = _parts(d, p, L, n, 700 + it)
            src = np.ascontiguousarray(full[:, :d])
            par = np.zeros((n, p, L), np.uint8)
            dg = np.zeros((n, t, 32), np.uint8)
            m.wait(m.encode_hash(src, n, par, dg))
            assert np.array_equal(par, full[:, d:]) and np.array_equal(dg, dig_ref), it

    def per_call(i):
        def run():
            src = np.random.default_rng(900 + i).integers(0, 256, d * L, dtype=np.uint8)
            _, ref, _ = oracle.part_encode(d, p, src, d * L)
            for _ in range(3):
                ep = ce.part_encode(rs, src.tobytes(), d * L)
                assert b"".join(ep.parity) == np.asarray(ref).tobytes(), i
        return run

    def pipeline_reads():
        rp = ce.ReadPipeline(rs, L, 6, 2, 0)
        full, dig_ref = _parts(d, p, L, 6, 800)
        for it in range(6):
            slot, chunks, present, expected = rp.acquire()
            chunks[:] = full
            expected[:] = dig_ref
            present[:] = 0
            for k in range(6):
                present[k, [(k + it + j) % t for j in range(d)]] = 1
            rp.submit(slot, 6)
            _, _, st = rp.wait(slot)
            assert not any(st), it
            for k in range(6):
                assert rp.part_bytes(slot, 6, k) == full[k, :d].tobytes(), (it, k)

    ths = [threading.Thread(target=guard(scheduler_stream, "scheduler"))]
    ths += [threading.Thread(target=guard(per_call(i), f"per-call {i}")) for i in range(24)]
    args = types.SimpleNamespace(iters=4)
    ths += [threading.Thread(target=srb.worker, args=(100 + i, args, errors)) for i in range(6)]
    ths += [threading.Thread(target=guard(pipeline_reads, "read pipeline"))]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=150)
    assert not any(th.is_alive() for th in ths), "a tier never finished"
    assert not errors, errors
