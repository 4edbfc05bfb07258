"""GPU tests of the multi-GPU part scheduler (cec_multi_*), the zero-copy paths for
page-locked caller buffers (cec_host_alloc, *_submit_from, per-call DMA), and the library's
behaviour in a long-running multi-threaded host (pooled staging, bounded caches).

Everything runs through the C-ABI and is compared bit for bit with the oracle / hashlib.
"""
import hashlib
import os
import socket

import numpy as np
import pytest

import oracle
from _gen import gen_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import chunky_ec as ce  # noqa: E402

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)


def _write_inputs(n, d, L, seed):
    return gen_bytes(seed, n * d * L).reshape(n, d, L)


def _check_write(data, parity, digests, d, p):
    for k in range(data.shape[0]):
        st, par = oracle.encode_sep(d, p, [data[k, j] for j in range(d)])
        assert st == 0
        for i in range(p):
            assert np.array_equal(parity[k, i], par[i]), (k, i)
        chunks = [data[k, j] for j in range(d)] + par
        for j in range(d + p):
            assert digests[k, j].tobytes() == hashlib.sha256(chunks[j].tobytes()).digest(), (k, j)


def _device_lists():
    n = torch.cuda.device_count()
    lists = [list(range(n)), [0, 0]]  # every visible device; a forced 2-shard split on one
    if n > 1:
        lists.append([n - 1, 0, n - 1])
    return lists


# ----------------------------------------------------------------------------------------------
# Multi-GPU scheduler: write
# ----------------------------------------------------------------------------------------------

@pytest.mark.parametrize("devices", _device_lists())
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("d,p,L,n,ppb", [(10, 4, 4096, 37, 4), (3, 2, 683, 11, 3),
                                         (20, 8, 1024, 9, 2)])
def test_multi_encode_hash_vs_oracle(devices, pinned, d, p, L, n, ppb):
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, ppb, 3, devices)
    assert m.shards() == len(devices)
    src = _write_inputs(n, d, L, 100 * d + L)
    if pinned:
        hb = [ce.HostBuffer(n * d * L, devices[0]), ce.HostBuffer(n * p * L),
              ce.HostBuffer(n * (d + p) * 32)]
        data, parity, dig = hb[0].view(n, d, L), hb[1].view(n, p, L), hb[2].view(n, d + p, 32)
        assert ce.host_is_pinned(hb[0]) and ce.host_is_pinned(hb[1])
    else:
        data = np.empty((n, d, L), np.uint8)
        parity = np.zeros((n, p, L), np.uint8)
        dig = np.zeros((n, d + p, 32), np.uint8)
        assert not ce.host_is_pinned(data)
    data[:] = src
    # two jobs in flight, then a third reusing the first's buffers after its wait
    j1 = m.encode_hash(data, n, parity, dig)
    half = n // 2
    par2 = np.zeros((half, p, L), np.uint8)
    dig2 = np.zeros((half, d + p, 32), np.uint8)
    j2 = m.encode_hash(data[n - half:], half, par2, dig2)
    m.wait(j1)
    m.wait(j2)
    _check_write(src, parity, dig, d, p)
    _check_write(src[n - half:], par2, dig2, d, p)
    # contiguous ranges: shard g processed n*(g+1)//G - n*g//G parts of each job
    G = len(devices)
    for g in range(G):
        dev, numa, parts = m.shard_info(g)
        assert dev == devices[g]
        want = (n * (g + 1) // G - n * g // G) + (half * (g + 1) // G - half * g // G)
        assert parts == want


def test_multi_empty_and_tiny_jobs():
    d, p, L = 4, 2, 256
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, 2, 2, [0, 0, 0])
    m.encode_hash_sync(np.zeros((1, d, L), np.uint8), 0, np.zeros(1, np.uint8),
                       np.zeros(1, np.uint8))
    # fewer parts than shards: some shards get an empty range
    src = _write_inputs(2, d, L, 5)
    par = np.zeros((2, p, L), np.uint8)
    dig = np.zeros((2, d + p, 32), np.uint8)
    m.encode_hash_sync(src.copy(), 2, par, dig)
    _check_write(src, par, dig, d, p)


# ----------------------------------------------------------------------------------------------
# Multi-GPU scheduler: read (read_with_context compute)
# ----------------------------------------------------------------------------------------------

def _read_case(n, d, p, L, seed):
    """Encoded parts, loaded sets like file_part.rs:97 (d random of d+p, or more, or fewer), a
    few corrupted loaded chunks; expected statuses from the oracle's rules."""
    t = d + p
    rng = np.random.default_rng(seed)
    data = _write_inputs(n, d, L, seed)
    chunks = np.zeros((n, t, L), np.uint8)
    expected = np.zeros((n, t, 32), np.uint8)
    present = np.zeros((n, t), np.uint8)
    ok = np.zeros((n, t), np.uint8)
    for k in range(n):
        st, par = oracle.encode_sep(d, p, [data[k, j] for j in range(d)])
        full = [data[k, j] for j in range(d)] + par
        for i in range(t):
            chunks[k, i] = full[i]
            expected[k, i] = np.frombuffer(hashlib.sha256(full[i].tobytes()).digest(), np.uint8)
        kind = k % 6
        size = {0: t, 1: d, 2: d - 1, 3: d + 1, 4: d, 5: d + 1}[kind]
        loaded = rng.choice(t, size, replace=False)
        present[k, loaded] = 1 if kind != 5 else 0xFF  # any nonzero flag means loaded
        ok[k] = present[k] != 0
        if kind in (3, 4):  # corrupt one loaded chunk
            victim = int(loaded[0])
            chunks[k, victim, L // 3] ^= 0x44
            ok[k, victim] = 0
        for i in range(t):
            if not present[k, i]:
                chunks[k, i] = 0
    status = [0 if ok[k].sum() >= d else 10 for k in range(n)]
    return data, chunks, present, expected, ok, status


@pytest.mark.parametrize("devices", _device_lists())
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("rebuilt_only", [False, True])
def test_multi_read_vs_oracle(devices, pinned, rebuilt_only):
    d, p, L, n = 10, 4, 2048, 30
    t = d + p
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, 4, 2, devices)
    data, chunks, present, expected, ok, status = _read_case(n, d, p, L, 77)
    if pinned:
        hb = [ce.HostBuffer(n * t * L), ce.HostBuffer(n * d * L)]
        ch, out = hb[0].view(n, t, L), hb[1].view(n, d, L)
        ch[:] = chunks
        out[:] = 0
    else:
        ch, out = chunks.copy(), np.zeros((n, d, L), np.uint8)
    ver = np.zeros((n, t), np.uint8)
    st = np.zeros(n, np.int32)
    ptrs = m.read_sync(ch, present, expected, n, out, ver, st, rebuilt_only)
    assert list(st) == status
    assert np.array_equal(ver, ok)
    for k in range(n):
        if status[k]:
            if not pinned:  # went through the scheduler's reused staging: no dangling pointers
                assert all(ptrs[k * d + j] == 0 for j in range(d)), k
            continue
        got = b"".join(__import__("ctypes").string_at(ptrs[k * d + j], L) for j in range(d))
        assert got == data[k].tobytes(), k
        if not rebuilt_only:
            assert np.array_equal(out[k], data[k]), k


# ----------------------------------------------------------------------------------------------
# world-size-2 gloo: two ranks on cuda:0, each drives the HIP path for its own part range
# ----------------------------------------------------------------------------------------------

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_worker(rank, world, port, n_parts, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for pth in (root, os.path.join(root, "chunky-bits_amd"), os.path.join(root, "tests")):
        if pth not in sys.path:
            sys.path.insert(0, pth)
    import torch
    import torch.distributed as dist
    import chunky_ec as ce
    from chunky_ec.sharding import barrier, max_over_ranks, part_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        d, p, L = 10, 4, 4096
        t = d + p
        lo, hi = part_range(n_parts, rank, world)
        buf = torch.zeros((hi - lo, t, L), dtype=torch.uint8, device="cuda:0")
        batch = ce.PartBatch.from_tensor(buf, L)
        host = np.stack([gen_bytes(20_000 + k, d * L).reshape(d, L) for k in range(lo, hi)])
        buf[:, :d].copy_(torch.from_numpy(host))
        dig = torch.zeros((hi - lo, t, 32), dtype=torch.uint8, device="cuda:0")
        rs = ce.ReedSolomon(d, p)
        barrier(world)
        ce.encode_hash_batch(rs, batch, dig.data_ptr())
        torch.cuda.synchronize()
        barrier(world)
        el = max_over_ranks(float(rank + 1), world, None)
        out_q.put((rank, lo, hi, el, buf[:, d:].cpu().numpy(), dig.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_drives_hip_path_vs_oracle():
    import torch.multiprocessing as mp
    world, n_parts = 2, 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, n_parts, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    results = [q.get(timeout=180) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    covered = []
    d, p, L = 10, 4, 4096
    for rank, lo, hi, el, parity, dig in results:
        assert el == 2.0  # max over ranks
        covered.extend(range(lo, hi))
        for k in range(lo, hi):
            data = gen_bytes(20_000 + k, d * L).reshape(d, L)
            st, par = oracle.encode_sep(d, p, list(data))
            for i in range(p):
                assert np.array_equal(parity[k - lo, i], par[i]), (rank, k, i)
            chunks = list(data) + par
            for j in range(d + p):
                assert dig[k - lo, j].tobytes() == hashlib.sha256(chunks[j].tobytes()).digest()
    assert sorted(covered) == list(range(n_parts))


# ----------------------------------------------------------------------------------------------
# Zero-copy pipelines and per-call DMA
# ----------------------------------------------------------------------------------------------

def test_pipeline_submit_from_pinned_and_pageable():
    d, p, L, P = 10, 4, 4096, 6
    rs = ce.ReedSolomon(d, p)
    pl = ce.Pipeline(rs, L, P, 2, ce.PIPE_EXTERNAL)
    src = _write_inputs(P, d, L, 9)
    hin, hpar = ce.HostBuffer(P * d * L), ce.HostBuffer(P * p * L)
    hin.view(P, d, L)[:] = src
    dig = np.zeros((P, d + p, 32), np.uint8)
    s0, _ = pl.acquire()
    pl.submit_from(s0, hin.view(P, d, L), P, hpar.view(P, p, L), dig)
    par_a, dig_a = pl.wait(s0)
    _check_write(src, hpar.view(P, p, L), dig, d, p)
    s1, _ = pl.acquire()
    pageable = src.copy()
    par2 = np.zeros((P, p, L), np.uint8)
    pl.submit_from(s1, pageable, P, par2, None)  # digests into the slot's own buffer
    _, dig_b = pl.wait(s1)
    _check_write(src, par2, dig_b, d, p)


def test_per_call_mixed_pinned_and_pageable_callers_bit_exact():
    """cec_part_encode from page-locked buffers (DMA'd directly) and from pageable ones (staged)
    in the same coalesced batches: every caller gets its own part's parity and digests."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    d, p = 10, 4
    rs = ce.ReedSolomon(d, p)
    L = 65536

    def task(i):
        src = gen_bytes(7000 + i, d * L)
        if i % 2:
            hb_in, hb_out = ce.HostBuffer(d * L), ce.HostBuffer(p * L)
            data, par = hb_in.array, hb_out.array
            data[:] = src
        else:
            data, par = src.copy(), np.zeros(p * L, np.uint8)
        dig = (ctypes.c_uint8 * (32 * (d + p)))()
        cs = ctypes.c_size_t(0)
        code = ce._lib.cec_part_encode(rs.handle, ctypes.cast(ce._addr(data), ce._u8p), d * L,
                                       ctypes.cast(ce._addr(par), ce._u8p), dig, ctypes.byref(cs))
        assert code == 0
        _, ref, rdig = oracle.part_encode(d, p, src, d * L)
        assert np.array_equal(par.reshape(p, L), np.stack(ref)), i
        assert bytes(dig) == b"".join(x.tobytes() for x in rdig), i
        return i

    c0, l0 = ce.coalesce_stats()
    with ThreadPoolExecutor(max_workers=24) as ex:
        assert sorted(ex.map(task, range(48))) == list(range(48))
    c1, l1 = ce.coalesce_stats()
    assert l1 - l0 < c1 - c0


def _overflow_callers_child():
    """Run in a child with a small CEC_COALESCE_MAX_MIB: 48 pageable callers x 4 calls, so
    nearly every batch overflows the cap and two batches are in flight over and over."""
    from concurrent.futures import ThreadPoolExecutor
    d, p, L = 10, 4, 65536
    rs = ce.ReedSolomon(d, p)

    def task(i):
        src = gen_bytes(9000 + i, d * L)
        _, ref, rdig = oracle.part_encode(d, p, src, d * L)
        for _ in range(4):
            ep = ce.part_encode(rs, src.tobytes(), d * L)
            assert b"".join(ep.parity) == np.asarray(ref).tobytes(), i
            assert [str(h) for h in ep.hashes] == [bytes(x).hex() for x in np.asarray(rdig)], i
        return i

    c0, l0 = ce.coalesce_stats()
    with ThreadPoolExecutor(max_workers=48) as ex:
        assert sorted(ex.map(task, range(48))) == list(range(48))
    c1, l1 = ce.coalesce_stats()
    assert c1 - c0 == 192 and l1 - l0 > 192 // 8


def _mixed_keys_child():
    """Child with a small batch cap: callers of three coalescing keys at once (RS(10,4) at
    64 KiB chunks, RS(3,2) at 683-byte chunks, and plain SHA-256 of odd lengths), so batches of
    one key overflow while callers of the others wait behind them."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    codecs = {(10, 4): ce.ReedSolomon(10, 4), (3, 2): ce.ReedSolomon(3, 2)}

    def task(i):
        kind = i % 3
        for it in range(3):
            if kind == 2:
                buf = gen_bytes(11000 + 7 * i + it, 1000 + 37 * i)
                h = ce.Sha256Hash.from_buf(buf.tobytes())
                assert str(h) == hashlib.sha256(buf.tobytes()).hexdigest(), i
                continue
            d, p, L = (10, 4, 65536) if kind == 0 else (3, 2, 683)
            src = gen_bytes(12000 + 7 * i + it, d * L)
            ep = ce.part_encode(codecs[(d, p)], src.tobytes(), d * L)
            _, ref, rdig = oracle.part_encode(d, p, src, d * L)
            assert b"".join(ep.parity) == np.asarray(ref).tobytes(), i
            assert [str(h) for h in ep.hashes] == [bytes(x).hex() for x in np.asarray(rdig)], i
        return i

    with ThreadPoolExecutor(max_workers=60) as ex:
        assert sorted(ex.map(task, range(60))) == list(range(60))


def test_per_call_mixed_keys_under_overflow():
    """Three coalescing keys at once under a 1 MiB batch cap (child process): every caller
    finishes with its own bit-exact result."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path.insert(0, %r); import conftest, torch, test_gpu_multi as m; "
            "m._mixed_keys_child(); print('ok')" % here)
    env = dict(os.environ, CEC_COALESCE_MAX_MIB="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_per_call_two_batches_in_flight_never_strand_a_caller():
    """Regression: with two batches in flight (the overflow rule), a caller already taken into
    a batch that was woken before the batch formed once led a batch of its own, so its first
    leader waited forever for its copy-in (percall_bench, 256 pageable callers).  A child
    process with a 2 MiB batch cap overflows on nearly every batch; it must finish, bit-exact."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path.insert(0, %r); import conftest, torch, test_gpu_multi as m; "
            "m._overflow_callers_child(); print('ok')" % here)
    env = dict(os.environ, CEC_COALESCE_MAX_MIB="2")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


# ----------------------------------------------------------------------------------------------
# Long-running host: pooled staging, no per-thread leaks, product build ignores A/B modes
# ----------------------------------------------------------------------------------------------

def test_many_short_lived_threads_do_not_leak_device_memory():
    """Tokio's blocking pool retires threads; 200 short-lived threads that each call the
    per-call entry points must leave device memory where it was (pooled staging)."""
    import threading
    d, p, L = 10, 4, 8192
    rs = ce.ReedSolomon(d, p)
    src = gen_bytes(1, d * L).tobytes()

    def body():
        ce.Sha256Hash.from_buf(src[:1000])
        ce.part_encode(rs, src, d * L)
        shards = [bytearray(src[j * L:(j + 1) * L]) for j in range(d)] + [None] * p
        rs.reconstruct(shards)  # rebuilds parity: per-call staging context
        rs.encode_sep([src[j * L:(j + 1) * L] for j in range(d)], [bytearray(L) for _ in range(p)])

    def wave(n):
        ths = [threading.Thread(target=body) for _ in range(n)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        torch.cuda.synchronize()

    wave(200)  # warm: pools and coalescing arenas reach their steady size
    free0, _ = torch.cuda.mem_get_info()
    wave(200)
    wave(200)
    free1, _ = torch.cuda.mem_get_info()
    # A per-thread leak costs >= 1 MiB of staging per retired thread: >= 400 MiB over these 400
    # threads.  What may still grow is bounded and timing-dependent: a coalescing arena whose
    # batch gathered more callers than in the warm-up wave (<= 200 parts x 14 x 8 KiB ~ 22 MiB,
    # in 1 MiB steps; one repeat run saw +2 MiB) and scratch buffers for a higher peak of
    # concurrent launches (64 KiB each).
    assert free0 - free1 <= (32 << 20), (free0 - free1)


def test_product_build_ignores_attribution_modes(knob_env):
    assert "ab_tools=0" in ce.build_info()
    d, p, L, n = 10, 4, 4096, 20
    for knob, val in [("CEC_FUSED_MODE", "1"), ("CEC_FUSED_MODE", "2"), ("CEC_SHA_VARIANT", "7"),
                      ("CEC_SHA_VARIANT", "8")]:
        knob_env.set(knob, val)
        knob_env.set("CEC_FUSED", "1")
        buf = torch.zeros((n, d + p, L), dtype=torch.uint8, device="cuda:0")
        batch = ce.PartBatch.from_tensor(buf, L)
        ce.fill_synthetic(batch, d, 3)
        dig = torch.zeros((n, d + p, 32), dtype=torch.uint8, device="cuda:0")
        ce.encode_hash_batch(ce.ReedSolomon(d, p), batch, dig.data_ptr())
        torch.cuda.synchronize()
        host, hd = buf.cpu().numpy(), dig.cpu().numpy()
        _check_write(host[:, :d], host[:, d:], hd, d, p)
        knob_env.delenv(knob)


def test_decode_cache_is_bounded_lru():
    d, p, L = 20, 8, 16
    rs = ce.ReedSolomon(d, p)
    full = [bytes([i]) * L for i in range(d + p)]
    rng = np.random.default_rng(3)
    seen = set()
    while len(seen) < 4200:
        miss = tuple(sorted(rng.choice(d + p, 4, replace=False).tolist()))
        if miss in seen:
            continue
        seen.add(miss)
        shards = [None if i in miss else bytearray(full[i]) for i in range(d + p)]
        rs.reconstruct(shards)
    assert rs.cached_patterns() == 4096


# ----------------------------------------------------------------------------------------------
# Read retry (file_part.rs:92-107): resubmit just the undecodable parts with more chunks
# ----------------------------------------------------------------------------------------------

def test_read_retry_with_one_more_chunk_vs_oracle():
    """Exactly d chunks loaded, one of them corrupt -> TooFewShardsPresent; the caller loads one
    more chunk for just those parts and resubmits, marking the chunks that verified
    CEC_PRESENT_VERIFIED (not hashed again): the part then decodes bit-exact."""
    d, p, L, n = 10, 4, 4096 + 16, 8
    t = d + p
    rs = ce.ReedSolomon(d, p)
    buf = torch.zeros((n, t, L), dtype=torch.uint8, device="cuda:0")
    batch = ce.PartBatch.from_tensor(buf, L)
    ce.fill_synthetic(batch, d, 99)
    dig = torch.zeros((n, t, 32), dtype=torch.uint8, device="cuda:0")
    ce.encode_hash_batch(rs, batch, dig.data_ptr())
    torch.cuda.synchronize()
    ref = buf.cpu().numpy().copy()
    rng = np.random.default_rng(12)
    present = np.zeros((n, t), np.uint8)
    unloaded = {}
    for k in range(n):
        loaded = rng.choice(t, d, replace=False)
        present[k, loaded] = 1
        unloaded[k] = [i for i in range(t) if not present[k, i]]
    host = ref.copy()
    host[present == 0] = 0
    bad = [1, 4, 6]
    for k in bad:  # one corrupt loaded chunk: d - 1 verify
        i = int(np.flatnonzero(present[k])[3])
        host[k, i, 5] ^= 0x80
    buf.copy_(torch.from_numpy(host))
    verified, status = ce.read_batch(rs, batch, present.tobytes(), dig.data_ptr())
    v = np.frombuffer(verified, np.uint8).reshape(n, t)
    assert [k for k in range(n) if status[k] != ce.OK] == bad
    # retry just the failed parts: verified chunks marked 2, one more chunk loaded (1)
    sub = torch.zeros((len(bad), t, L), dtype=torch.uint8, device="cuda:0")
    sub_dig = dig[bad].contiguous()
    pres2 = np.zeros((len(bad), t), np.uint8)
    sub_host = np.zeros((len(bad), t, L), np.uint8)
    for q, k in enumerate(bad):
        for i in range(t):
            if v[k, i]:
                pres2[q, i] = ce.PRESENT_VERIFIED
                sub_host[q, i] = host[k, i]
        extra = unloaded[k][0]
        pres2[q, extra] = 1
        sub_host[q, extra] = ref[k, extra]
    sub.copy_(torch.from_numpy(sub_host))
    sub_batch = ce.PartBatch.from_tensor(sub, L)
    verified2, status2 = ce.read_batch(rs, sub_batch, pres2.tobytes(), sub_dig.data_ptr())
    torch.cuda.synchronize()
    assert status2 == [ce.OK] * len(bad)
    v2 = np.frombuffer(verified2, np.uint8).reshape(len(bad), t)
    got = sub.cpu().numpy()
    for q, k in enumerate(bad):
        assert np.array_equal(v2[q], (pres2[q] != 0).astype(np.uint8))
        shards = [ref[k, i] if v2[q, i] else None for i in range(t)]
        st, out = oracle.reconstruct(d, p, shards, data_only=True)
        assert st == 0
        for j in range(d):
            assert np.array_equal(got[q, j], out[j]) and np.array_equal(got[q, j], ref[k, j])


def test_multi_read_retry_pass():
    d, p, L, n = 6, 3, 1024, 12
    t = d + p
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, 3, 2, [0, 0])
    data = _write_inputs(n, d, L, 31)
    chunks = np.zeros((n, t, L), np.uint8)
    expected = np.zeros((n, t, 32), np.uint8)
    for k in range(n):
        st, par = oracle.encode_sep(d, p, [data[k, j] for j in range(d)])
        full = [data[k, j] for j in range(d)] + par
        for i in range(t):
            chunks[k, i] = full[i]
            expected[k, i] = np.frombuffer(hashlib.sha256(full[i].tobytes()).digest(), np.uint8)
    good = chunks.copy()
    present = np.zeros((n, t), np.uint8)
    present[:, :d] = 1  # the data chunks first
    for k in range(0, n, 3):
        chunks[k, 2, 0] ^= 1  # corrupt: that part needs one more chunk
    out = np.zeros((n, d, L), np.uint8)
    ver = np.zeros((n, t), np.uint8)
    st = np.zeros(n, np.int32)
    m.read_sync(chunks, present, expected, n, out, ver, st)
    failed = [k for k in range(n) if st[k]]
    assert failed == list(range(0, n, 3))
    f = len(failed)
    ch2 = np.zeros((f, t, L), np.uint8)
    pr2 = np.zeros((f, t), np.uint8)
    for q, k in enumerate(failed):
        pr2[q] = np.where(ver[k] != 0, ce.PRESENT_VERIFIED, 0)
        ch2[q] = np.where(ver[k][:, None] != 0, chunks[k], 0)
        pr2[q, d] = 1
        ch2[q, d] = good[k, d]
    out2 = np.zeros((f, d, L), np.uint8)
    ver2 = np.zeros((f, t), np.uint8)
    st2 = np.zeros(f, np.int32)
    m.read_sync(ch2, pr2, expected[failed].copy(), f, out2, ver2, st2)
    assert list(st2) == [0] * f
    for q, k in enumerate(failed):
        assert np.array_equal(out2[q], data[k])
    for k in range(n):
        if k not in failed:
            assert np.array_equal(out[k], data[k])


def test_multi_many_tiny_jobs_fewer_parts_than_shards():
    """Jobs smaller than the shard count leave some shards without a range: those never see the
    job, so a caller may free it as soon as it completes (no shard touches it afterwards)."""
    d, p, L = 4, 2, 512
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, 2, 2, [0, 0, 0, 0])
    for it in range(150):
        n = 1 + it % 3
        src = _write_inputs(n, d, L, 40_000 + it)
        par = np.zeros((n, p, L), np.uint8)
        dig = np.zeros((n, d + p, 32), np.uint8)
        m.encode_hash_sync(src.copy(), n, par, dig)
        if it % 25 == 0:
            _check_write(src, par, dig, d, p)
    with pytest.raises(ce.Error):
        m.wait(123456789)  # unknown job


def test_multi_freed_with_jobs_in_flight_finishes_them():
    """Destroying the scheduler with jobs still queued completes them first (their buffers are
    the caller's until then)."""
    d, p, L, n = 10, 4, 4096, 12
    rs = ce.ReedSolomon(d, p)
    src = _write_inputs(n, d, L, 77)
    par = np.zeros((n, p, L), np.uint8)
    dig = np.zeros((n, d + p, 32), np.uint8)
    m = ce.Multi(rs, L, 2, 2, [0, 0])
    m.encode_hash(src.copy(), n, par, dig)
    del m
    import gc
    gc.collect()
    _check_write(src, par, dig, d, p)


# ----------------------------------------------------------------------------------------------
# Resilver / verify through the scheduler (FilePart::resilver / verify compute)
# ----------------------------------------------------------------------------------------------

@pytest.mark.parametrize("devices", _device_lists())
@pytest.mark.parametrize("pinned", [False, True])
def test_multi_resilver_and_verify_vs_oracle(devices, pinned):
    """file_part.rs:253-308: every chunk that is missing or fails its hash is rebuilt (data AND
    parity) from the verified ones; file_part.rs:228-251: verify reports every loaded chunk."""
    d, p, L, n = 6, 3, 1536, 26
    t = d + p
    rs = ce.ReedSolomon(d, p)
    m = ce.Multi(rs, L, 3, 2, devices)
    data, chunks, present, expected, ok, status = _read_case(n, d, p, L, 91)
    full = np.zeros((n, t, L), np.uint8)
    for k in range(n):
        st, par = oracle.encode_sep(d, p, [data[k, j] for j in range(d)])
        full[k, :d] = data[k]
        full[k, d:] = np.stack(par)
    if pinned:
        hb = [ce.HostBuffer(n * t * L), ce.HostBuffer(n * t * L)]
        ch, rebuilt = hb[0].view(n, t, L), hb[1].view(n, t, L)
        ch[:] = chunks
        rebuilt[:] = 0
    else:
        ch, rebuilt = chunks.copy(), np.zeros((n, t, L), np.uint8)
    ver = np.zeros((n, t), np.uint8)
    st = np.zeros(n, np.int32)
    ptrs = m.resilver_sync(ch, present, expected, n, rebuilt, ver, st)
    assert list(st) == status
    assert np.array_equal(ver, ok)
    import ctypes
    for k in range(n):
        if status[k]:
            continue
        for i in range(t):
            got = ctypes.string_at(ptrs[k * t + i], L)
            assert got == full[k, i].tobytes(), (k, i)  # every chunk, verified or rebuilt
            if not ok[k, i]:
                assert np.array_equal(rebuilt[k, i], full[k, i]), (k, i)
    ver2 = np.zeros((n, t), np.uint8)
    m.verify_sync(ch, present, expected, n, ver2)
    assert np.array_equal(ver2, ok)


def test_read_pipeline_resilver_flag_vs_oracle():
    d, p, L, P = 4, 3, 2048 + 16, 10
    t = d + p
    rs = ce.ReedSolomon(d, p)
    rp = ce.ReadPipeline(rs, L, P, 2, ce.READ_RESILVER)
    data, chunks, present, expected, ok, status = _read_case(P, d, p, L, 13)
    slot, c, pr, ex = rp.acquire()
    c[:] = chunks
    pr[:] = present
    ex[:] = expected
    rp.submit(slot, P)
    out, ver, stt = rp.wait(slot)
    assert list(stt) == status
    assert np.array_equal(ver, ok)
    import ctypes
    ptrs = (ctypes.c_void_p * (P * t))()
    assert ce._lib.cec_read_pipeline_data_chunks(rp._h, slot, ptrs, len(ptrs)) == 0
    for k in range(P):
        if status[k]:
            continue
        st, par = oracle.encode_sep(d, p, [data[k, j] for j in range(d)])
        want = [data[k, j] for j in range(d)] + par
        for i in range(t):
            assert ctypes.string_at(ptrs[k * t + i], L) == want[i].tobytes(), (k, i)


# ----------------------------------------------------------------------------------------------
# HostBuffer views keep their page-locked memory alive
# ----------------------------------------------------------------------------------------------

def test_host_buffer_view_outlives_its_owner():
    """A view of a HostBuffer that was dropped keeps the buffer (and its page-locked memory)
    alive; the memory is freed only once the last view is gone.  Used to be a use-after-free:
    the view's base was a bare ctypes pointer."""
    import gc
    import weakref
    n = 1 << 20
    hb = ce.HostBuffer(n)
    owner = weakref.ref(hb)
    v = hb.view(256, 4096)
    v2 = ce.HostBuffer(n).array  # a temporary: only its view is kept
    del hb
    gc.collect()
    assert owner() is not None
    assert ce.host_is_pinned(v) and ce.host_is_pinned(v2)
    v[:] = 7
    v2[:] = 9
    others = [ce.HostBuffer(n) for _ in range(4)]  # would reuse freed pinned pages
    for o in others:
        o.array[:] = 0
    assert int(v.min()) == int(v.max()) == 7 and int(v2.min()) == int(v2.max()) == 9
    # the engine DMAs it: the buffer's bytes go through a per-call SHA-256
    assert str(ce.Sha256Hash.from_buf(v)) == hashlib.sha256(bytes(v)).hexdigest()
    del v
    gc.collect()
    assert owner() is None
