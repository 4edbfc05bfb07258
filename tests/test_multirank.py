"""N > 1 path on CPU: two gloo ranks shard parts with chunky_ec.sharding exactly as bench.py
does, compute their parts independently (oracle, since there is no GPU here), and the union of
the per-rank results equals the single-process result; the max-over-ranks step time and the
barrier behave as the bench needs."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from chunky_ec.sharding import part_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _part_digests(part, d, p, L):
    import hashlib
    import oracle
    from _gen import gen_bytes
    data = gen_bytes(10_000 + part, d * L).reshape(d, L)
    st, par = oracle.encode_sep(d, p, list(data))
    assert st == 0
    chunks = [x.tobytes() for x in data] + [x.tobytes() for x in par]
    return [hashlib.sha256(c).hexdigest() for c in chunks]


def _worker(rank, world, port, n_parts, out_q):
    import torch
    import torch.distributed as dist
    from chunky_ec.sharding import all_ranks_ok, barrier, gather_rows, max_over_ranks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = part_range(n_parts, rank, world)
        res = {k: _part_digests(k, 3, 2, 257) for k in range(lo, hi)}
        barrier(world)
        t = max_over_ranks(float(rank + 1) * 0.5, world, torch.device("cpu"))
        # bench.py's optional end-to-end step: skipped on every rank when one rank cannot run it
        ok_all = all_ranks_ok(True, world)
        ok_one_fails = all_ranks_ok(rank != world - 1, world)
        # bench.py's per-rank array: each rank's own row, in rank order, on every rank
        rows = gather_rows([rank, 10.0 * rank + 0.5, hi - lo], world)
        # bench.py's N > 1 line: each rank's C3 / C4 figures in the RANK_FIELDS row, the node's
        # configs[2] / configs[3] figures computed from the gathered rows on every rank
        import bench
        from chunky_ec.sharding import multi_copy_threads, quota_share, rank_threads
        row = [rank, 0, 1, 8, 40.0, 50.0, 55.0, 0.8, 0.74, 0.7 + 0.01 * rank, 1e9 * (rank + 1),
               5.0 + rank, 10.0 + rank, (rank + 1) * 1e9, 30.0,
               quota_share(world) or 0.0, rank_threads(world), multi_copy_threads(world)]
        ranks = [bench.rank_row(r, x) for r, x in enumerate(gather_rows(row, world))]
        node = bench.node_figures(ranks)
        node["rank_rows"] = ranks
        gathered = [None] * world
        dist.all_gather_object(gathered, res)
        out_q.put((rank, t, gathered, ok_all, ok_one_fails, rows, node))
    finally:
        dist.destroy_process_group()


def test_part_range_partitions_exactly():
    for n in (0, 1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = part_range(n, r, world)
                assert lo <= hi
                seen.extend(range(lo, hi))
            assert seen == list(range(n))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_sharding_matches_single_process(world):
    """World sizes 2, 4 and 8 (the driver's 1/2/4/8-GPU runs use the same helpers over RCCL)."""
    n_parts = 9 if world == 2 else 19  # 19 over 8 ranks: ragged ranges (2 or 3 parts each)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_parts, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    single = {k: _part_digests(k, 3, 2, 257) for k in range(n_parts)}
    for rank, t, gathered, ok_all, ok_one_fails, rows, node in results:
        # node C4 = all ranks' data over the slowest rank's time; C3 min frac = rank 0's
        c4 = node["c4_encode_hash"]
        assert c4["data_bytes"] == sum((r + 1) * 1e9 for r in range(world))
        assert c4["max_ms"] == 10.0 + world - 1
        assert c4["value"] == round(c4["data_bytes"] / ((10.0 + world - 1) / 1e3) / 1e9, 2)
        assert node["c3_reconstruct"]["min_frac"] == 0.7 and node["ranks"] == world
        # every rank reports the host threads it used and its share of the job's CPU quota
        from chunky_ec.sharding import cpu_quota
        quota = cpu_quota()[1]
        for row in node["rank_rows"]:
            assert row["host_threads"] >= 1 and row["multi_copy_threads"] >= 1
            if quota:
                assert row["quota_share_cpus"] == pytest.approx(quota / world, rel=1e-3)
                assert row["host_threads"] <= max(1, int(quota / world) - 1)
        assert t == pytest.approx(0.5 * world)  # max over ranks of (rank+1)*0.5
        assert ok_all and not ok_one_fails
        assert rows == [[float(r), 10.0 * r + 0.5,
                         float(part_range(n_parts, r, world)[1] - part_range(n_parts, r, world)[0])]
                        for r in range(world)]
        merged = {}
        for part_map in gathered:
            assert not (set(merged) & set(part_map))  # disjoint ownership
            merged.update(part_map)
        assert merged == single


def _single_pg_worker(port, out_q):
    import torch.distributed as dist
    from chunky_ec import sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    before = sharding.collective(1)
    dist.init_process_group("gloo", rank=0, world_size=1)
    calls = []
    real = dist.all_reduce
    dist.all_reduce = lambda *a, **k: (calls.append(1), real(*a, **k))[1]
    try:
        out_q.put((before, sharding.collective(1), sharding.max_over_ranks(2.5, 1),
                   sharding.gather_rows([1, 2], 1), sharding.all_ranks_ok(True, 1), len(calls)))
        sharding.barrier(1)
    finally:
        dist.all_reduce = real
        dist.destroy_process_group()


def test_world1_process_group_takes_collective_path():
    """bench.py's CEC_BENCH_PG=1 rehearsal: with a process group at world 1 the rank helpers go
    through torch.distributed (3 all-reduces), with the same results as without one."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_single_pg_worker, args=(_free_port(), q))
    pr.start()
    res = q.get(timeout=120)
    pr.join(60)
    assert pr.exitcode == 0
    assert res == (False, True, 2.5, [[1.0, 2.0]], True, 3)
