"""bench.py's host-side logic on the CPU: the end-to-end forms' source ring and copy threads,
the erasure sets of north_star's reconstruct case, and the host / CPU-quota report."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

bench = pytest.importorskip("bench")


def test_host_copier_copies_every_part_exactly():
    c = bench.HostCopier(3)
    try:
        src = np.random.default_rng(1).integers(0, 256, size=(7, 3, 1000), dtype=np.uint8)
        for n in (1, 2, 3, 7):  # fewer parts than threads included
            dst = np.zeros_like(src)
            c.copy(dst[:n], src[:n])
            assert np.array_equal(dst[:n], src[:n]) and not dst[n:].any()
    finally:
        c.close()


def test_source_ring_parts_are_distinct_and_stamped():
    c = bench.HostCopier(2)
    try:
        ring = bench.source_ring(40, 3, 4096, 5, c)
    finally:
        c.close()
    assert ring.shape == (40, 3, 4096)
    idx = ring[:, 0, :8].copy().view(np.uint64).ravel()
    assert np.array_equal(idx, np.arange(40, dtype=np.uint64))
    # every part's bytes differ from every other part's (the stamp alone guarantees it)
    assert len({ring[k].tobytes() for k in range(40)}) == 40
    # beyond the stamp the content is the random block, not zeros
    assert ring[:, 1:].any()


def test_two_erasures_exactly_two_per_part_and_bytes():
    pres = bench.two_erasures(64, 14, 0)
    assert pres.shape == (64, 14)
    assert (pres.sum(1) == 12).all()
    assert bench.two_erasures(64, 14, 0).equal(pres)  # seeded: the c3e2 sets
    d, L = 10, 1 << 20
    miss = d - pres[:, :d].sum(1)
    want = int((miss > 0).sum()) * d * L + int(miss.sum()) * L
    assert bench.reconstruct_data_bytes(pres, d, L) == want


def test_c3_erasures_one_to_p_per_part_and_seeded():
    pres = bench.c3_erasures(200, 14, 4, 0)
    miss = 14 - pres.sum(1)
    assert ((miss >= 1) & (miss <= 4)).all()
    assert set(miss.tolist()) == {1, 2, 3, 4}
    assert bench.c3_erasures(200, 14, 4, 0).equal(pres)  # the c3 config's sets
    assert not bench.c3_erasures(200, 14, 4, 1).equal(pres)  # per-rank seed


def test_host_report_and_quota():
    info = bench.host_info()
    assert info["logical_cpus"] == os.cpu_count()
    assert info["affinity_cpus"] == len(os.sched_getaffinity(0))
    aff, quota = bench.cpu_quota()
    assert aff >= 1 and (quota is None or quota > 0)


def test_measured_traffic_names_its_source():
    tr, src = bench.measured_traffic("c2", "encode_hash_kernel", True, with_source=True)
    assert tr and tr > 0 and src.startswith("committed PMC run (not this run): profiles/")
    assert bench.measured_traffic("c2", "encode_hash_kernel", False, with_source=True) == \
        (None, None)


class _FakeWritePipeline:
    """cec_pipeline's slot contract on the CPU: acquire -> [P][d][L] slot, submit hashes the
    data chunks (hashlib), wait -> (parity placeholder, digests [n][d][32])."""

    def __init__(self, d, L, parts, depth):
        self.d, self.L, self.parts, self.depth = d, L, parts, depth
        self.slots = [np.zeros((parts, d, L), np.uint8) for _ in range(depth)]
        self.dig = [None] * depth
        self.next = 0
        self.seen = []

    def acquire(self):
        i = self.next
        self.next = (self.next + 1) % self.depth
        return i, self.slots[i]

    def submit(self, slot, n):
        import hashlib
        data = self.slots[slot][:n]
        self.seen.append(data[:, 0, :8].copy().view(np.uint64).ravel().tolist())
        self.dig[slot] = np.array([[np.frombuffer(hashlib.sha256(c.tobytes()).digest(), np.uint8)
                                    for c in part] for part in data])

    def wait(self, slot):
        return None, self.dig[slot]

    def drain(self):
        pass


def test_ring_reader_stream_stamps_every_part_and_checks_digests():
    c = bench.HostCopier(3)
    try:
        d, L, P, depth = 3, 512, 4, 2
        ring = bench.source_ring(5, d, L, 9, c)  # 5 ring parts: the stream wraps the ring
        pl = _FakeWritePipeline(d, L, P, depth)
        el, slot, n = bench.timed_write(pl, bench.ring_reader(ring, c), 100, 11, 1)
        assert el >= 0 and n == 11 - 2 * P
        # warmup batches first, then parts 100..110 in order, each stamped with its number
        timed = [x for batch in pl.seen[depth:] for x in batch]
        assert timed == list(range(100, 111))
        assert bench.write_check(pl, ring, slot, n, 110)
        # the check sees a wrong digest
        pl.dig[slot][0, 1, 0] ^= 1
        assert not bench.write_check(pl, ring, slot, n, 110)
        # part k's bytes are ring part k mod 5 with its stamp
        want = ring[107 % 5].copy()
        want[0, :8] = bench.part_stamps(107, 1)[0]
        import hashlib
        assert bench.ring_part_digests(ring, 107) == [hashlib.sha256(x.tobytes()).digest()
                                                      for x in want]
    finally:
        c.close()


def test_host_copier_map_covers_range_once():
    c = bench.HostCopier(4)
    try:
        seen = []
        c.map(lambda a, b: seen.extend(range(a, b)), 10)
        assert sorted(seen) == list(range(10))
        c.map(lambda a, b: seen.append((a, b)), 0)  # nothing to do
        assert len(seen) == 10
    finally:
        c.close()


def test_check_vs_oracle_catches_a_wrong_byte():
    """The default line's oracle leg on small parts: good parts pass every check; one flipped
    parity byte / digest byte / rebuilt byte fails the matching check."""
    import hashlib
    import oracle
    d, p, L = 10, 4, 1000
    rng = np.random.default_rng(3)
    parts, digs = [], []
    for _ in range(3):
        data = rng.integers(0, 256, size=(d, L), dtype=np.uint8)
        st, par = oracle.encode_sep(d, p, list(data))
        part = np.concatenate([data, np.stack(par)])
        parts.append(part)
        digs.append(np.array([np.frombuffer(hashlib.sha256(x.tobytes()).digest(), np.uint8)
                              for x in part]))
    ks = (0, 5, 9)
    snap = {"parts": ks, "headline": [(k, parts[i], digs[i]) for i, k in enumerate(ks)],
            "north_star_encode": [(k, parts[i].copy(), None) for i, k in enumerate(ks)],
            "c3_reconstruct": [(k, parts[i].copy(), None) for i, k in enumerate(ks)]}
    res = bench.check_vs_oracle(snap, d, p)
    assert res["ok"] and all(res["checks"].values())
    snap["north_star_encode"][1][1][d + 2, 7] ^= 1
    snap["c3_reconstruct"][2][1][3, 0] ^= 1
    res = bench.check_vs_oracle(snap, d, p)
    assert not res["ok"]
    assert res["checks"] == {"headline": True, "north_star_encode": False,
                             "c3_reconstruct": False}
    snap["headline"][0][2][4, 0] ^= 1
    assert not bench.check_vs_oracle(snap, d, p)["checks"]["headline"]


def test_node_figures_from_rank_rows():
    rows = [[r, 0, 1, 64, 40.0 + r, 50.0, 55.0, 0.8, 0.74, 0.74 - 0.01 * r, 4e10, 7.0 + r,
             14.0 + r, 21474836480, 40.0] for r in range(4)]
    ranks = [bench.rank_row(r, row) for r, row in enumerate(rows)]
    assert ranks[2]["c4_ms"] == 16.0 and ranks[3]["c3_reconstruct_frac"] == 0.71
    node = bench.node_figures(ranks)
    assert node["c4_encode_hash"]["data_bytes"] == 4 * 21474836480
    assert node["c4_encode_hash"]["value"] == round(4 * 21474836480 / 0.017 / 1e9, 2)
    assert node["c3_reconstruct"]["min_frac"] == 0.71
    assert node["c3_reconstruct"]["achieved"] == round(4 * 4e10 / 0.010 / 1e9, 1)
    assert node["min_north_star_encode_frac"] == 0.8
    # a rank without the blocks (0 -> None): no node figure rather than a wrong one
    rows[1][12] = 0
    assert "c4_encode_hash" not in bench.node_figures(
        [bench.rank_row(r, row) for r, row in enumerate(rows)])


def test_check_vs_oracle_whole_batch():
    """The cpu_baseline leg's whole-batch check (batch_vs_oracle, slab by slab): every part's
    parity against the oracle's encode_sep of its data and its digests against SHA-256 of its
    chunks; a single wrong digest or parity byte is reported with its part."""
    import torch

    import oracle

    def batch(rng, d, p, L, n):
        data = rng.integers(0, 256, (n, d, L), dtype=np.uint8)
        full = np.zeros((n, d + p, L), np.uint8)
        full[:, :d] = data
        for k in range(n):
            st, par = oracle.encode_sep(d, p, list(data[k]))
            full[k, d:] = np.stack(par)
        return torch.from_numpy(full), oracle.encode_hash_parts(d, p, data, 2)

    d, p, L, n = 3, 2, 512, 6
    t = d + p
    rng = np.random.default_rng(5)
    buf, dig = batch(rng, d, p, L, n)
    snap = {"parts": (0, n - 1)}
    snap["headline"] = [(k, buf[k].numpy().copy(), dig[k]) for k in snap["parts"]]
    snap["c2_digests"], snap["c2_dev"] = dig.copy(), buf
    det = bench.check_vs_oracle(snap, d, p, 2)
    assert det["ok"] and det["checks"]["c2_all_parts"]
    assert det["c2_all_parts_checked"] == {"parts": n, "digests": n * t}
    assert det["c2_all_parts_mismatched"] == []
    assert bench.batch_vs_oracle(buf, dig, d, p, 2, slab=4) == []
    snap["c2_digests"][4, t - 1, 7] ^= 1  # one parity digest of part 4
    det = bench.check_vs_oracle(snap, d, p, 2)
    assert not det["ok"] and det["c2_all_parts_mismatched"] == [4]
    snap["c2_digests"][4, t - 1, 7] ^= 1
    buf[2, d, 100] ^= 1  # a parity byte of part 2 (its digest is the oracle's, so it differs)
    buf[5, 0, 0] ^= 1  # a data byte of part 5 (parity and digest both differ)
    assert bench.batch_vs_oracle(buf, dig, d, p, 2, slab=4) == [2, 5]
    buf[2, d, 100] ^= 1
    buf[5, 0, 0] ^= 1
    # C4's buffer (the config's RS(20,8) shape), 3 small parts
    c4 = bench.CONFIGS["c4"]
    d4, p4 = c4["d"], c4["p"]
    snap["c4_dev"], snap["c4_digests"] = batch(rng, d4, p4, 256, 3)
    det = bench.check_vs_oracle(snap, d, p, 2)
    assert det["ok"] and det["checks"]["c4_all_parts"]
    assert det["c4_all_parts_checked"] == {"parts": 3, "digests": 3 * (d4 + p4)}
    snap["c4_digests"][1, 0, 0] ^= 0x80  # a data digest of part 1
    det = bench.check_vs_oracle(snap, d, p, 2)
    assert not det["ok"] and det["c4_all_parts_mismatched"] == [1]


class _OracleWritePipeline(_FakeWritePipeline):
    """The same slot contract, with the d + p digests of the oracle's encode + SHA-256."""

    def __init__(self, d, p, L, parts, depth):
        super().__init__(d, L, parts, depth)
        self.p = p

    def submit(self, slot, n):
        import oracle
        data = self.slots[slot][:n]
        self.seen.append(data[:, 0, :8].copy().view(np.uint64).ravel().tolist())
        self.dig[slot] = oracle.encode_hash_parts(self.d, self.p, data, 1)


def test_write_stream_collects_every_digest_and_checks_them():
    """end_to_end's full check: timed_write copies each batch's digests out when its slot comes
    round again (and after the drain), and stream_check re-derives every part (ring part k mod R,
    stamped with k) with the oracle; one wrong digest is reported with its part."""
    c = bench.HostCopier(2)
    try:
        d, p, L, P, depth, n = 3, 2, 256, 4, 3, 23
        ring = bench.source_ring(5, d, L, 11, c)  # 23 stream parts wrap the 5-part ring
        pl = _OracleWritePipeline(d, p, L, P, depth)
        got = np.full((n, d + p, 32), 0xEE, np.uint8)
        bench.timed_write(pl, bench.ring_reader(ring, c), 0, n, 1, got)
        assert not (got == 0xEE).all(axis=(1, 2)).any()  # every part's digests were collected
        assert bench.stream_check(ring.copy(), got, d, p, 2) == []
        got[17, d + 1, 3] ^= 1
        assert bench.stream_check(ring.copy(), got, d, p, 2) == [17]
    finally:
        c.close()


def test_rank_threads_respect_the_quota_share(monkeypatch):
    """N ranks share one cgroup CPU quota: each rank's reader threads stay within its share (less
    one CPU for its main thread), the scheduler's staging threads take half of it; without a quota
    the affinity rule (half the CPUs, 8 at most) applies."""
    from chunky_ec import sharding
    monkeypatch.delenv("CEC_E2E_THREADS", raising=False)
    monkeypatch.delenv("CEC_MULTI_COPY_THREADS", raising=False)
    monkeypatch.setattr(sharding.os, "sched_getaffinity", lambda pid: set(range(128)))
    monkeypatch.setattr(sharding, "cpu_quota", lambda: (128, 16.0))
    assert [sharding.rank_threads(w) for w in (1, 2, 4, 8)] == [8, 7, 3, 1]
    assert [sharding.multi_copy_threads(w) for w in (1, 2, 4, 8)] == [4, 4, 2, 1]
    assert sharding.quota_share(8) == 2.0
    monkeypatch.setattr(sharding, "cpu_quota", lambda: (128, None))
    assert [sharding.rank_threads(w) for w in (1, 8)] == [8, 8]
    assert sharding.multi_copy_threads(8) == 4 and sharding.quota_share(8) is None
    monkeypatch.setenv("CEC_E2E_THREADS", "3")
    assert sharding.rank_threads(8) == 3


def test_measured_valu_names_its_source():
    """valu_roofline.counters: the headline kernel's VALU issue from the committed SQ counters
    (profiles/valu.json, profiles/summarize_shapes.py): about one VALU per 4.15 SIMD-cycles, i.e.
    ~0.96 of a lone wave's one-per-4-cycles issue floor; None for unprofiled shapes."""
    v = bench.measured_valu("c2", "encode_hash_kernel", True)
    assert v and 4.0 < v["simd_cycles_per_valu"] < 4.4 and 0.9 < v["valu_busy"] <= 1.0
    assert "not this run" in v["source"] and "r4e_c2_summary.md" in v["source"]
    assert bench.measured_valu("c2", "encode_hash_kernel", False) is None
    assert bench.measured_valu("c4", "encode_hash_kernel", True) is None


def test_gpus_n_without_launcher_starts_the_ranks_as_a_child(monkeypatch):
    """`bench.py --gpus 8` with no WORLD_SIZE: the script starts torch.distributed.run with 8
    ranks on 127.0.0.1 as a CHILD (subprocess, never exec), passes its own arguments through, and
    exits with the child's status; nothing touches the GPU first."""
    import subprocess
    seen = {}

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return subprocess.CompletedProcess(cmd, 3)

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "5", "--warmup", "2"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 3
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    assert cmd[-7:] == [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "5",
                        "--warmup", "2"]
    assert bench.rank_launch_cmd(2, ["--gpus", "2"], 29500)[4] == "--nproc-per-node=2"


def test_world_size_other_than_gpus_exits_nonzero():
    """Under a launcher whose world size differs from --gpus the bench refuses to print a line
    (exit 2) instead of reporting the wrong n_gpus; run as the driver would, in a subprocess."""
    import subprocess
    assert bench.world_mismatch(4, 4) is None and "WORLD_SIZE=2" in bench.world_mismatch(2, 8)
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 2, out.stderr[-2000:]
    assert "WORLD_SIZE=2 but --gpus=1" in out.stderr and not out.stdout.strip()


def test_rank_rows_carry_each_ranks_oracle_check():
    """The N > 1 line's per-rank rows: check_vs_oracle 1 / 0 / -1 -> True / False / None."""
    base = [0, 0, 1, 64, 40.0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4]
    assert bench.rank_row(0, base + [1.0])["check_vs_oracle"] is True
    assert bench.rank_row(1, base + [0.0])["check_vs_oracle"] is False
    assert bench.rank_row(2, base + [-1.0])["check_vs_oracle"] is None


def test_rccl_ranks_never_share_a_gpu():
    """More RCCL ranks than visible GPUs would fail or hang in the communicator's init: the bench
    exits 2 first.  The gloo rehearsal may put several ranks on one GPU."""
    assert bench.rccl_overcommit(8, "nccl", 8) is None
    assert bench.rccl_overcommit(1, "nccl", 0) is None
    assert "2 RCCL ranks but 1 visible GPU" in bench.rccl_overcommit(2, "nccl", 1)
    assert bench.rccl_overcommit(4, "gloo", 1) is None
