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
