"""chunky_ec.readstream over the real cec_read_pipeline (HIP verify + decode): the batched
read_with_context retry loop (file_part.rs:86-122) against oracle-encoded stored chunks with
damaged fetches -- every decoded part equals the stored data, every damaged chunk is rejected,
parts that run out of chunks are reported, and the same loop through bench.py's
timed_read_repair (the c5r / end_to_end.read_repair path)."""
import hashlib
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

import chunky_ec as ce  # noqa: E402
import oracle  # noqa: E402
from chunky_ec.readstream import ReadRepairStream  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _store(n, d, p, L, seed):
    rng = np.random.default_rng(seed)
    chunks = np.zeros((n, d + p, L), np.uint8)
    dig = np.zeros((n, d + p, 32), np.uint8)
    for k in range(n):
        data = rng.integers(0, 256, size=(d, L), dtype=np.uint8)
        st, par = oracle.encode_sep(d, p, list(data))
        assert st == 0
        chunks[k, :d], chunks[k, d:] = data, np.stack(par)
        for i in range(d + p):
            dig[k, i] = np.frombuffer(hashlib.sha256(chunks[k, i].tobytes()).digest(), np.uint8)
    return chunks, dig


@pytest.mark.parametrize("d,p,L,corrupt", [(10, 4, 4096, 0.05), (3, 2, 1000, 0.2),
                                           (20, 8, 777, 0.03)])
def test_read_repair_stream_on_the_pipeline(d, p, L, corrupt):
    n, P, depth = 61, 8, 3
    chunks, dig = _store(n, d, p, L, d * 100 + p)
    codec = ce.ReedSolomon(d, p)
    rp = ce.ReadPipeline(codec, L, P, depth, ce.ReadPipeline.REBUILT_ONLY)
    rng = np.random.default_rng(5)
    damaged = [0]

    def fetch(slot_chunks, rows):
        for k, part, flags in rows:
            for j in np.flatnonzero(flags):
                slot_chunks[k, j] = chunks[part, j]
                if flags[j] == 1 and rng.random() < corrupt:
                    slot_chunks[k, j, rng.integers(L)] ^= 0x81
                    damaged[0] += 1

    got = {}

    def on_part(slot, nb, k, part, attempts):
        got[part] = (rp.part_bytes(slot, nb, k), attempts)

    s = ReadRepairStream(rp, fetch, lambda ids: dig[ids], seed=1, on_part=on_part).run(0, n)
    assert s.parts + s.undecodable_parts == n
    assert s.rejected_chunks == damaged[0] > 0 and s.retried_parts > 0
    for part, (out, _) in got.items():
        assert out == chunks[part, :d].tobytes(), part
    assert any(a > 1 for _, a in got.values())
    assert set(got) | set(s.undecodable) == set(range(n))


def test_read_repair_stream_runs_out_of_chunks_on_the_pipeline():
    d, p, L, n = 3, 2, 512, 10
    chunks, dig = _store(n, d, p, L, 4)
    rp = ce.ReadPipeline(ce.ReedSolomon(d, p), L, 4, 2, ce.ReadPipeline.REBUILT_ONLY)

    def fetch(slot_chunks, rows):
        for k, part, flags in rows:
            for j in np.flatnonzero(flags):
                slot_chunks[k, j] = chunks[part, j]
                # part 7: chunks 0-1 always served damaged (3 good of 5: it decodes after
                # retries); part 3: chunks 0-2 (2 good of 5 < d: undecodable)
                if flags[j] == 1 and ((part == 7 and j < 2) or (part == 3 and j < 3)):
                    slot_chunks[k, j, 0] ^= 1

    s = ReadRepairStream(rp, fetch, lambda ids: dig[ids], seed=0).run(0, n)
    assert s.undecodable == [3] and s.parts == n - 1


def test_bench_timed_read_repair_small():
    sys.path.insert(0, ROOT)
    import bench
    d, p, L, P, depth = 10, 4, 65536, 16, 3
    chunks, dig = _store(40, d, p, L, 9)
    copier = bench.HostCopier(4)
    try:
        el, stats, checks = bench.timed_read_repair(ce.ReedSolomon(d, p), chunks, dig, L, P, depth,
                                                    0, 200, 1, 0.05, copier, 3)
    finally:
        copier.close()
    assert el > 0 and stats["parts"] == 200 and stats["undecodable_parts"] == 0
    assert stats["rejected_chunks"] == stats["damaged_loads"] > 0
    assert checks and all(c["ok"] for c in checks)
    assert any(c["attempts"] > 1 for c in checks)
