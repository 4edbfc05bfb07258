"""The C1 format fixture (tests/golden/make_format_fixture.py): a 50 MiB file, d=3, p=2, 1 MiB
chunks, whose FileReference YAML and chunk files the REFERENCE's own reader
(python/chunky-bits.py) read back bit-exact with an empty stderr, in the build container.

CPU: the fixture is what the oracle produces for that input (so the oracle's part slicing,
chunk sizes and digests are pinned by a run of the reference's code), and the recorded run is
clean (and its corrupted-chunk control was caught).
GPU: the engine, through the per-call C-ABI (cec_part_encode, FilePart::write_with_encoder's
compute) and through the device batch (cec_encode_hash_batch), gives every part the YAML's
chunk size and data/parity digests, and its data chunks, concatenated in order and truncated to
`length` as the reference's reader does, hash to the reference run's stdout.  Parity digests
are the oracle's (the reference's script reads data chunks only: RS parity stays unpinned).
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_format_fixture as fx  # noqa: E402  (test infrastructure: slicing + oracle)
from _gen import gen_bytes  # noqa: E402

YAML = os.path.join(HERE, "golden", "c1_file_reference.yaml")
RUN = os.path.join(HERE, "golden", "c1_reference_run.json")


def _fixture():
    return yaml.safe_load(open(YAML)), json.load(open(RUN))


def test_reference_run_was_clean_and_its_control_caught():
    ref, run = _fixture()
    assert run["returncode"] == 0 and run["stderr"] == ""
    assert run["stdout_len"] == ref["length"] == fx.LENGTH
    assert run["stdout_sha256"] == run["input_sha256"] == \
        hashlib.sha256(fx.c1_input().tobytes()).hexdigest()
    c = run["corrupted_control"]
    assert c["stderr_lines"] == 1 and c["stderr_names_the_chunk"] and c["stdout_sha256_differs"]
    assert run["parts"] == len(ref["parts"]) == 17 and run["last_chunksize"] == 699051


def test_oracle_reproduces_the_fixture():
    ref, _ = _fixture()
    assert fx.file_reference(fx.c1_input()) == ref
    # serde field order of the layout the reference's reader parsed
    assert list(ref) == ["length", "parts"]
    for part in ref["parts"]:
        assert list(part) == ["chunksize", "data", "parity"]
        for ch in part["data"] + part["parity"]:
            assert list(ch) == ["sha256", "locations"]
            assert ch["locations"] == [f"sha256-{ch['sha256']}"]


def _reader_stdout(ref, data_chunks):
    """python/chunky-bits.py's output: data chunks in order, truncated to `length`."""
    left, out = ref["length"], hashlib.sha256()
    for c in data_chunks:
        c = c[:left]
        left -= len(c)
        out.update(c)
    return out.hexdigest()


@pytest.mark.gpu
def test_engine_per_call_matches_reference_format():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import chunky_ec as ce
    ref, run = _fixture()
    data = fx.c1_input()
    rs = ce.ReedSolomon(fx.D, fx.P)
    chunks_out = []
    step = fx.D * fx.CHUNK
    for k, part in enumerate(ref["parts"]):
        n = min(step, len(data) - k * step)
        buf = np.zeros(step, np.uint8)  # writer.rs:172: a zeroed d*chunk_size buffer
        buf[:n] = data[k * step:k * step + n]
        enc = ce.part_encode(rs, buf, n)
        assert enc.chunksize == part["chunksize"], k
        want = [c["sha256"] for c in part["data"] + part["parity"]]
        assert [str(h) for h in enc.hashes] == want, k
        L = enc.chunksize
        chunks_out += [buf[j * L:(j + 1) * L].tobytes() for j in range(fx.D)]
        for i, pc in enumerate(enc.parity):
            assert hashlib.sha256(pc).hexdigest() == part["parity"][i]["sha256"], (k, i)
    assert _reader_stdout(ref, chunks_out) == run["stdout_sha256"]


@pytest.mark.gpu
def test_engine_device_batch_matches_reference_format():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import chunky_ec as ce
    ref, _ = _fixture()
    data = fx.c1_input()
    d, p = fx.D, fx.P
    t = d + p
    rs = ce.ReedSolomon(d, p)
    # the 16 full parts as one batch ([part][d+p][L], 16-byte aligned: the fused path), the short
    # last part (699 051-byte chunks: the byte-granular path) as a batch of its own
    groups = [(list(range(16)), fx.CHUNK, fx.CHUNK), ([16], 699051, 699051 + 5)]
    for parts, L, stride in groups:
        host = np.zeros((len(parts), t, stride), np.uint8)
        for q, k in enumerate(parts):
            n = min(d * fx.CHUNK, len(data) - k * d * fx.CHUNK)
            buf = np.zeros(d * L, np.uint8)
            buf[:n] = data[k * d * fx.CHUNK:k * d * fx.CHUNK + n]
            host[q, :d, :L] = buf.reshape(d, L)
        dev = torch.from_numpy(host).cuda()
        dig = torch.zeros((len(parts), t, 32), dtype=torch.uint8, device="cuda")
        ce.encode_hash_batch(rs, ce.PartBatch.from_tensor(dev, L), dig.data_ptr())
        torch.cuda.synchronize()
        got = dig.cpu().numpy()
        for q, k in enumerate(parts):
            assert ref["parts"][k]["chunksize"] == L
            want = [c["sha256"] for c in ref["parts"][k]["data"] + ref["parts"][k]["parity"]]
            assert [got[q, i].tobytes().hex() for i in range(t)] == want, k


# --- the engine's own store, read back by the reference (tests/golden/make_dropin_record.py) ---

DROPIN_YAML = os.path.join(HERE, "golden", "dropin_file_reference.yaml")
DROPIN_RUN = os.path.join(HERE, "golden", "dropin_reference_run.json")


def test_reference_reader_reads_the_engines_repaired_store():
    """tools/dropin_cp_repair.py wrote a 22 MiB file through the batched writer on the GPU,
    deleted / damaged five chunk files, read it back through the batched reader and repaired
    the store through the scheduler's resilver; the reference's python/chunky-bits.py then read
    the engine's FileReference and chunk files: exit 0, no digest mismatch, stdout = the input
    (and its control with one flipped byte was caught)."""
    run = json.load(open(DROPIN_RUN))
    gpu = run["gpu_side"]
    assert run["returncode"] == 0 and run["stderr"] == ""
    data = gen_bytes(gpu["seed"], gpu["length"])
    assert run["stdout_len"] == gpu["length"]
    assert run["stdout_sha256"] == gpu["input_sha256"] == hashlib.sha256(data.tobytes()).hexdigest()
    assert gpu["cat_equals_input"] is True and gpu["cat_after_repair_equals_input"] is True
    assert sorted(map(tuple, gpu["repaired"])) == sorted(map(tuple, gpu["deleted"] +
                                                             [gpu["corrupted"]]))
    # the engine's verify before the repair: exactly the deleted locations unavailable and the
    # damaged one invalid; after it, every location of every chunk valid
    assert sorted(tuple(x[:2]) for x in gpu["verify_before"]["unavailable"]) == \
        sorted(map(tuple, gpu["deleted"]))
    assert [x[:2] for x in gpu["verify_before"]["invalid"]] == [gpu["corrupted"]]
    assert gpu["verify_after"] == {"unavailable": [], "invalid": [], "unhealthy_chunks": 0}
    c = run["corrupted_control"]
    assert c["stderr_lines"] == 1 and c["stderr_names_the_chunk"] and c["stdout_sha256_differs"]


def test_engine_reads_chunks_listed_bad_then_good():
    """stale.yaml: p + 1 chunks of every part listed [stale copy, good copy], so fewer than d first
    copies verify.  The engine's batched reader walked each chunk's locations like
    read_with_context (file_part.rs:100-107) and read the file back; its verify flagged exactly the
    stale copies and resilver rebuilt nothing (each chunk has a valid copy).  The reference's
    python reader, which checks each data chunk's FIRST location only, confirms those first copies
    are the bad ones: its mismatch lines name exactly the stale data chunks."""
    run = json.load(open(DROPIN_RUN))
    s = run["gpu_side"]["stale"]
    assert s["cat_equals_input"] is True and s["repaired"] == [] and s["resilver_errors"] == []
    assert sorted(x[:2] for x in s["verify"]["invalid"]) == sorted(s["stale_chunks"])
    assert all(x[2] == 0 for x in s["verify"]["invalid"]) and s["verify"]["unhealthy_chunks"] == 0
    d, p = run["gpu_side"]["d"], run["gpu_side"]["p"]
    assert len(s["stale_chunks"]) == s["parts"] * (p + 1)
    ref = run["stale_file"]
    assert sorted(x.split(" != ")[0] for x in ref["stderr_lines"]) == \
        sorted(ref["stale_data_hashes"])
    assert len(ref["stale_data_hashes"]) == sum(1 for k, i in s["stale_chunks"] if i < d)


def test_engines_store_equals_the_oracle_file_reference():
    """The FileReference the GPU wrote -- chunk sizes, data digests AND parity digests -- equals
    the oracle's for the same input: the engine's parity bytes (batched writer for the full
    parts, cec_part_encode for the short last one) match the CPU restatement of the crate on
    every part of this file."""
    ref = yaml.safe_load(open(DROPIN_YAML))
    gpu = json.load(open(DROPIN_RUN))["gpu_side"]
    d, p, chunk = gpu["d"], gpu["p"], gpu["chunk_size"]
    data = gen_bytes(gpu["seed"], gpu["length"])
    assert ref["length"] == gpu["length"] and len(ref["parts"]) == gpu["parts"]
    for k, (L, chunks) in enumerate(fx.parts_of(data, d, p, chunk)):
        part = ref["parts"][k]
        assert part["chunksize"] == L
        hexes = [hashlib.sha256(c.tobytes()).hexdigest() for c in chunks]
        assert [c["sha256"] for c in part["data"]] == hexes[:d], k
        assert [c["sha256"] for c in part["parity"]] == hexes[d:], k
        # one location per chunk; a repaired chunk lists its rewritten file a second time
        # (resilver appends the new location, file_part.rs:346)
        for i, c in enumerate(part["data"] + part["parity"]):
            n = 2 if [k, i] in gpu["repaired"] else 1
            assert c["locations"] == [f"sha256-{c['sha256']}"] * n, (k, i)
