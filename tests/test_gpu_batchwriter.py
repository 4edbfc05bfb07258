"""chunky_ec.batchwriter.BatchWriter (the executed twin of the Rust crate's batch::BatchWriter and
the C++ write_full_parts) on the GPU: every part it hands out equals FilePart::write_with_encoder's
output restated with the oracle -- part cut by writer.rs:172-194 (read until d*chunk_size bytes or
end of input), chunk size ceil(len/d) with zero padding (file_part.rs:150-158), parity by
encode_sep, d+p SHA-256 digests in order -- at lengths around the window and part boundaries,
with a reader that returns short reads, and over two scheduler shards."""
import hashlib
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

import oracle  # noqa: E402
from chunky_ec.batchwriter import BatchWriter  # noqa: E402

D, P, L = 3, 2, 4096
CAP = D * L


class Trickle(io.RawIOBase):
    """A reader that returns at most `step` bytes per read (the reference's loop must keep
    reading until the part buffer is full, writer.rs:176-192)."""

    def __init__(self, data, step):
        self.src, self.pos, self.step = data, 0, step

    def readable(self):
        return True

    def readinto(self, b):
        n = min(len(b), self.step, len(self.src) - self.pos)
        b[:n] = self.src[self.pos:self.pos + n]
        self.pos += n
        return n


def _expected_part(file_bytes, k):
    """write_with_encoder for part k of file_bytes, restated with the oracle."""
    part = file_bytes[k * CAP:(k + 1) * CAP]
    n = len(part)
    Lk = (n + D - 1) // D
    buf = np.zeros(D * Lk, np.uint8)
    buf[:n] = np.frombuffer(part, np.uint8)
    data = [buf[j * Lk:(j + 1) * Lk] for j in range(D)]
    st, par = oracle.encode_sep(D, P, data)
    assert st == 0
    chunks = [x.tobytes() for x in data] + [x.tobytes() for x in par]
    return n, Lk, chunks, [hashlib.sha256(c).digest() for c in chunks]


def _write(writer, file_bytes, step=None):
    parts = []

    def sink(p):
        parts.append((p.index, p.length, p.chunksize, list(p.digests),
                      [bytes(c) for c in p.chunks]))

    reader = Trickle(file_bytes, step) if step else io.BytesIO(file_bytes)
    total = writer.write(reader, sink)
    return total, parts


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_batch_writer_parts_equal_write_with_encoder(devices):
    w = BatchWriter(D, P, L, 2, 2, devices)
    W = w.window  # 4 parts per shard-window
    rng = np.random.default_rng(7)
    for n in (0, 1, CAP - 1, CAP, CAP + 1, 3 * CAP + 7, W * CAP, W * CAP + CAP,
              2 * W * CAP + 123, 3 * W * CAP - 1):
        file_bytes = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        total, parts = _write(w, file_bytes, step=1000 if n % 2 else None)
        assert total == n
        assert [p[0] for p in parts] == list(range((n + CAP - 1) // CAP)), n
        for idx, length, chunksize, digests, chunks in parts:
            want_n, want_L, want_chunks, want_dig = _expected_part(file_bytes, idx)
            assert (length, chunksize) == (want_n, want_L), (n, idx)
            assert chunks == want_chunks, (n, idx)
            assert digests == want_dig, (n, idx)


def test_batch_writer_sink_error_leaves_no_job_running():
    """A sink that fails mid-file: the error surfaces, the window in flight is waited for, and
    the writer is reusable for the next file (its windows are free)."""
    w = BatchWriter(D, P, L, 2, 2, [0])
    data = np.random.default_rng(1).integers(0, 256, 5 * w.window * CAP, dtype=np.uint8).tobytes()
    seen = []

    def sink(p):
        seen.append(p.index)
        if p.index == w.window + 1:
            raise RuntimeError("destination full")

    with pytest.raises(RuntimeError, match="destination full"):
        w.write(io.BytesIO(data), sink)
    assert seen == list(range(w.window + 2))
    total, parts = _write(w, data[:CAP + 5])
    assert total == CAP + 5 and [p[0] for p in parts] == [0, 1]
    assert parts[1][4] == _expected_part(data[:CAP + 5], 1)[2]
