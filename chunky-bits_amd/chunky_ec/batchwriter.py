"""FileWriteBuilder::write batched over the multi-GPU scheduler: the Python twin of the Rust
crate's ``chunky_ec_sys::batch::BatchWriter`` (chunky-bits_amd/rust/chunky-ec-sys/src/batch.rs)
and of the C++ ``FileWriteBuilder::write_full_parts`` (include/chunky_ec.hpp), step for step, so
the loop the Rust side would run is executed and tested on the GPU (tests/test_gpu_batchwriter.py).

The reference reads one part at a time into ``vec![0; data * chunk_size]`` (src/file/writer.rs:
172-194: read until the buffer is full or a read returns 0) and runs
``FilePart::write_with_encoder`` per part (file_part.rs:137-225).  :class:`BatchWriter` reads the
same parts with the same rule, a window of ``parts_per_batch * depth * len(devices)`` at a time
into a page-locked buffer, submits every full part of the window as one scheduler job (encode +
SHA-256, parts split over the GPUs in contiguous ranges) while the reader fills the other window,
and hands each part to ``sink`` in file order as write_with_encoder produces it.  A short last part
(chunk size ``ceil(len / d)``) goes through :func:`chunky_ec.part_encode`.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional

from . import HostBuffer, Multi, ReedSolomon, part_encode


@dataclass
class EncodedPart:
    """One part as FilePart::write_with_encoder produces it (file_part.rs:150-199)."""

    index: int            # part number in file order
    length: int           # bytes of the file in this part (bytes_read, writer.rs:173-194)
    chunksize: int        # ceil(length / d) (file_part.rs:152)
    digests: List[bytes]  # d data then p parity SHA-256 digests (file_part.rs:185)
    chunks: List[memoryview]  # d data then p parity chunks, chunksize bytes each (valid in sink)


@dataclass
class _Live:
    slot: int
    job: Optional[int]
    first: int
    full: int


class BatchWriter:
    def __init__(self, data: int, parity: int, chunk_size: int, parts_per_batch: int, depth: int,
                 devices: List[int]):
        self.codec = ReedSolomon(data, parity)  # writer.rs:131
        self.multi = Multi(self.codec, chunk_size, parts_per_batch, depth, devices,
                           kinds=Multi.WRITE)
        self.d, self.p, self.L = data, parity, chunk_size
        self.window = parts_per_batch * depth * max(len(devices), 1)
        dev0 = devices[0] if devices else -1
        t = data + parity
        self.data = [HostBuffer(self.window * data * chunk_size, dev0) for _ in range(2)]
        self.parity = [HostBuffer(self.window * parity * chunk_size, dev0) for _ in range(2)]
        self.digests = [HostBuffer(self.window * t * 32, dev0) for _ in range(2)]

    def write(self, reader, sink: Callable[[EncodedPart], None]) -> int:
        """Reads ``reader`` (any object with ``readinto``) to its end, calling ``sink`` once per
        part in file order; returns the file length (FileReference::length)."""
        part_cap = self.d * self.L
        total = index = slot = 0
        pending: Optional[_Live] = None
        while True:
            try:
                full, short, eof = self._fill(reader, slot)
            except BaseException:
                self._drain(pending)
                raise
            total += full * part_cap + short
            job = None
            if full:
                try:
                    job = self._submit(slot, full)
                except BaseException:
                    self._drain(pending)
                    raise
            current = _Live(slot, job, index, full)
            index += full
            if pending is not None:  # the older window first: file order
                prev, pending = pending, None
                try:
                    self._collect(prev, sink)
                except BaseException:
                    self._drain(current)
                    raise
            if eof:
                self._collect(current, sink)
                if short:
                    self._short_part(slot, full, short, index, sink)
                return total
            pending = current
            slot ^= 1

    def _fill(self, reader, slot: int):
        """Up to `window` parts into window `slot`, each as writer.rs:172-194 reads one; the
        unread tail of a short part is zeroed.  Returns (full parts, short part bytes, eof)."""
        part_cap = self.d * self.L
        buf = memoryview(self.data[slot].array)
        for k in range(self.window):
            part = buf[k * part_cap:(k + 1) * part_cap]
            got = 0
            while got < part_cap:
                n = reader.readinto(part[got:])
                if not n:
                    break
                got += n
            if got < part_cap:
                self.data[slot].array[k * part_cap + got:(k + 1) * part_cap] = 0
                return k, got, True
        return self.window, 0, False

    def _submit(self, slot: int, n: int) -> int:
        return self.multi.encode_hash(self.data[slot], n, self.parity[slot], self.digests[slot])

    def _collect(self, w: _Live, sink) -> None:
        if w.job is not None:
            self.multi.wait(w.job)
        d, p, L = self.d, self.p, self.L
        t = d + p
        data = memoryview(self.data[w.slot].array)
        par = memoryview(self.parity[w.slot].array)
        dig = self.digests[w.slot].array
        for k in range(w.full):
            chunks = [data[(k * d + i) * L:(k * d + i + 1) * L] for i in range(d)]
            chunks += [par[(k * p + i) * L:(k * p + i + 1) * L] for i in range(p)]
            digests = [dig[(k * t + i) * 32:(k * t + i + 1) * 32].tobytes() for i in range(t)]
            sink(EncodedPart(w.first + k, d * L, L, digests, chunks))

    def _short_part(self, slot: int, k: int, length: int, index: int, sink) -> None:
        part_cap = self.d * self.L
        buf = memoryview(self.data[slot].array)[k * part_cap:(k + 1) * part_cap]
        enc = part_encode(self.codec, buf, length)
        L = enc.chunksize
        chunks = [buf[j * L:(j + 1) * L] for j in range(self.d)]
        chunks += [memoryview(c) for c in enc.parity]
        sink(EncodedPart(index, length, L, [h.digest for h in enc.hashes], chunks))

    def _drain(self, w: Optional[_Live]) -> None:
        if w is not None and w.job is not None:
            try:
                self.multi.wait(w.job)
            except Exception:  # noqa: BLE001 (the error being raised is the caller's)
                pass
