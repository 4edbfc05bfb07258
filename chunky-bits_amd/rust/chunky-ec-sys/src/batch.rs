//! `FileWriteBuilder::write` batched over the multi-GPU scheduler (the loop INTEGRATION.md §3.1
//! wires into src/file/writer.rs:117-255).
//!
//! The reference reads the input one part at a time into `vec![0; data * chunk_size]`
//! (writer.rs:172-194: read until the buffer is full or the reader returns 0), spawns
//! `FilePart::write_with_encoder` per part (≤ `concurrency` = 10 at once, writer.rs:56,130) and
//! collects the parts in file order.  [`BatchWriter::write`] reads the same parts with the same
//! rule, but a window of `parts_per_batch × depth × shards` of them at a time into a page-locked
//! buffer, encodes + hashes every full part of the window in one scheduler job (the parts of a
//! job are split over the GPUs in contiguous ranges) while the reader fills the other window, and
//! hands each part to the caller's sink in file order, as `write_with_encoder` would produce it:
//! the chunk size, the d + p digests in order, and the chunk bytes to store.  A short last part
//! (fewer than `data * chunk_size` bytes: chunk size `ceil(len / d)`, zero padded,
//! file_part.rs:150-158) goes through the per-call [`part_encode`].
//!
//! `include/chunky_ec.hpp`'s `FileWriteBuilder::write_full_parts` is the same loop in C++ (tested
//! on the GPU by tests/test_cpp_mirror.py); this file mirrors it step for step.  Like the rest of
//! the crate it has not been compiled here (no cargo in the build image).
use std::io::{self, Read};
use std::os::raw::c_int;

use crate::{part_encode, CecError, HostBuffer, Multi, ReedSolomon};

/// One part as `FilePart::write_with_encoder` produces it (file_part.rs:150-199).
pub struct EncodedPart<'a> {
    /// Part number in file order, from 0.
    pub index: u64,
    /// Bytes of the file in this part (`bytes_read`, writer.rs:173-194).
    pub length: usize,
    /// `FilePart::chunksize`: `ceil(length / d)` (file_part.rs:152).
    pub chunksize: usize,
    /// The d data digests then the p parity digests (`Chunk::hash`, file_part.rs:185).
    pub digests: Vec<[u8; 32]>,
    /// The d data chunks then the p parity chunks, `chunksize` bytes each: what `write_shard`
    /// stores under each digest (file_part.rs:186).  Borrowed from the writer's buffers for the
    /// duration of the sink call.
    pub chunks: Vec<&'a [u8]>,
}

/// Failure of [`BatchWriter::write`]: the reader's, the engine's, or the sink's own error.
#[derive(Debug)]
pub enum BatchWriteError<E> {
    Io(io::Error),
    Engine(CecError),
    Sink(E),
}

impl<E: std::fmt::Debug> std::fmt::Display for BatchWriteError<E> {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        match self {
            BatchWriteError::Io(e) => write!(f, "read error: {}", e),
            BatchWriteError::Engine(e) => write!(f, "{}", e),
            BatchWriteError::Sink(e) => write!(f, "sink error: {:?}", e),
        }
    }
}

/// A window submitted to the scheduler and not yet handed to the sink.
struct Live {
    slot: usize,
    job: Option<u64>,
    first: u64,
    full: usize,
}

/// The batched part writer: a codec, a scheduler over `devices`, and two page-locked windows of
/// parts (data in, parity and digests out).  One thread drives it (`Send`, not `Sync`).
pub struct BatchWriter {
    // declared (so dropped) first: the scheduler refers to the codec and the windows
    multi: Multi,
    codec: ReedSolomon,
    d: usize,
    p: usize,
    chunk_size: usize,
    window: usize,
    data: [HostBuffer; 2],
    parity: [HostBuffer; 2],
    digests: [HostBuffer; 2],
}

impl BatchWriter {
    /// `FileWriteBuilder { chunk_size, data, parity }` (writer.rs:88-110) on `devices` (one
    /// scheduler shard each), `parts_per_batch` parts per GPU launch and `depth` launches in
    /// flight per GPU; a window is `parts_per_batch * depth * devices.len()` parts.
    pub fn new(
        data: usize,
        parity: usize,
        chunk_size: usize,
        parts_per_batch: usize,
        depth: usize,
        devices: &[c_int],
    ) -> Result<BatchWriter, CecError> {
        let codec = ReedSolomon::new(data, parity)?;  // writer.rs:131
        let multi = Multi::new(&codec, chunk_size, parts_per_batch, depth, devices)?;
        let window = parts_per_batch * depth * devices.len().max(1);
        // page-locked on the first GPU's NUMA node (the C++ loop's placement)
        let dev0 = devices.first().copied().unwrap_or(-1);
        let buf = |n: usize| HostBuffer::zeroed(n, dev0);
        let t = data + parity;
        Ok(BatchWriter {
            data: [buf(window * data * chunk_size)?, buf(window * data * chunk_size)?],
            parity: [buf(window * parity * chunk_size)?, buf(window * parity * chunk_size)?],
            digests: [buf(window * t * 32)?, buf(window * t * 32)?],
            multi,
            codec,
            d: data,
            p: parity,
            chunk_size,
            window,
        })
    }

    /// Parts per window (per scheduler job).
    pub fn window(&self) -> usize {
        self.window
    }

    /// Reads `reader` to its end and calls `sink` once per part, in file order; returns the
    /// file length (`FileReference::length`, writer.rs:194,252).  On any error the jobs in
    /// flight are waited for before it returns (no job outlives the call).
    pub fn write<R, F, E>(&mut self, reader: &mut R, mut sink: F) -> Result<u64, BatchWriteError<E>>
    where
        R: Read,
        F: FnMut(EncodedPart<'_>) -> Result<(), E>,
    {
        let part_cap = self.d * self.chunk_size;
        let mut total = 0u64;
        let mut index = 0u64;
        let mut pending: Option<Live> = None;
        let mut slot = 0usize;
        loop {
            // the reader fills this window while the other one's job runs
            let (full, short, eof) = match self.fill(reader, slot) {
                Ok(v) => v,
                Err(e) => {
                    self.drain(pending.take());
                    return Err(BatchWriteError::Io(e));
                },
            };
            total += (full * part_cap + short) as u64;
            let job = if full > 0 {
                match unsafe { self.submit(slot, full) } {
                    Ok(j) => Some(j),
                    Err(e) => {
                        self.drain(pending.take());
                        return Err(BatchWriteError::Engine(e));
                    },
                }
            } else {
                None
            };
            let current = Live { slot, job, first: index, full };
            index += full as u64;
            // the older window's parts go out first: file order
            if let Some(prev) = pending.take() {
                if let Err(e) = self.collect(prev, &mut sink) {
                    self.drain(Some(current));
                    return Err(e);
                }
            }
            if eof {
                self.collect(current, &mut sink)?;
                if short > 0 {
                    self.short_part(slot, full, short, index, &mut sink)?;
                }
                return Ok(total);
            }
            pending = Some(current);
            slot ^= 1;
        }
    }

    /// Reads up to `window` parts into window `slot`, each exactly as writer.rs:172-194 reads
    /// one: until `d * chunk_size` bytes or a read of 0; the unread tail of a short part is
    /// zeroed (`vec![0; data * chunk_size]`).  Returns (full parts, bytes of a trailing short
    /// part or 0, end of input reached).
    fn fill<R: Read>(&mut self, reader: &mut R, slot: usize) -> io::Result<(usize, usize, bool)> {
        let part_cap = self.d * self.chunk_size;
        let buf: &mut [u8] = &mut self.data[slot];
        for k in 0..self.window {
            let part = &mut buf[k * part_cap..(k + 1) * part_cap];
            let mut got = 0usize;
            while got < part_cap {
                match reader.read(&mut part[got..]) {
                    Ok(0) => break,
                    Ok(n) => got += n,
                    Err(e) if e.kind() == io::ErrorKind::Interrupted => continue,
                    Err(e) => return Err(e),
                }
            }
            if got < part_cap {
                for b in part[got..].iter_mut() {
                    *b = 0;
                }
                return Ok((k, got, true));
            }
        }
        Ok((self.window, 0, false))
    }

    /// Queues the encode + SHA-256 of the first `n` parts of window `slot`.
    ///
    /// # Safety
    /// The window's buffers are not touched again until the job is collected or drained (the
    /// loop in `write` alternates windows and always collects before refilling one).
    unsafe fn submit(&mut self, slot: usize, n: usize) -> Result<u64, CecError> {
        let data = self.data[slot].as_ptr();
        let parity = self.parity[slot].as_mut_ptr();
        let digests = self.digests[slot].as_mut_ptr();
        self.multi.submit_encode_hash(data, n, parity, digests)
    }

    /// Waits for a window's job, then hands its parts to the sink in order.
    fn collect<F, E>(&self, w: Live, sink: &mut F) -> Result<(), BatchWriteError<E>>
    where
        F: FnMut(EncodedPart<'_>) -> Result<(), E>,
    {
        if let Some(job) = w.job {
            self.multi.wait(job).map_err(BatchWriteError::Engine)?;
        }
        let (d, p, l) = (self.d, self.p, self.chunk_size);
        let t = d + p;
        let data: &[u8] = &self.data[w.slot];
        let parity: &[u8] = &self.parity[w.slot];
        let dig: &[u8] = &self.digests[w.slot];
        for k in 0..w.full {
            let mut chunks: Vec<&[u8]> = Vec::with_capacity(t);
            for i in 0..d {
                chunks.push(&data[(k * d + i) * l..(k * d + i + 1) * l]);
            }
            for i in 0..p {
                chunks.push(&parity[(k * p + i) * l..(k * p + i + 1) * l]);
            }
            let digests = (0..t)
                .map(|i| {
                    let mut h = [0u8; 32];
                    h.copy_from_slice(&dig[(k * t + i) * 32..(k * t + i + 1) * 32]);
                    h
                })
                .collect();
            let part = EncodedPart { index: w.first + k as u64, length: d * l, chunksize: l, digests, chunks };
            sink(part).map_err(BatchWriteError::Sink)?;
        }
        Ok(())
    }

    /// The short last part (k-th of window `slot`, `length` bytes): `part_encode` at chunk size
    /// ceil(length / d), data chunks sliced from the zero-padded part buffer (file_part.rs:152-155).
    fn short_part<F, E>(
        &self,
        slot: usize,
        k: usize,
        length: usize,
        index: u64,
        sink: &mut F,
    ) -> Result<(), BatchWriteError<E>>
    where
        F: FnMut(EncodedPart<'_>) -> Result<(), E>,
    {
        let part_cap = self.d * self.chunk_size;
        let buf: &[u8] = &self.data[slot][k * part_cap..(k + 1) * part_cap];
        let (chunksize, parity, digests) =
            part_encode(&self.codec, buf, length).map_err(BatchWriteError::Engine)?;
        let mut chunks: Vec<&[u8]> =
            (0..self.d).map(|j| &buf[j * chunksize..(j + 1) * chunksize]).collect();
        chunks.extend(parity.iter().map(|c| c.as_slice()));
        sink(EncodedPart { index, length, chunksize, digests, chunks }).map_err(BatchWriteError::Sink)
    }

    /// Waits for a window's job without handing out its parts (error paths).
    fn drain(&self, w: Option<Live>) {
        if let Some(Live { job: Some(job), .. }) = w {
            let _ = self.multi.wait(job);
        }
    }
}
