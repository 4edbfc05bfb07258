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

// ---------------------------------------------------------------------------------------------
// Reads
// ---------------------------------------------------------------------------------------------

/// Failure of [`BatchReader::read`]: the engine's (a part that runs out of chunks is
/// `CecError::Erasure(Error::TooFewShardsPresent)`, as the reference's read fails), or the
/// sink's own error.
#[derive(Debug)]
pub enum BatchReadError<E> {
    Engine(CecError),
    Sink(E),
}

/// A read window submitted to the scheduler and not yet handed to the sink.
struct LiveRead {
    slot: usize,
    job: u64,
    first: usize,
    n: usize,
}

/// `FileReadBuilder`'s reader (reader.rs:40-75) batched over the multi-GPU scheduler with
/// `read_with_context`'s retry rule (file_part.rs:86-129), parts handed out in file order.
///
/// For each part of a window of `parts_per_batch * devices.len()` parts it loads the first d
/// chunks `fetch` returns (data chunks first, so an intact part needs no rebuild) into a
/// page-locked buffer, and submits the window as one scheduler job: every loaded chunk verified
/// against its metadata digest, the data chunks rebuilt.  It loads the next window while that one
/// runs.  A part whose loaded chunks do not all verify goes again with the chunks that verified
/// (`CEC_PRESENT_VERIFIED`: used, not hashed again) and as many untried chunks as it is short of
/// d, until it decodes or runs out of chunks.  `include/chunky_ec.hpp`'s
/// `FileReference::read_run` / `retry` is the same loop in C++ and
/// `chunky-bits_amd/chunky_ec/batchreader.py` its Python twin; both are tested on the GPU.
pub struct BatchReader {
    // declared (so dropped) first: the scheduler refers to the codec and the windows
    multi: Multi,
    codec: ReedSolomon,
    d: usize,
    t: usize,
    chunk_size: usize,
    window: usize,
    chunks: [HostBuffer; 2],
    out: [HostBuffer; 2],
    present: [Vec<u8>; 2],
    expected: [Vec<u8>; 2],
    verified: [Vec<u8>; 2],
    status: [Vec<c_int>; 2],
    retries: u64,
}

impl BatchReader {
    /// A reader of RS(`data`, `parity`) parts of `chunk_size`-byte chunks on `devices`.
    pub fn new(
        data: usize,
        parity: usize,
        chunk_size: usize,
        parts_per_batch: usize,
        depth: usize,
        devices: &[c_int],
    ) -> Result<BatchReader, CecError> {
        let codec = ReedSolomon::new(data, parity)?;  // file_part.rs:77
        let multi = Multi::new(&codec, chunk_size, parts_per_batch, depth, devices)?;
        let window = parts_per_batch * devices.len().max(1);
        let dev0 = devices.first().copied().unwrap_or(-1);
        let t = data + parity;
        let buf = |n: usize| HostBuffer::zeroed(n, dev0);
        Ok(BatchReader {
            chunks: [buf(window * t * chunk_size)?, buf(window * t * chunk_size)?],
            out: [buf(window * data * chunk_size)?, buf(window * data * chunk_size)?],
            present: [vec![0u8; window * t], vec![0u8; window * t]],
            expected: [vec![0u8; window * t * 32], vec![0u8; window * t * 32]],
            verified: [vec![0u8; window * t], vec![0u8; window * t]],
            status: [vec![0; window], vec![0; window]],
            multi,
            codec,
            d: data,
            t,
            chunk_size,
            window,
            retries: 0,
        })
    }

    /// Part resubmissions so far (a part retried twice counts twice).
    pub fn retries(&self) -> u64 {
        self.retries
    }

    /// The codec the parts were written with (`FilePart`'s d and p).
    pub fn codec(&self) -> &ReedSolomon {
        &self.codec
    }

    /// Parts `0..n_parts` of a file: `digests` holds the metadata digests, `n_parts * (d + p)`
    /// of them, part by part (`FilePart::data` then `parity`); `fetch(part, chunk)` returns the
    /// stored chunk's bytes, or `None` when no location has it (`Location::read_with_context`
    /// over the chunk's locations, file_part.rs:100-107); `sink(part, data_chunks)` gets the d
    /// data chunks of every part in file order, valid during the call.
    pub fn read<F, S, E>(
        &mut self,
        n_parts: usize,
        digests: &[[u8; 32]],
        mut fetch: F,
        mut sink: S,
    ) -> Result<(), BatchReadError<E>>
    where
        F: FnMut(usize, usize) -> Option<Vec<u8>>,
        S: FnMut(usize, &[&[u8]]) -> Result<(), E>,
    {
        if digests.len() < n_parts * self.t {
            return Err(BatchReadError::Engine(crate::too_small("digests")));
        }
        let mut at = 0usize;
        let mut slot = 0usize;
        let mut pending: Option<LiveRead> = None;
        loop {
            let mut current = None;
            if at < n_parts {
                let cnt = self.window.min(n_parts - at);
                self.load(slot, at, cnt, digests, &mut fetch);
                match unsafe { self.submit(slot, cnt) } {
                    Ok(job) => current = Some(LiveRead { slot, job, first: at, n: cnt }),
                    Err(e) => {
                        self.drain(pending.take());
                        return Err(BatchReadError::Engine(e));
                    },
                }
                at += cnt;
            }
            // the older window's parts go out first: file order
            if let Some(prev) = pending.take() {
                if let Err(e) = self.collect(prev, &mut fetch, &mut sink) {
                    self.drain(current);
                    return Err(e);
                }
            }
            match current {
                None => return Ok(()),
                Some(c) => pending = Some(c),
            }
            slot ^= 1;
        }
    }

    /// The first d chunks `fetch` returns for each part of window `slot` (file_part.rs:86-107
    /// loads d), and every chunk's metadata digest.
    fn load<F>(&mut self, slot: usize, first: usize, cnt: usize, digests: &[[u8; 32]], fetch: &mut F)
    where
        F: FnMut(usize, usize) -> Option<Vec<u8>>,
    {
        let (d, t, l) = (self.d, self.t, self.chunk_size);
        let ch: &mut [u8] = &mut self.chunks[slot];
        let pres = &mut self.present[slot];
        let exp = &mut self.expected[slot];
        for q in 0..cnt {
            let mut loaded = 0usize;
            for i in 0..t {
                let x = q * t + i;
                exp[x * 32..(x + 1) * 32].copy_from_slice(&digests[(first + q) * t + i]);
                pres[x] = 0;
                if loaded == d {
                    continue;
                }
                if let Some(b) = fetch(first + q, i) {
                    if b.len() == l {
                        ch[x * l..(x + 1) * l].copy_from_slice(&b);
                        pres[x] = 1;
                        loaded += 1;
                    }
                }
            }
        }
    }

    /// Queues the verify + rebuild of the first `cnt` parts of window `slot`.
    ///
    /// # Safety
    /// The window's buffers are not touched again until the job is collected or drained.
    unsafe fn submit(&mut self, slot: usize, cnt: usize) -> Result<u64, CecError> {
        let chunks = self.chunks[slot].as_ptr();
        let present = self.present[slot].as_ptr();
        let expected = self.expected[slot].as_ptr();
        let out = self.out[slot].as_mut_ptr();
        let verified = self.verified[slot].as_mut_ptr();
        let status = self.status[slot].as_mut_ptr();
        self.multi.submit_read(chunks, present, expected, cnt, out, verified, status)
    }

    /// Waits for a window's job, retries its failed parts, then hands its parts to the sink.
    fn collect<F, S, E>(&mut self, w: LiveRead, fetch: &mut F, sink: &mut S) -> Result<(), BatchReadError<E>>
    where
        F: FnMut(usize, usize) -> Option<Vec<u8>>,
        S: FnMut(usize, &[&[u8]]) -> Result<(), E>,
    {
        self.multi.wait(w.job).map_err(BatchReadError::Engine)?;
        let failed: Vec<usize> = (0..w.n).filter(|&q| self.status[w.slot][q] != 0).collect();
        if !failed.is_empty() {
            self.retry(&w, &failed, fetch).map_err(BatchReadError::Engine)?;
        }
        let (d, l) = (self.d, self.chunk_size);
        let out: &[u8] = &self.out[w.slot];
        for q in 0..w.n {
            let data: Vec<&[u8]> = (0..d).map(|j| &out[(q * d + j) * l..(q * d + j + 1) * l]).collect();
            sink(w.first + q, &data).map_err(BatchReadError::Sink)?;
        }
        Ok(())
    }

    /// file_part.rs:92-107: the failed parts go again with the chunks that verified (flagged
    /// `CEC_PRESENT_VERIFIED`, taken from the window's buffer: the bytes that verified) plus
    /// untried ones up to d, until each decodes; a part with no untried chunk left fails the read.
    fn retry<F>(&mut self, w: &LiveRead, failed: &[usize], fetch: &mut F) -> Result<(), CecError>
    where
        F: FnMut(usize, usize) -> Option<Vec<u8>>,
    {
        let (d, t, l) = (self.d, self.t, self.chunk_size);
        let f = failed.len();
        let mut tried = vec![false; f * t];
        let mut good = vec![false; f * t];
        let mut keep = vec![0u8; f * t * l];  // bytes of every chunk loaded so far
        {
            let ch: &[u8] = &self.chunks[w.slot];
            for (r, &q) in failed.iter().enumerate() {
                for i in 0..t {
                    tried[r * t + i] = self.present[w.slot][q * t + i] != 0;
                    good[r * t + i] = self.verified[w.slot][q * t + i] != 0;
                }
                keep[r * t * l..(r + 1) * t * l].copy_from_slice(&ch[q * t * l..(q + 1) * t * l]);
            }
        }
        // pageable (the scheduler stages them): pinning a retry buffer per window would cost more
        // than the few parts it carries (~0.35 s per GiB)
        let mut r_chunks = vec![0u8; f * t * l];
        let mut r_out = vec![0u8; f * d * l];
        let mut r_pres = vec![0u8; f * t];
        let mut r_exp = vec![0u8; f * t * 32];
        let mut r_ver = vec![0u8; f * t];
        let mut open: Vec<usize> = (0..f).collect();
        while !open.is_empty() {
            let g = open.len();
            for (s, &r) in open.iter().enumerate() {
                let q = failed[r];
                r_exp[s * t * 32..(s + 1) * t * 32]
                    .copy_from_slice(&self.expected[w.slot][q * t * 32..(q + 1) * t * 32]);
                let have = (0..t).filter(|&i| good[r * t + i]).count();
                let mut added = 0usize;
                for i in 0..t {
                    let (x, y) = (r * t + i, s * t + i);
                    r_pres[y] = 0;
                    if good[x] {
                        r_chunks[y * l..(y + 1) * l].copy_from_slice(&keep[x * l..(x + 1) * l]);
                        r_pres[y] = crate::sys::CEC_PRESENT_VERIFIED;
                    } else if !tried[x] && have + added < d {
                        tried[x] = true;
                        if let Some(b) = fetch(w.first + q, i) {
                            if b.len() == l {
                                keep[x * l..(x + 1) * l].copy_from_slice(&b);
                                r_chunks[y * l..(y + 1) * l].copy_from_slice(&b);
                                r_pres[y] = 1;
                                added += 1;
                            }
                        }
                    }
                }
                if added == 0 {
                    return Err(CecError::Erasure(crate::Error::TooFewShardsPresent));
                }
            }
            let status = self.multi.read(&r_chunks, &r_pres, &r_exp, g, &mut r_out, &mut r_ver)?;
            self.retries += g as u64;
            let mut still = Vec::new();
            let out: &mut [u8] = &mut self.out[w.slot];
            for (s, &r) in open.iter().enumerate() {
                let q = failed[r];
                for i in 0..t {
                    good[r * t + i] = r_ver[s * t + i] != 0;
                }
                if status[s].is_ok() {
                    out[q * d * l..(q + 1) * d * l].copy_from_slice(&r_out[s * d * l..(s + 1) * d * l]);
                } else {
                    still.push(r);
                }
            }
            open = still;
        }
        Ok(())
    }

    /// Waits for a window's job without handing out its parts (error paths).
    fn drain(&self, w: Option<LiveRead>) {
        if let Some(w) = w {
            let _ = self.multi.wait(w.job);
        }
    }
}
