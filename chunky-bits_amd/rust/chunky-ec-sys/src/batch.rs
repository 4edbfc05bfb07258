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
        let multi = Multi::with_kinds(&codec, chunk_size, parts_per_batch, depth, devices,
                                     crate::sys::CEC_MULTI_WRITE)?;
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

/// Window buffers of a [`BatchReader`] of scheduler depth `depth`: up to `depth` windows' read
/// jobs in flight (at most 7) and one being emitted.
fn read_windows_for(depth: usize) -> usize {
    depth.clamp(2, 7) + 1
}

/// A read window submitted to the scheduler and not yet handed to the sink.
struct LiveRead {
    slot: usize,
    job: u64,
    first: usize,
    n: usize,
    checked: bool,         // its read job waited for (and its retry started)
    retry: Option<Retry>,  // its failed parts, while they are being read again
}

/// The retry of a window's failed parts (file_part.rs:92-107), one round in flight at a time.
struct Retry {
    failed: Vec<usize>,  // window rows of the failed parts
    open: Vec<usize>,    // indices into `failed` of the parts not yet decoded
    tried: Vec<bool>,    // [f][t]
    good: Vec<bool>,
    exhausted: Vec<bool>,
    cursor: Vec<usize>,
    cid: Vec<i32>,  // [f] carry id of the part's verified chunks (-1: none)
    // the round in flight
    g: usize,
    job: u64,
    in_flight: bool,
    r_pres: Vec<u8>,
    r_exp: Vec<u8>,
    r_ver: Vec<u8>,
    r_status: Vec<c_int>,
    r_cin: Vec<i32>,
    r_cout: Vec<i32>,
}

/// The chunk's next copy from location `start` on (`fetch` reads `chunk.locations[start..]` and
/// returns `(index, bytes)` of the first location that reads): `(next start, bytes)`, or `None`
/// when the locations are exhausted.  A copy that is not `size` bytes cannot hash to the metadata
/// digest (the reference hashes it and moves on, file_part.rs:100-107), so it is passed over.
fn next_copy<F>(fetch: &mut F, part: usize, chunk: usize, start: usize, size: usize) -> Option<(usize, Vec<u8>)>
where
    F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
{
    let mut start = start;
    loop {
        let (loc, bytes) = fetch(part, chunk, start)?;
        start = loc + 1;
        if bytes.len() == size {
            return Some((start, bytes));
        }
    }
}

/// Chunks to load next for a part short of d verified chunks: those whose copy failed
/// verification first (their next location: file_part.rs:100-107 walks a chunk's locations
/// before it draws another chunk), then the untried ones.
fn draw_order(good: &[bool], tried: &[bool], exhausted: &[bool]) -> Vec<usize> {
    let t = good.len();
    let again = (0..t).filter(|&i| tried[i] && !good[i] && !exhausted[i]);
    let fresh = (0..t).filter(|&i| !tried[i] && !exhausted[i]);
    again.chain(fresh).collect()
}

/// `FileReadBuilder`'s reader (reader.rs:40-75) batched over the multi-GPU scheduler with
/// `read_with_context`'s retry rule (file_part.rs:86-129), parts handed out in file order.
///
/// `fetch(part, chunk, start)` is one step of the reference's walk over a chunk's locations: it
/// reads `chunk.locations[start..]` in order and returns `(index, bytes)` of the first location
/// that reads, or `None` when none is left.  For each part of a window of
/// `parts_per_batch * devices.len()` parts (all of this reader's shape) the reader loads the first
/// d chunks that have a copy (data chunks first, so an intact part needs no rebuild) into a
/// page-locked buffer and submits the window as one scheduler job: every loaded chunk verified
/// against its metadata digest, the data chunks rebuilt.  It loads the next windows while the
/// earlier ones run (up to `depth` read jobs in flight).  A part whose loaded chunks do not all
/// verify goes again with the chunks that verified (`CEC_PRESENT_VERIFIED`: used, not hashed
/// again; kept on the GPU under the part's carry id), the failed chunks' NEXT copies (the same
/// chunk's next location is read before another chunk is drawn, file_part.rs:100-107), then
/// untried chunks, up to d, until it decodes or runs out of copies.  Every window is polled
/// (`Multi::query`): checked (its job waited for, the first round of its failed parts' retry
/// queued ahead of the windows queued after it, `CEC_MULTI_AHEAD`) as soon as its job is done,
/// and each next round queued as soon as the last one is, so retries run beside the loading of
/// the next windows.  Only the rebuilt data chunks come down (`CEC_READ_REBUILT_ONLY`): a loaded
/// one reaches the sink from the window's chunk buffer.  So a chunk listed `[bad, good]` -- what
/// resilver leaves when it appends a rebuilt copy's location (file_part.rs:346) -- reads as in
/// the reference.  [`FileReader`] splits a file into runs of one shape (the short last part has
/// its own chunk size).
/// `include/chunky_ec.hpp`'s `FileReference::read_run` / `retry_start` / `retry_collect` is the
/// same loop in C++ and `chunky-bits_amd/chunky_ec/batchreader.py` its Python twin; both are
/// tested on the GPU.
pub struct BatchReader {
    // declared (so dropped) first: the scheduler refers to the codec and the windows
    multi: Multi,
    codec: ReedSolomon,
    d: usize,
    t: usize,
    chunk_size: usize,
    window: usize,
    windows: usize,  // window buffers (read_windows_for(depth))
    chunks: Vec<HostBuffer>,
    out: Vec<HostBuffer>,
    present: Vec<Vec<u8>>,
    expected: Vec<Vec<u8>>,
    verified: Vec<Vec<u8>>,
    status: Vec<Vec<c_int>>,
    // per chunk of a window: the next location to read, and whether none is left
    cursor: Vec<Vec<usize>>,
    exhausted: Vec<Vec<bool>>,
    // per part of a window: the scheduler's carry id of its verified chunks (-1: none kept)
    carry: Vec<Vec<i32>>,
    // per data chunk of a window: its address (`CEC_READ_REBUILT_ONLY`: in the window's chunk
    // buffer where it was loaded, else in its output), and per part whether a retry rebuilt it
    // into the output
    ptrs: Vec<Vec<usize>>,
    redone: Vec<Vec<bool>>,
    retries: u64,
    carried: u64,
    dev0: c_int,
    // per window: retry buffers, kept between retries (grown only): fresh zeroed ones cost
    // ~200 ms of page faults per retry of a dozen RS(10,4) 1 MiB parts, and page-locked ones go
    // up unstaged
    retry_bufs: Vec<RetryBuffers>,
}

#[derive(Default)]
struct RetryBuffers {
    chunks: Option<HostBuffer>,
    out: Option<HostBuffer>,
    keep: Vec<u8>,
}

/// The `len` bytes at address `addr` if they lie inside `buf`.
fn window_slice(buf: &[u8], addr: usize, len: usize) -> Option<&[u8]> {
    let off = addr.checked_sub(buf.as_ptr() as usize)?;
    buf.get(off..off.checked_add(len)?)
}

/// `buf` grown to at least `n` bytes (page-locked on `dev`'s node), its first `n` bytes.
fn grown(buf: &mut Option<HostBuffer>, n: usize, dev: c_int) -> Result<&mut [u8], CecError> {
    if buf.as_ref().map_or(true, |b| b.len() < n) {
        *buf = None;  // the old buffer goes before the new one is pinned
        *buf = Some(HostBuffer::zeroed(n, dev)?);
    }
    match buf.as_mut() {
        Some(b) => Ok(&mut b[..n]),
        None => Err(crate::too_small("retry buffer")),
    }
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
        let multi = Multi::with_kinds(&codec, chunk_size, parts_per_batch, depth, devices,
                                     crate::sys::CEC_MULTI_READ)?;
        let window = parts_per_batch * devices.len().max(1);
        let dev0 = devices.first().copied().unwrap_or(-1);
        let t = data + parity;
        let r = read_windows_for(depth);
        let bufs = |n: usize| -> Result<Vec<HostBuffer>, CecError> {
            (0..r).map(|_| HostBuffer::zeroed(n, dev0)).collect()
        };
        Ok(BatchReader {
            chunks: bufs(window * t * chunk_size)?,
            out: bufs(window * data * chunk_size)?,
            present: vec![vec![0u8; window * t]; r],
            expected: vec![vec![0u8; window * t * 32]; r],
            verified: vec![vec![0u8; window * t]; r],
            status: vec![vec![0; window]; r],
            cursor: vec![vec![0; window * t]; r],
            exhausted: vec![vec![false; window * t]; r],
            carry: vec![vec![-1; window]; r],
            ptrs: vec![vec![0usize; window * data]; r],
            redone: vec![vec![false; window]; r],
            windows: r,
            multi,
            codec,
            d: data,
            t,
            chunk_size,
            window,
            retries: 0,
            carried: 0,
            dev0,
            retry_bufs: (0..r).map(|_| RetryBuffers::default()).collect(),
        })
    }

    /// Part resubmissions so far (a part retried twice counts twice).
    pub fn retries(&self) -> u64 {
        self.retries
    }

    /// Resubmissions whose verified chunks stayed on the GPU (only the new chunks were sent).
    pub fn carried(&self) -> u64 {
        self.carried
    }

    /// The codec the parts were written with (`FilePart`'s d and p).
    pub fn codec(&self) -> &ReedSolomon {
        &self.codec
    }

    /// Parts `0..n_parts` of a file, all of this reader's shape: `digests` holds the metadata
    /// digests, `n_parts * (d + p)` of them, part by part (`FilePart::data` then `parity`);
    /// `fetch(part, chunk, start)` as above; `sink(part, data_chunks)` gets the d data chunks of
    /// every part in file order, valid during the call.
    pub fn read<F, S, E>(
        &mut self,
        n_parts: usize,
        digests: &[[u8; 32]],
        mut fetch: F,
        mut sink: S,
    ) -> Result<(), BatchReadError<E>>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
        S: FnMut(usize, &[&[u8]]) -> Result<(), E>,
    {
        if digests.len() < n_parts * self.t {
            return Err(BatchReadError::Engine(crate::too_small("digests")));
        }
        let mut live: Vec<Option<LiveRead>> = (0..self.windows).map(|_| None).collect();
        let res = self.read_windows(n_parts, digests, &mut fetch, &mut sink, &mut live);
        if res.is_err() {
            self.drain(&live);
        }
        res
    }

    fn read_windows<F, S, E>(&mut self, n_parts: usize, digests: &[[u8; 32]], fetch: &mut F,
                             sink: &mut S, live: &mut [Option<LiveRead>])
                             -> Result<(), BatchReadError<E>>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
        S: FnMut(usize, &[&[u8]]) -> Result<(), E>,
    {
        let r = self.windows;
        let mut at = 0usize;
        let mut i = 0usize;
        loop {
            // windows are emitted in submission order: live[i % r] went out r steps ago
            self.poll(live, i + 1, at >= n_parts, fetch).map_err(BatchReadError::Engine)?;
            let s = i % r;
            if let Some(mut w) = live[s].take() {
                if let Err(e) = self.finish(&mut w, live, i, at >= n_parts, fetch, sink) {
                    live[s] = Some(w);  // drained by the caller
                    return Err(e);
                }
            }
            if at < n_parts {
                let cnt = self.window.min(n_parts - at);
                self.load(s, at, cnt, digests, fetch);
                let job = unsafe { self.submit(s, cnt) }.map_err(BatchReadError::Engine)?;
                live[s] = Some(LiveRead { slot: s, job, first: at, n: cnt, checked: false, retry: None });
                at += cnt;
            } else if live.iter().all(|w| w.is_none()) {
                return Ok(());
            }
            i += 1;
        }
    }

    /// The first d chunks of each part of window `slot` that have a copy (file_part.rs:86-107
    /// loads d), each at its first location that reads, and every chunk's metadata digest.
    fn load<F>(&mut self, slot: usize, first: usize, cnt: usize, digests: &[[u8; 32]], fetch: &mut F)
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
    {
        let (d, t, l) = (self.d, self.t, self.chunk_size);
        let ch: &mut [u8] = &mut self.chunks[slot];
        let pres = &mut self.present[slot];
        let exp = &mut self.expected[slot];
        let cur = &mut self.cursor[slot];
        let ex = &mut self.exhausted[slot];
        for x in self.redone[slot].iter_mut().take(cnt) {
            *x = false;
        }
        for c in self.carry[slot].iter_mut().take(cnt) {
            *c = -1;
        }
        for q in 0..cnt {
            let mut loaded = 0usize;
            for i in 0..t {
                let x = q * t + i;
                exp[x * 32..(x + 1) * 32].copy_from_slice(&digests[(first + q) * t + i]);
                pres[x] = 0;
                cur[x] = 0;
                ex[x] = false;
                if loaded == d {
                    continue;
                }
                match next_copy(fetch, first + q, i, 0, l) {
                    Some((next, b)) => {
                        cur[x] = next;
                        ch[x * l..(x + 1) * l].copy_from_slice(&b);
                        pres[x] = 1;
                        loaded += 1;
                    },
                    None => ex[x] = true,
                }
            }
        }
    }

    /// Queues the verify + rebuild of the first `cnt` parts of window `slot`.  Only the rebuilt
    /// data chunks come down (`CEC_READ_REBUILT_ONLY`): a loaded one is handed to the sink from
    /// the window's chunk buffer it went up from, `ptrs` says which.
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
        let carry = self.carry[slot].as_mut_ptr();
        // usize and a data pointer have one size and layout: the C side writes addresses
        let ptrs = self.ptrs[slot].as_mut_ptr() as *mut *const u8;
        self.multi.submit_read_carry(chunks, present, expected, cnt, out, verified, status,
                                     std::ptr::null(), carry, ptrs, false)
    }

    /// Waits for a window's read job; its failed parts' first retry round goes out.
    fn check<F>(&mut self, w: &mut LiveRead, fetch: &mut F) -> Result<(), CecError>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
    {
        w.checked = true;
        self.multi.wait(w.job)?;
        let failed: Vec<usize> = (0..w.n).filter(|&q| self.status[w.slot][q] != 0).collect();
        if !failed.is_empty() {
            self.retry_start(w, failed, fetch)?;
        }
        Ok(())
    }

    /// Every live window: checked as soon as its job is done and its retry's next round queued
    /// as soon as the last one is (`Multi::query` never blocks), so retries run on the GPUs while
    /// windows load and while the loop waits for the window it emits (a retry round costs one
    /// SHA-256 chain, ~33 ms for 1 MiB chunks, whatever its size).  `everything`: checked
    /// whatever its state (nothing is left to load: the last retries run together).
    fn poll<F>(&mut self, live: &mut [Option<LiveRead>], first: usize, everything: bool,
               fetch: &mut F) -> Result<(), CecError>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
    {
        let r = live.len();
        for a in 0..r {
            if let Some(x) = live[(first + a) % r].as_mut() {
                if !x.checked {
                    if everything || self.multi.query(x.job)? {
                        self.check(x, fetch)?;
                    }
                } else if let Some(job) = x.retry.as_ref().filter(|rt| rt.in_flight).map(|rt| rt.job) {
                    if self.multi.query(job)? {
                        self.retry_collect(x, fetch)?;
                    }
                }
            }
        }
        Ok(())
    }

    /// Window `w` (taken out of `live`): its job, then its retry rounds, polling the other
    /// windows meanwhile; then its parts to the sink.
    #[allow(clippy::too_many_arguments)]
    fn finish<F, S, E>(&mut self, w: &mut LiveRead, live: &mut [Option<LiveRead>], i: usize,
                       everything: bool, fetch: &mut F, sink: &mut S) -> Result<(), BatchReadError<E>>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
        S: FnMut(usize, &[&[u8]]) -> Result<(), E>,
    {
        loop {
            if !w.checked && self.multi.query(w.job).map_err(BatchReadError::Engine)? {
                self.check(w, fetch).map_err(BatchReadError::Engine)?;
            }
            if w.checked {
                if let Some(job) = w.retry.as_ref().filter(|rt| rt.in_flight).map(|rt| rt.job) {
                    if self.multi.query(job).map_err(BatchReadError::Engine)? {
                        self.retry_collect(w, fetch).map_err(BatchReadError::Engine)?;
                    }
                }
            }
            let in_flight = w.retry.as_ref().map_or(false, |rt| rt.in_flight);
            if w.checked && !in_flight {
                break;
            }
            self.poll(live, i + 1, everything, fetch).map_err(BatchReadError::Engine)?;
            std::thread::sleep(std::time::Duration::from_micros(100));
        }
        w.retry = None;
        let (d, l) = (self.d, self.chunk_size);
        let out: &[u8] = &self.out[w.slot];
        let ch: &[u8] = &self.chunks[w.slot];
        for q in 0..w.n {
            let mut data: Vec<&[u8]> = Vec::with_capacity(d);
            for j in 0..d {
                // a retried part's data is in the output at its place; otherwise the chunk is
                // where the job said (an address inside the chunk buffer or the output)
                let bytes = if self.redone[w.slot][q] {
                    out.get((q * d + j) * l..(q * d + j + 1) * l)
                } else {
                    let p = self.ptrs[w.slot][q * d + j];
                    window_slice(ch, p, l).or_else(|| window_slice(out, p, l))
                };
                match bytes {
                    Some(b) => data.push(b),
                    None => return Err(BatchReadError::Engine(crate::too_small("data pointer"))),
                }
            }
            sink(w.first + q, &data).map_err(BatchReadError::Sink)?;
        }
        Ok(())
    }

    /// file_part.rs:92-107: the failed parts go again with the chunks that verified (flagged
    /// `CEC_PRESENT_VERIFIED`: kept on the GPU under the part's carry id, or, when the scheduler
    /// kept none, sent again from the window's buffer: the bytes that verified) plus, up to d, the
    /// failed chunks' next copies and then untried chunks, until each decodes; a part with no copy
    /// left fails the read (its and the other open parts' carry ids go back, `drain`).  This
    /// queues the first round; `retry_collect` takes each round's results and queues the next.
    fn retry_start<F>(&mut self, w: &mut LiveRead, failed: Vec<usize>, fetch: &mut F) -> Result<(), CecError>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
    {
        let (t, l) = (self.t, self.chunk_size);
        let f = failed.len();
        let mut rt = Retry {
            open: (0..f).collect(),
            tried: vec![false; f * t],
            good: vec![false; f * t],
            exhausted: vec![false; f * t],
            cursor: vec![0usize; f * t],
            cid: vec![-1; f],
            g: 0,
            job: 0,
            in_flight: false,
            r_pres: Vec::new(),
            r_exp: Vec::new(),
            r_ver: Vec::new(),
            r_status: Vec::new(),
            r_cin: Vec::new(),
            r_cout: Vec::new(),
            failed,
        };
        for (r, &q) in rt.failed.iter().enumerate() {
            rt.cid[r] = self.carry[w.slot][q];  // the retry holds the id now
            self.carry[w.slot][q] = -1;
            for i in 0..t {
                rt.tried[r * t + i] = self.present[w.slot][q * t + i] != 0;
                rt.good[r * t + i] = self.verified[w.slot][q * t + i] != 0;
                rt.exhausted[r * t + i] = self.exhausted[w.slot][q * t + i];
                rt.cursor[r * t + i] = self.cursor[w.slot][q * t + i];
            }
        }
        // bytes of every chunk loaded so far, in the window's retry buffers
        let bufs = &mut self.retry_bufs[w.slot];
        if bufs.keep.len() < f * t * l {
            bufs.keep.resize(f * t * l, 0);
        }
        let ch: &[u8] = &self.chunks[w.slot];
        for (r, &q) in rt.failed.iter().enumerate() {
            bufs.keep[r * t * l..(r + 1) * t * l].copy_from_slice(&ch[q * t * l..(q + 1) * t * l]);
        }
        w.retry = Some(rt);
        self.retry_round(w, fetch)
    }

    /// Builds and queues one round over the window's still-open failed parts.
    fn retry_round<F>(&mut self, w: &mut LiveRead, fetch: &mut F) -> Result<(), CecError>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
    {
        let (d, t, l) = (self.d, self.t, self.chunk_size);
        let rt = match w.retry.as_mut() {
            Some(rt) => rt,
            None => return Ok(()),
        };
        let f = rt.failed.len();
        let g = rt.open.len();
        let bufs = &mut self.retry_bufs[w.slot];
        let r_chunks = grown(&mut bufs.chunks, f * t * l, self.dev0)?;
        let r_out = grown(&mut bufs.out, f * d * l, self.dev0)?;
        let keep = &mut bufs.keep[..f * t * l];
        rt.r_pres = vec![0u8; g * t];
        rt.r_exp = vec![0u8; g * t * 32];
        rt.r_ver = vec![0u8; g * t];
        rt.r_status = vec![0 as c_int; g];
        rt.r_cin = vec![-1i32; g];
        rt.r_cout = vec![-1i32; g];
        for s in 0..g {
            let r = rt.open[s];
            let q = rt.failed[r];
            rt.r_exp[s * t * 32..(s + 1) * t * 32]
                .copy_from_slice(&self.expected[w.slot][q * t * 32..(q + 1) * t * 32]);
            let have = (0..t).filter(|&i| rt.good[r * t + i]).count();
            rt.r_cin[s] = rt.cid[r];
            for i in 0..t {
                let (x, y) = (r * t + i, s * t + i);
                if rt.good[x] {
                    if rt.cid[r] < 0 {  // not kept on the GPU: send the bytes that verified
                        r_chunks[y * l..(y + 1) * l].copy_from_slice(&keep[x * l..(x + 1) * l]);
                    }
                    rt.r_pres[y] = crate::sys::CEC_PRESENT_VERIFIED;
                }
            }
            let mut added = 0usize;
            let order = draw_order(&rt.good[r * t..(r + 1) * t], &rt.tried[r * t..(r + 1) * t],
                                   &rt.exhausted[r * t..(r + 1) * t]);
            for i in order {
                if !(have + added < d) {
                    break;
                }
                let (x, y) = (r * t + i, s * t + i);
                rt.tried[x] = true;
                match next_copy(fetch, w.first + q, i, rt.cursor[x], l) {
                    Some((next, b)) => {
                        rt.cursor[x] = next;
                        keep[x * l..(x + 1) * l].copy_from_slice(&b);
                        r_chunks[y * l..(y + 1) * l].copy_from_slice(&b);
                        rt.r_pres[y] = 1;
                        added += 1;
                    },
                    None => rt.exhausted[x] = true,
                }
            }
            if added == 0 {
                return Err(CecError::Erasure(crate::Error::TooFewShardsPresent));
            }
        }
        let carry_out = rt.r_cout.as_mut_ptr();
        rt.job = unsafe {
            self.multi.submit_read_carry(r_chunks.as_ptr(), rt.r_pres.as_ptr(), rt.r_exp.as_ptr(), g,
                                         r_out.as_mut_ptr(), rt.r_ver.as_mut_ptr(),
                                         rt.r_status.as_mut_ptr(), rt.r_cin.as_ptr(), carry_out,
                                         std::ptr::null_mut(), true)
        }?;
        for s in 0..g {  // submitted: the ids are the job's now
            let r = rt.open[s];
            if rt.cid[r] >= 0 {
                self.carried += 1;
            }
            rt.cid[r] = -1;
        }
        rt.g = g;
        rt.in_flight = true;
        Ok(())
    }

    /// Waits for the round in flight: the parts that decoded go to the window's output, the
    /// others go again in the next round, queued here (until every part decodes or one runs out
    /// of copies).
    fn retry_collect<F>(&mut self, w: &mut LiveRead, fetch: &mut F) -> Result<(), CecError>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
    {
        let (d, t, l) = (self.d, self.t, self.chunk_size);
        let again = {
            let rt = match w.retry.as_mut() {
                Some(rt) if rt.in_flight => rt,
                _ => return Ok(()),
            };
            rt.in_flight = false;
            self.multi.wait(rt.job)?;
            self.retries += rt.g as u64;
            let r_out: &[u8] = match self.retry_bufs[w.slot].out.as_ref() {
                Some(b) => &b[..],
                None => return Err(crate::too_small("retry buffer")),
            };
            let out: &mut [u8] = &mut self.out[w.slot];
            let mut still = Vec::new();
            for s in 0..rt.g {
                let r = rt.open[s];
                let q = rt.failed[r];
                for i in 0..t {
                    rt.good[r * t + i] = rt.r_ver[s * t + i] != 0;
                }
                if rt.r_status[s] == 0 {
                    out[q * d * l..(q + 1) * d * l].copy_from_slice(&r_out[s * d * l..(s + 1) * d * l]);
                    self.redone[w.slot][q] = true;
                } else if rt.r_status[s] == crate::sys::CEC_TOO_FEW_SHARDS_PRESENT {
                    rt.cid[r] = rt.r_cout[s];
                    still.push(r);
                } else {
                    return Err(crate::check(rt.r_status[s]).unwrap_err());
                }
            }
            rt.open = still;
            !rt.open.is_empty()
        };
        if again {
            self.retry_round(w, fetch)?;
        }
        Ok(())
    }

    /// Error paths: no job may still write into the windows, and carry ids nobody will use go
    /// back to their GPUs.
    fn drain(&self, live: &[Option<LiveRead>]) {
        for w in live.iter().flatten() {
            if !w.checked {
                let _ = self.multi.wait(w.job);
            }
            for &id in self.carry[w.slot].iter().take(w.n).filter(|&&id| id >= 0) {
                let _ = self.multi.carry_release(id);
            }
            if let Some(rt) = w.retry.as_ref() {
                if rt.in_flight && self.multi.wait(rt.job).is_ok() {
                    // the round's ids for its parts still short of d: nobody collects them now
                    for &id in rt.r_cout.iter().take(rt.g).filter(|&&id| id >= 0) {
                        let _ = self.multi.carry_release(id);
                    }
                }
                for &id in rt.cid.iter().filter(|&&id| id >= 0) {
                    let _ = self.multi.carry_release(id);
                }
            }
        }
    }
}

/// `read_with_context` (file_part.rs:73-135) for one part through the per-call API, with the
/// batched loop's rule: chunks drawn data first, each kept at its first copy that verifies (one
/// `sha256_many`-style round of GPU digests per draw), the failed chunks' next copies and then
/// untried chunks until d verify (`TooFewShardsPresent` when the copies run out), missing data
/// rebuilt with `reconstruct_data`; returns the d data chunks concatenated.  The path for a part
/// whose shape no batched run has: the short last part (chunk size ceil(len / d)).
pub fn read_part<F>(
    codec: &ReedSolomon,
    chunksize: usize,
    digests: &[[u8; 32]],
    part: usize,
    mut fetch: F,
) -> Result<Vec<u8>, CecError>
where
    F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
{
    let (d, t) = (codec.data_shard_count(), codec.total_shard_count());
    if digests.len() < t {
        return Err(crate::too_small("digests"));
    }
    let (mut good, mut tried, mut exhausted) = (vec![false; t], vec![false; t], vec![false; t]);
    let mut cursor = vec![0usize; t];
    let mut shards: Vec<Option<Vec<u8>>> = vec![None; t];
    let mut have = 0usize;
    while have < d {
        let mut round: Vec<(usize, Vec<u8>)> = Vec::new();
        for i in draw_order(&good, &tried, &exhausted) {
            if have + round.len() >= d {
                break;
            }
            tried[i] = true;
            match next_copy(&mut fetch, part, i, cursor[i], chunksize) {
                Some((next, b)) => {
                    cursor[i] = next;
                    round.push((i, b));
                },
                None => exhausted[i] = true,
            }
        }
        if round.is_empty() {
            return Err(CecError::Erasure(crate::Error::TooFewShardsPresent));
        }
        let hashes = crate::sha256_many(&round.iter().map(|(_, b)| b.as_slice()).collect::<Vec<_>>())?;
        for ((i, b), h) in round.into_iter().zip(hashes) {
            if h == digests[i] {
                good[i] = true;
                shards[i] = Some(b);
                have += 1;
            }
        }
    }
    if shards[..d].iter().any(Option::is_none) {
        codec.reconstruct_data(&mut shards)?;
    }
    let mut out = Vec::with_capacity(d * chunksize);
    for s in shards.into_iter().take(d).flatten() {
        out.extend_from_slice(&s);
    }
    Ok(out)
}

/// A part's shape: (d, p, chunk size).  Consecutive parts of one shape form a batched run.
pub type Shape = (usize, usize, usize);

/// Keeps the `keep` most recently used values per key (the readers' and checkers' windows pin
/// host memory, ~0.35 s per GiB, so a service reuses them across files).
struct ShapeCache<K, V> {
    keep: usize,
    entries: Vec<(K, V)>,
}

impl<K: PartialEq + Copy, V> ShapeCache<K, V> {
    fn new(keep: usize) -> Self {
        ShapeCache { keep: keep.max(1), entries: Vec::new() }
    }

    /// The value for `shape`, made by `make` when absent (evicting the least recently used).
    fn get<M>(&mut self, shape: K, make: M) -> Result<&mut V, CecError>
    where
        M: FnOnce() -> Result<V, CecError>,
    {
        if let Some(at) = self.entries.iter().position(|(s, _)| *s == shape) {
            let e = self.entries.remove(at);
            self.entries.push(e);
        } else {
            while self.entries.len() >= self.keep {
                self.entries.remove(0);  // dropped: frees its pinned windows
            }
            let v = make()?;
            self.entries.push((shape, v));
        }
        match self.entries.last_mut() {
            Some((_, v)) => Ok(v),
            None => Err(crate::too_small("shape cache")),
        }
    }
}

/// Runs of consecutive equal shapes: (first part, parts in the run).
fn shape_runs(shapes: &[Shape], first: usize, end: usize) -> Vec<(usize, usize)> {
    let mut runs = Vec::new();
    let end = end.min(shapes.len());
    let mut k = first;
    while k < end {
        let mut n = 1;
        while k + n < end && shapes[k + n] == shapes[k] {
            n += 1;
        }
        runs.push((k, n));
        k += n;
    }
    runs
}

/// `FileReadBuilder::len_bytes` (reader.rs:129-138): the bytes a read from `seek` taking `take`
/// (0: to the end) gives of a `length`-byte file; 0 for a seek past the end (where the reference's
/// u64 subtraction would underflow).
pub fn range_len(length: u64, seek: u64, take: u64) -> u64 {
    if seek >= length {
        0
    } else if take == 0 {
        length - seek
    } else {
        take.min(length - seek)
    }
}

/// `FileReadBuilder`'s reader over a whole file (reader.rs:32-74): consecutive parts of one shape
/// go through a [`BatchReader`] of that shape, kept for later files (the `keep` most recently
/// used shapes); a lone part -- the short last part, whose chunk size is ceil(len / d)
/// (file_part.rs:152) -- through [`read_part`].  One `FileReader` per service thread replaces
/// the per-file `BatchReader::new` of INTEGRATION.md §3.2.
pub struct FileReader {
    parts_per_batch: usize,
    depth: usize,
    devices: Vec<c_int>,
    readers: ShapeCache<Shape, BatchReader>,
    codecs: ShapeCache<(usize, usize), ReedSolomon>,
}

impl FileReader {
    pub fn new(parts_per_batch: usize, depth: usize, devices: &[c_int], keep: usize) -> FileReader {
        FileReader {
            parts_per_batch,
            depth,
            devices: devices.to_vec(),
            readers: ShapeCache::new(keep),
            codecs: ShapeCache::new(keep),
        }
    }

    /// Every part of a file, in order: `shapes[k]` is part k's (d, p, chunksize), `digests` its
    /// d + p metadata digests part by part, `fetch` / `sink` as [`BatchReader::read`] with file
    /// part numbers.
    pub fn read<F, S, E>(
        &mut self,
        shapes: &[Shape],
        digests: &[[u8; 32]],
        fetch: F,
        sink: S,
    ) -> Result<(), BatchReadError<E>>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
        S: FnMut(usize, &[&[u8]]) -> Result<(), E>,
    {
        self.read_parts(shapes, digests, 0, shapes.len(), fetch, sink)
    }

    /// `FileReadBuilder::seek` / `take` (reader.rs:22-173; the gateway's Range reads, http.rs:
    /// 37-56): the file's bytes `[seek, seek + range_len(length, seek, take))` -- `length` is
    /// `FileReference::len_bytes` -- from the parts that hold them, `sink(part, pieces)` getting
    /// each part's bytes inside the range.  Parts wholly before the range are not read and the
    /// first part's leading bytes are dropped, as the reference does (reader.rs:44-65); parts
    /// wholly past it are not read either (the reference reads them and empties their bytes,
    /// reader.rs:67-75, so an undecodable part past the range fails its read and not this one).
    /// Returns the bytes handed out.
    pub fn read_range<F, S, E>(
        &mut self,
        shapes: &[Shape],
        digests: &[[u8; 32]],
        length: u64,
        seek: u64,
        take: u64,
        fetch: F,
        mut sink: S,
    ) -> Result<u64, BatchReadError<E>>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
        S: FnMut(usize, &[&[u8]]) -> Result<(), E>,
    {
        let want = range_len(length, seek, take);
        if want == 0 {
            return Ok(0);
        }
        let part_len = |k: usize| (shapes[k].0 * shapes[k].2) as u64;
        let (mut first, mut skip) = (0usize, seek);
        while first < shapes.len() && skip >= part_len(first) {
            skip -= part_len(first);
            first += 1;
        }
        let (mut end, mut covered) = (first, 0u64);
        while end < shapes.len() && covered < skip + want {
            covered += part_len(end);
            end += 1;
        }
        let mut left = want;
        self.read_parts(shapes, digests, first, end, fetch, |k, data| {
            let mut pieces: Vec<&[u8]> = Vec::with_capacity(data.len());
            for &c in data {
                let s = (c.len() as u64).min(skip) as usize;
                skip -= s as u64;
                let m = ((c.len() - s) as u64).min(left) as usize;
                left -= m as u64;
                if m > 0 {
                    pieces.push(&c[s..s + m]);
                }
            }
            sink(k, &pieces)
        })?;
        Ok(want - left)
    }

    /// Parts `[first, end)` to `sink` in file order (as [`FileReader::read`]).
    pub fn read_parts<F, S, E>(
        &mut self,
        shapes: &[Shape],
        digests: &[[u8; 32]],
        first: usize,
        end: usize,
        mut fetch: F,
        mut sink: S,
    ) -> Result<(), BatchReadError<E>>
    where
        F: FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>,
        S: FnMut(usize, &[&[u8]]) -> Result<(), E>,
    {
        let mut base = 0usize;  // index of part k's first digest
        let mut offsets = Vec::with_capacity(shapes.len() + 1);
        for &(d, p, _) in shapes {
            offsets.push(base);
            base += d + p;
        }
        if digests.len() < base {
            return Err(BatchReadError::Engine(crate::too_small("digests")));
        }
        let (ppb, depth) = (self.parts_per_batch, self.depth);
        for (k0, n) in shape_runs(shapes, first, end) {
            let (d, p, l) = shapes[k0];
            let dig = &digests[offsets[k0]..offsets[k0] + n * (d + p)];
            if n == 1 {
                let codec = self.codecs.get((d, p), || ReedSolomon::new(d, p))
                    .map_err(BatchReadError::Engine)?;
                let data = read_part(codec, l, dig, k0, &mut fetch).map_err(BatchReadError::Engine)?;
                let chunks: Vec<&[u8]> = data.chunks(l.max(1)).take(d).collect();
                sink(k0, &chunks).map_err(BatchReadError::Sink)?;
                continue;
            }
            let devices = &self.devices;
            let reader = self.readers.get((d, p, l), || BatchReader::new(d, p, l, ppb, depth, devices))
                .map_err(BatchReadError::Engine)?;
            reader.read(n, dig, |q, i, s| fetch(k0 + q, i, s), |q, data| sink(k0 + q, data))?;
        }
        Ok(())
    }
}

// ---------------------------------------------------------------------------------------------
// Verify and resilver
// ---------------------------------------------------------------------------------------------

/// One location's copy, as the reference reports it (`Result<bool, LocationError>` of
/// file_part.rs:236-243 / :277-289: `Ok(true)`, `Ok(false)`, `Err(_)`).
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum CopyCheck {
    Valid,
    Invalid,
    Unreadable,
}

/// One part of a [`BatchChecker`] pass, handed to the sink in file order.
pub struct CheckedPart<'a> {
    /// Part number in file order.
    pub index: usize,
    /// `[chunk][location]`, d data then p parity chunks, each chunk's locations in the
    /// metadata's order: the reference's `read_results`.
    pub locations: Vec<Vec<CopyCheck>>,
    /// Resilver: every chunk with no valid copy, rebuilt (data and parity), to be written back
    /// with its new location appended to `chunk.locations` (file_part.rs:331-347).  Valid during
    /// the sink call.
    pub rebuilt: Vec<(usize, &'a [u8])>,
    /// Resilver: this part's rebuild failure (`ResilverPartReport::write_error`,
    /// file_part.rs:296-308), e.g. `TooFewShardsPresent`; the other parts go on.
    pub error: Option<CecError>,
}

impl CheckedPart<'_> {
    /// Chunks with a valid copy (file_part.rs:545-547's healthy chunks, before any write-back).
    pub fn valid_chunks(&self) -> usize {
        self.locations.iter().filter(|l| l.contains(&CopyCheck::Valid)).count()
    }
}

/// A verify / resilver window submitted to the scheduler and not yet handed to the sink.  Its
/// `Vec`s are the job's buffers: their heap storage does not move with the struct and they are
/// dropped only after the job was waited for.
struct LiveCheck {
    slot: usize,
    job: Option<u64>,
    first: usize,
    n: usize,
    locations: Vec<Vec<Vec<CopyCheck>>>,
    items: Vec<(usize, usize, usize)>,
    single: Vec<(usize, usize)>,
    present: Vec<u8>,
    expected: Vec<u8>,
    ver: Vec<u8>,
}

/// `FileReference::verify` / `resilver` (file_reference.rs:78-113 over `FilePart::verify` /
/// `resilver`, file_part.rs:228-390) batched over the multi-GPU scheduler, hashing every location
/// of every chunk like the reference.  `read_all(part, chunk)` returns one entry per location of
/// the chunk, in the metadata's order: the copy's bytes, or `None` where the location does not
/// read (`Location::read`).  Each readable copy is one hashing item:
///
/// * verify: every copy of a window goes to one `cec_multi_verify` job, d + p items per scheduler
///   row whatever chunk they belong to;
/// * resilver: a window whose chunks have one location each is one `cec_multi_resilver` job;
///   when some chunk has several, those chunks' copies are hashed first (a verify job) and the
///   resilver job gets their first valid copy flagged `CEC_PRESENT_VERIFIED`: every copy is still
///   hashed exactly once, each chunk keeps its first valid copy (:277-289) and only the chunks
///   with none are rebuilt (:296-308).
///
/// Two windows in flight (the next one loads while the GPU hashes the current one).
/// `chunky-bits_amd/chunky_ec/batchcheck.py` is its Python twin (tested on the GPU) and
/// `include/chunky_ec.hpp`'s `FileReference::check_run` the same loop in C++.
pub struct BatchChecker {
    // declared (so dropped) first: the scheduler refers to the codec and the windows
    multi: Multi,
    codec: ReedSolomon,
    t: usize,
    chunk_size: usize,
    window: usize,
    dev0: c_int,
    // [window][t][chunk_size] the copies, DMA'd directly; verify grows a slot's buffer when a
    // window has more copies than chunks (chunks with several locations) and keeps it
    chunks: [HostBuffer; 2],
    rebuilt: [HostBuffer; 2],
    prepass: [Option<HostBuffer>; 2],  // resilver: the copies of multi-location chunks
    present: [Vec<u8>; 2],
    expected: [Vec<u8>; 2],
    verified: [Vec<u8>; 2],
    status: [Vec<c_int>; 2],
}

impl BatchChecker {
    pub fn new(
        data: usize,
        parity: usize,
        chunk_size: usize,
        parts_per_batch: usize,
        depth: usize,
        devices: &[c_int],
    ) -> Result<BatchChecker, CecError> {
        let codec = ReedSolomon::new(data, parity)?;  // file_part.rs:302
        let multi = Multi::with_kinds(&codec, chunk_size, parts_per_batch, depth, devices,
                                     crate::sys::CEC_MULTI_READ)?;
        let window = parts_per_batch * devices.len().max(1);
        let dev0 = devices.first().copied().unwrap_or(-1);
        let t = data + parity;
        let buf = |n: usize| HostBuffer::zeroed(n, dev0);
        Ok(BatchChecker {
            chunks: [buf(window * t * chunk_size)?, buf(window * t * chunk_size)?],
            rebuilt: [buf(window * t * chunk_size)?, buf(window * t * chunk_size)?],
            prepass: [None, None],
            present: [vec![0u8; window * t], vec![0u8; window * t]],
            expected: [vec![0u8; window * t * 32], vec![0u8; window * t * 32]],
            verified: [vec![0u8; window * t], vec![0u8; window * t]],
            status: [vec![0; window], vec![0; window]],
            multi,
            codec,
            t,
            chunk_size,
            window,
            dev0,
        })
    }

    /// The codec of the parts (`FilePart`'s d and p).
    pub fn codec(&self) -> &ReedSolomon {
        &self.codec
    }

    /// `FilePart::verify` of parts `0..n_parts` (this checker's shape), reports in file order.
    pub fn verify<R, S, E>(&mut self, n_parts: usize, digests: &[[u8; 32]], read_all: R, sink: S)
        -> Result<(), BatchReadError<E>>
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
        S: FnMut(&CheckedPart<'_>) -> Result<(), E>,
    {
        self.run(0, n_parts, digests, read_all, sink, false)
    }

    /// `FilePart::resilver` of parts `0..n_parts`: the sink writes each part's `rebuilt` chunks
    /// and appends their new locations.
    pub fn resilver<R, S, E>(&mut self, n_parts: usize, digests: &[[u8; 32]], read_all: R, sink: S)
        -> Result<(), BatchReadError<E>>
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
        S: FnMut(&CheckedPart<'_>) -> Result<(), E>,
    {
        self.run(0, n_parts, digests, read_all, sink, true)
    }

    /// The window loop; `base` is added to the part numbers the sink sees (a run of a file).
    #[allow(clippy::too_many_arguments)]
    fn run<R, S, E>(&mut self, base: usize, n_parts: usize, digests: &[[u8; 32]], mut read_all: R,
                    mut sink: S, resilver: bool) -> Result<(), BatchReadError<E>>
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
        S: FnMut(&CheckedPart<'_>) -> Result<(), E>,
    {
        if digests.len() < n_parts * self.t {
            return Err(BatchReadError::Engine(crate::too_small("digests")));
        }
        let mut at = 0usize;
        let mut slot = 0usize;
        let mut pending: Option<LiveCheck> = None;
        loop {
            let mut current = None;
            if at < n_parts {
                let cnt = self.window.min(n_parts - at);
                let submitted = if resilver {
                    self.submit_resilver(slot, at, cnt, digests, &mut read_all)
                } else {
                    self.submit_verify(slot, at, cnt, digests, &mut read_all)
                };
                match submitted {
                    Ok(w) => current = Some(w),
                    Err(e) => {
                        self.drain(pending.take());
                        return Err(BatchReadError::Engine(e));
                    },
                }
                at += cnt;
            }
            // the older window's parts go out first: file order
            if let Some(prev) = pending.take() {
                let done = if resilver {
                    self.collect_resilver(prev, base, &mut sink)
                } else {
                    self.collect_verify(prev, base, &mut sink)
                };
                if let Err(e) = done {
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

    /// Every location's copy of every chunk of window [first, first + cnt) and the results'
    /// skeleton: `Unreadable` where a location does not read, `Invalid` where its copy has the
    /// wrong size (it cannot hash to the digest), `Valid` (still to be checked) otherwise.
    #[allow(clippy::type_complexity)]
    fn copies<R>(&self, first: usize, cnt: usize, read_all: &mut R)
        -> (Vec<Vec<Vec<Option<Vec<u8>>>>>, Vec<Vec<Vec<CopyCheck>>>)
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
    {
        let copies: Vec<Vec<Vec<Option<Vec<u8>>>>> =
            (0..cnt).map(|q| (0..self.t).map(|i| read_all(first + q, i)).collect()).collect();
        let l = self.chunk_size;
        let locations = copies
            .iter()
            .map(|part| {
                part.iter()
                    .map(|locs| {
                        locs.iter()
                            .map(|c| match c {
                                None => CopyCheck::Unreadable,
                                Some(b) if b.len() != l => CopyCheck::Invalid,
                                Some(_) => CopyCheck::Valid,
                            })
                            .collect()
                    })
                    .collect()
            })
            .collect();
        (copies, locations)
    }

    /// Fills a verify job's rows for `items` [(part, chunk, location)]: the copies into `buf`, d
    /// + p per row; returns (rows, present, expected, verified flags).
    #[allow(clippy::type_complexity)]
    fn rows(t: usize, l: usize, items: &[(usize, usize, usize)],
            copies: &[Vec<Vec<Option<Vec<u8>>>>], first: usize, digests: &[[u8; 32]],
            buf: &mut [u8]) -> (usize, Vec<u8>, Vec<u8>, Vec<u8>) {
        let g = (items.len() + t - 1) / t;
        let mut present = vec![0u8; g * t];
        let mut expected = vec![0u8; g * t * 32];
        for (x, &(q, i, j)) in items.iter().enumerate() {
            if let Some(b) = &copies[q][i][j] {
                buf[x * l..(x + 1) * l].copy_from_slice(b);
                present[x] = 1;
                expected[x * 32..(x + 1) * 32].copy_from_slice(&digests[(first + q) * t + i]);
            }
        }
        (g, present, expected, vec![0u8; g * t])
    }

    fn submit_verify<R>(&mut self, slot: usize, first: usize, cnt: usize, digests: &[[u8; 32]],
                        read_all: &mut R) -> Result<LiveCheck, CecError>
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
    {
        let (copies, locations) = self.copies(first, cnt, read_all);
        let mut items = Vec::new();
        for (q, part) in locations.iter().enumerate() {
            for (i, locs) in part.iter().enumerate() {
                for (j, c) in locs.iter().enumerate() {
                    if *c == CopyCheck::Valid {
                        items.push((q, i, j));
                    }
                }
            }
        }
        let mut w = LiveCheck { slot, job: None, first, n: cnt, locations, items, single: Vec::new(),
                                present: Vec::new(), expected: Vec::new(), ver: Vec::new() };
        if w.items.is_empty() {
            return Ok(w);
        }
        let (t, l) = (self.t, self.chunk_size);
        let rows_needed = (w.items.len() + t - 1) / t;
        // more copies than the window holds (chunks with several locations): the slot's buffer
        // grows, page-locked (a pageable one would go through the scheduler's staging copies)
        if rows_needed * t * l > self.chunks[slot].len() {
            self.chunks[slot] = HostBuffer::zeroed(rows_needed * t * l, self.dev0)?;
        }
        let (g, present, expected, ver) =
            Self::rows(t, l, &w.items, &copies, first, digests, &mut self.chunks[slot]);
        w.present = present;
        w.expected = expected;
        w.ver = ver;
        let buf: *const u8 = self.chunks[slot].as_ptr();
        w.job = Some(unsafe {
            self.multi.submit_verify(buf, w.present.as_ptr(), w.expected.as_ptr(), g, w.ver.as_mut_ptr())
        }?);
        Ok(w)
    }

    fn collect_verify<S, E>(&mut self, mut w: LiveCheck, base: usize, sink: &mut S)
        -> Result<(), BatchReadError<E>>
    where
        S: FnMut(&CheckedPart<'_>) -> Result<(), E>,
    {
        if let Some(job) = w.job {
            self.multi.wait(job).map_err(BatchReadError::Engine)?;
        }
        for (x, &(q, i, j)) in w.items.iter().enumerate() {
            w.locations[q][i][j] = if w.ver[x] != 0 { CopyCheck::Valid } else { CopyCheck::Invalid };
        }
        for (q, locations) in w.locations.into_iter().enumerate() {
            let part = CheckedPart { index: base + w.first + q, locations, rebuilt: Vec::new(), error: None };
            sink(&part).map_err(BatchReadError::Sink)?;
        }
        Ok(())
    }

    fn submit_resilver<R>(&mut self, slot: usize, first: usize, cnt: usize, digests: &[[u8; 32]],
                          read_all: &mut R) -> Result<LiveCheck, CecError>
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
    {
        let (t, l) = (self.t, self.chunk_size);
        let (copies, mut locations) = self.copies(first, cnt, read_all);
        // chunks with several locations: every copy hashed first (file_part.rs:277-289)
        let mut multi = Vec::new();
        for (q, part) in locations.iter().enumerate() {
            for (i, locs) in part.iter().enumerate() {
                if locs.len() > 1 {
                    for (j, c) in locs.iter().enumerate() {
                        if *c == CopyCheck::Valid {
                            multi.push((q, i, j));
                        }
                    }
                }
            }
        }
        if !multi.is_empty() {
            let need = ((multi.len() + t - 1) / t) * t * l;
            if self.prepass[slot].as_ref().map_or(true, |b| b.len() < need) {
                self.prepass[slot] = Some(HostBuffer::zeroed(need, self.dev0)?);
            }
            if let Some(buf) = self.prepass[slot].as_mut() {
                let (g, present, expected, mut ver) = Self::rows(t, l, &multi, &copies, first, digests, buf);
                self.multi.verify(buf, &present, &expected, g, &mut ver)?;
                for (x, &(q, i, j)) in multi.iter().enumerate() {
                    locations[q][i][j] = if ver[x] != 0 { CopyCheck::Valid } else { CopyCheck::Invalid };
                }
            }
        }
        let mut single = Vec::new();
        {
            let ch: &mut [u8] = &mut self.chunks[slot];
            let pres = &mut self.present[slot];
            let exp = &mut self.expected[slot];
            for q in 0..cnt {
                for i in 0..t {
                    let x = q * t + i;
                    exp[x * 32..(x + 1) * 32].copy_from_slice(&digests[(first + q) * t + i]);
                    pres[x] = 0;
                    let locs = &locations[q][i];
                    // a lone copy is hashed by the resilver job; a chunk with several locations
                    // brings its first valid copy, already verified
                    let pick = match locs.iter().position(|c| *c == CopyCheck::Valid) {
                        Some(j) if locs.len() == 1 => Some((j, 1u8)),
                        Some(j) => Some((j, crate::sys::CEC_PRESENT_VERIFIED)),
                        None => None,
                    };
                    if let Some((j, flag)) = pick {
                        if let Some(b) = &copies[q][i][j] {
                            ch[x * l..(x + 1) * l].copy_from_slice(b);
                            pres[x] = flag;
                            if flag == 1 {
                                single.push((q, i));
                            }
                        }
                    }
                }
            }
        }
        let job = unsafe {
            self.multi.submit_resilver(
                self.chunks[slot].as_ptr(),
                self.present[slot].as_ptr(),
                self.expected[slot].as_ptr(),
                cnt,
                self.rebuilt[slot].as_mut_ptr(),
                self.verified[slot].as_mut_ptr(),
                self.status[slot].as_mut_ptr(),
            )
        }?;
        Ok(LiveCheck { slot, job: Some(job), first, n: cnt, locations, items: Vec::new(), single,
                       present: Vec::new(), expected: Vec::new(), ver: Vec::new() })
    }

    fn collect_resilver<S, E>(&mut self, mut w: LiveCheck, base: usize, sink: &mut S)
        -> Result<(), BatchReadError<E>>
    where
        S: FnMut(&CheckedPart<'_>) -> Result<(), E>,
    {
        if let Some(job) = w.job {
            self.multi.wait(job).map_err(BatchReadError::Engine)?;
        }
        let (t, l) = (self.t, self.chunk_size);
        let ver = &self.verified[w.slot];
        for &(q, i) in &w.single {
            w.locations[q][i][0] = if ver[q * t + i] != 0 { CopyCheck::Valid } else { CopyCheck::Invalid };
        }
        let rebuilt: &[u8] = &self.rebuilt[w.slot];
        for (q, locations) in w.locations.into_iter().enumerate() {
            let missing: Vec<usize> = (0..t).filter(|&i| ver[q * t + i] == 0).collect();
            let mut part = CheckedPart { index: base + w.first + q, locations, rebuilt: Vec::new(), error: None };
            if !missing.is_empty() {
                match crate::check(self.status[w.slot][q]) {
                    // this part's write_error; the other parts go on (file_reference.rs:103-110)
                    Err(e @ CecError::Erasure(_)) => part.error = Some(e),
                    Err(e) => return Err(BatchReadError::Engine(e)),
                    Ok(()) => {
                        part.rebuilt = missing
                            .into_iter()
                            .map(|i| (i, &rebuilt[(q * t + i) * l..(q * t + i + 1) * l]))
                            .collect();
                    },
                }
            }
            sink(&part).map_err(BatchReadError::Sink)?;
        }
        Ok(())
    }

    /// Waits for a window's job without handing out its parts (error paths).
    fn drain(&self, w: Option<LiveCheck>) {
        if let Some(LiveCheck { job: Some(job), .. }) = w {
            let _ = self.multi.wait(job);
        }
    }
}

/// `FileReference::verify` / `resilver` over a whole file: consecutive parts of one shape through
/// a [`BatchChecker`] of that shape (kept for later files, the `keep` most recently used), a lone
/// part (the short last part) through a checker of one part per window.  Reports reach the sink
/// in file order with file part numbers.
pub struct FileChecker {
    parts_per_batch: usize,
    depth: usize,
    devices: Vec<c_int>,
    checkers: ShapeCache<(Shape, usize), BatchChecker>,
}

impl FileChecker {
    pub fn new(parts_per_batch: usize, depth: usize, devices: &[c_int], keep: usize) -> FileChecker {
        FileChecker { parts_per_batch, depth, devices: devices.to_vec(), checkers: ShapeCache::new(keep) }
    }

    pub fn verify<R, S, E>(&mut self, shapes: &[Shape], digests: &[[u8; 32]], read_all: R, sink: S)
        -> Result<(), BatchReadError<E>>
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
        S: FnMut(&CheckedPart<'_>) -> Result<(), E>,
    {
        self.runs(shapes, digests, read_all, sink, false)
    }

    pub fn resilver<R, S, E>(&mut self, shapes: &[Shape], digests: &[[u8; 32]], read_all: R, sink: S)
        -> Result<(), BatchReadError<E>>
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
        S: FnMut(&CheckedPart<'_>) -> Result<(), E>,
    {
        self.runs(shapes, digests, read_all, sink, true)
    }

    fn runs<R, S, E>(&mut self, shapes: &[Shape], digests: &[[u8; 32]], mut read_all: R, mut sink: S,
                     resilver: bool) -> Result<(), BatchReadError<E>>
    where
        R: FnMut(usize, usize) -> Vec<Option<Vec<u8>>>,
        S: FnMut(&CheckedPart<'_>) -> Result<(), E>,
    {
        let mut offsets = Vec::with_capacity(shapes.len());
        let mut base = 0usize;
        for &(d, p, _) in shapes {
            offsets.push(base);
            base += d + p;
        }
        if digests.len() < base {
            return Err(BatchReadError::Engine(crate::too_small("digests")));
        }
        let depth = self.depth;
        for (k0, n) in shape_runs(shapes, 0, shapes.len()) {
            let (d, p, l) = shapes[k0];
            let ppb = if n > 1 { self.parts_per_batch } else { 1 };
            let devices = &self.devices;
            // a lone part's checker has one-part windows: the window size is part of the key
            let checker = self.checkers.get(((d, p, l), ppb), || {
                BatchChecker::new(d, p, l, ppb, depth, devices)
            }).map_err(BatchReadError::Engine)?;
            let dig = &digests[offsets[k0]..offsets[k0] + n * (d + p)];
            let read = |q: usize, i: usize| read_all(k0 + q, i);
            checker.run(k0, n, dig, read, &mut sink, resilver)?;
        }
        Ok(())
    }
}
