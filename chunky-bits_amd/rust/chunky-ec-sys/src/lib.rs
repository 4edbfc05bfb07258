//! Rust side of the drop-in boundary (include/chunky_ec.h).
//!
//! `sys` mirrors the C-ABI one-to-one; [`ReedSolomon`] and [`sha256`] reproduce the surface of
//! `reed_solomon_erasure::ReedSolomon<galois_8::Field>` and `sha2::Sha256::digest` that
//! Chunky Bits calls (src/file/file_part.rs:77,128,161-165,185,302-304), returning the crate's
//! own `reed_solomon_erasure::Error` so `FileWriteError::Erasure` / `FileReadError::Erasure`
//! keep working unchanged.  Written against the header; compile-checked only where `cargo` is
//! available (not in the build container — see DESIGN.md).
use std::os::raw::{c_int, c_void};

pub mod sys {
    use super::*;

    #[repr(C)]
    pub struct cec_codec {
        _private: [u8; 0],
    }

    #[repr(C)]
    pub struct cec_pipeline {
        _private: [u8; 0],
    }

    #[repr(C)]
    pub struct cec_read_pipeline {
        _private: [u8; 0],
    }

    /// cec_read_pipeline_new_ex flag: only rebuilt data chunks come back over PCIe.
    pub const CEC_READ_REBUILT_ONLY: std::os::raw::c_uint = 1;

    #[repr(C)]
    #[derive(Clone, Copy, Debug)]
    pub struct cec_part_batch {
        pub base: *mut u8,
        pub part_stride: usize,
        pub chunk_stride: usize,
        pub n_parts: usize,
        pub chunk_len: usize,
    }

    extern "C" {
        pub fn cec_abi_version() -> c_int;
        pub fn cec_status_name(status: c_int) -> *const std::os::raw::c_char;
        pub fn cec_last_error() -> *const std::os::raw::c_char;
        pub fn cec_device_count() -> c_int;
        pub fn cec_codec_new(d: usize, p: usize, out: *mut *mut cec_codec) -> c_int;
        pub fn cec_codec_free(codec: *mut cec_codec);
        pub fn cec_codec_data_shards(codec: *const cec_codec) -> usize;
        pub fn cec_codec_parity_shards(codec: *const cec_codec) -> usize;
        pub fn cec_codec_total_shards(codec: *const cec_codec) -> usize;
        pub fn cec_codec_matrix(codec: *const cec_codec, out: *mut u8, out_len: usize) -> c_int;
        pub fn cec_encode_sep(
            codec: *const cec_codec,
            data: *const *const u8,
            data_lens: *const usize,
            n_data: usize,
            parity: *const *mut u8,
            parity_lens: *const usize,
            n_parity: usize,
        ) -> c_int;
        pub fn cec_reconstruct(
            codec: *const cec_codec,
            shards: *const *mut u8,
            shard_lens: *const usize,
            present: *mut u8,
            n_shards: usize,
        ) -> c_int;
        pub fn cec_reconstruct_data(
            codec: *const cec_codec,
            shards: *const *mut u8,
            shard_lens: *const usize,
            present: *mut u8,
            n_shards: usize,
        ) -> c_int;
        pub fn cec_sha256(buf: *const u8, len: usize, out32: *mut u8) -> c_int;
        pub fn cec_sha256_many(
            bufs: *const *const u8,
            lens: *const usize,
            n: usize,
            out: *mut u8,
        ) -> c_int;
        pub fn cec_part_encode(
            codec: *const cec_codec,
            data_buf: *const u8,
            length: usize,
            parity_out: *mut u8,
            digests_out: *mut u8,
            chunksize: *mut usize,
        ) -> c_int;
        pub fn cec_encode_batch(
            codec: *const cec_codec,
            batch: *const cec_part_batch,
            stream: *mut c_void,
        ) -> c_int;
        pub fn cec_encode_hash_batch(
            codec: *const cec_codec,
            batch: *const cec_part_batch,
            digests: *mut u8,
            stream: *mut c_void,
        ) -> c_int;
        pub fn cec_sha256_batch(
            batch: *const cec_part_batch,
            first_chunk: usize,
            n_chunks: usize,
            digests: *mut u8,
            stream: *mut c_void,
        ) -> c_int;
        pub fn cec_reconstruct_batch(
            codec: *const cec_codec,
            batch: *const cec_part_batch,
            present: *const u8,
            data_only: c_int,
            stream: *mut c_void,
        ) -> c_int;
        pub fn cec_verify_batch(
            batch: *const cec_part_batch,
            first_chunk: usize,
            n_chunks: usize,
            present: *const u8,
            expected: *const u8,
            ok: *mut u8,
            stream: *mut c_void,
        ) -> c_int;
        pub fn cec_read_batch(
            codec: *const cec_codec,
            batch: *const cec_part_batch,
            present: *const u8,
            expected: *const u8,
            verified: *mut u8,
            part_status: *mut c_int,
            stream: *mut c_void,
        ) -> c_int;
        pub fn cec_resilver_batch(
            codec: *const cec_codec,
            batch: *const cec_part_batch,
            present: *const u8,
            expected: *const u8,
            verified: *mut u8,
            part_status: *mut c_int,
            stream: *mut c_void,
        ) -> c_int;
        pub fn cec_pipeline_new(
            codec: *const cec_codec,
            chunk_len: usize,
            parts_per_batch: usize,
            depth: usize,
            out: *mut *mut cec_pipeline,
        ) -> c_int;
        pub fn cec_pipeline_free(pipeline: *mut cec_pipeline);
        pub fn cec_pipeline_depth(pipeline: *const cec_pipeline) -> usize;
        pub fn cec_pipeline_acquire(
            pipeline: *mut cec_pipeline,
            slot: *mut usize,
            data: *mut *mut u8,
        ) -> c_int;
        pub fn cec_pipeline_submit(pipeline: *mut cec_pipeline, slot: usize, n_parts: usize) -> c_int;
        pub fn cec_pipeline_wait(
            pipeline: *mut cec_pipeline,
            slot: usize,
            parity: *mut *const u8,
            digests: *mut *const u8,
            n_parts: *mut usize,
        ) -> c_int;
        pub fn cec_pipeline_drain(pipeline: *mut cec_pipeline) -> c_int;
        pub fn cec_pipeline_last_error() -> *const std::os::raw::c_char;
        pub fn cec_read_pipeline_new(
            codec: *const cec_codec,
            chunk_len: usize,
            parts_per_batch: usize,
            depth: usize,
            out: *mut *mut cec_read_pipeline,
        ) -> c_int;
        pub fn cec_read_pipeline_free(pipeline: *mut cec_read_pipeline);
        pub fn cec_read_pipeline_depth(pipeline: *const cec_read_pipeline) -> usize;
        pub fn cec_read_pipeline_acquire(
            pipeline: *mut cec_read_pipeline,
            slot: *mut usize,
            chunks: *mut *mut u8,
            present: *mut *mut u8,
            expected: *mut *mut u8,
        ) -> c_int;
        pub fn cec_read_pipeline_submit(
            pipeline: *mut cec_read_pipeline,
            slot: usize,
            n_parts: usize,
        ) -> c_int;
        pub fn cec_read_pipeline_wait(
            pipeline: *mut cec_read_pipeline,
            slot: usize,
            data: *mut *const u8,
            verified: *mut *const u8,
            part_status: *mut *const c_int,
            n_parts: *mut usize,
        ) -> c_int;
        pub fn cec_read_pipeline_drain(pipeline: *mut cec_read_pipeline) -> c_int;
        pub fn cec_read_pipeline_new_ex(
            codec: *const cec_codec,
            chunk_len: usize,
            parts_per_batch: usize,
            depth: usize,
            flags: std::os::raw::c_uint,
            out: *mut *mut cec_read_pipeline,
        ) -> c_int;
        pub fn cec_read_pipeline_data_chunks(
            pipeline: *mut cec_read_pipeline,
            slot: usize,
            ptrs: *mut *const u8,
        ) -> c_int;
        pub fn cec_coalesce_stats(calls: *mut u64, launches: *mut u64);
    }
}

pub use reed_solomon_erasure::Error;

/// Engine failures with no crate equivalent (no GPU, HIP error, allocation failure).
#[derive(Debug)]
pub struct EngineError {
    pub code: c_int,
    pub message: String,
}

/// Error of a call through the boundary: a crate error (codes 1..13) or an engine error.
#[derive(Debug)]
pub enum CecError {
    Erasure(Error),
    Engine(EngineError),
}

impl From<CecError> for Error {
    /// For call sites typed `Result<_, reed_solomon_erasure::Error>`; engine errors have no
    /// crate variant and abort loudly instead of being disguised as one.
    fn from(e: CecError) -> Error {
        match e {
            CecError::Erasure(e) => e,
            CecError::Engine(e) => panic!("chunky_ec engine error {}: {}", e.code, e.message),
        }
    }
}

fn check(code: c_int) -> Result<(), CecError> {
    Err(CecError::Erasure(match code {
        0 => return Ok(()),
        1 => Error::TooFewShards,
        2 => Error::TooManyShards,
        3 => Error::TooFewDataShards,
        4 => Error::TooManyDataShards,
        5 => Error::TooFewParityShards,
        6 => Error::TooManyParityShards,
        7 => Error::TooFewBufferShards,
        8 => Error::TooManyBufferShards,
        9 => Error::IncorrectShardSize,
        10 => Error::TooFewShardsPresent,
        11 => Error::EmptyShard,
        12 => Error::InvalidShardFlags,
        13 => Error::InvalidIndex,
        other => {
            let message = unsafe { std::ffi::CStr::from_ptr(sys::cec_last_error()) }
                .to_string_lossy()
                .into_owned();
            return Err(CecError::Engine(EngineError { code: other, message }));
        },
    }))
}

/// As [`check`], with the pipeline's own message for engine errors.
fn check_pipe(code: c_int) -> Result<(), CecError> {
    match check(code) {
        Err(CecError::Engine(mut e)) => {
            e.message = unsafe { std::ffi::CStr::from_ptr(sys::cec_pipeline_last_error()) }
                .to_string_lossy()
                .into_owned();
            Err(CecError::Engine(e))
        },
        other => other,
    }
}

/// `ReedSolomon<galois_8::Field>` backed by the gfx950 kernels.  Immutable after `new`, so it
/// is `Send + Sync` and can be shared through `Arc` exactly like the crate's (writer.rs:131).
pub struct ReedSolomon {
    raw: *mut sys::cec_codec,
}

unsafe impl Send for ReedSolomon {}
unsafe impl Sync for ReedSolomon {}

impl Drop for ReedSolomon {
    fn drop(&mut self) {
        unsafe { sys::cec_codec_free(self.raw) }
    }
}

impl ReedSolomon {
    pub fn new(data_shards: usize, parity_shards: usize) -> Result<ReedSolomon, Error> {
        let mut raw = std::ptr::null_mut();
        check(unsafe { sys::cec_codec_new(data_shards, parity_shards, &mut raw) })?;
        Ok(ReedSolomon { raw })
    }

    pub fn data_shard_count(&self) -> usize {
        unsafe { sys::cec_codec_data_shards(self.raw) }
    }

    pub fn parity_shard_count(&self) -> usize {
        unsafe { sys::cec_codec_parity_shards(self.raw) }
    }

    pub fn total_shard_count(&self) -> usize {
        unsafe { sys::cec_codec_total_shards(self.raw) }
    }

    /// `encode_sep::<T, U>(&data, &mut parity)`.
    pub fn encode_sep<T: AsRef<[u8]>, U: AsRef<[u8]> + AsMut<[u8]>>(
        &self,
        data: &[T],
        parity: &mut [U],
    ) -> Result<(), Error> {
        let dptr: Vec<*const u8> = data.iter().map(|d| d.as_ref().as_ptr()).collect();
        let dlen: Vec<usize> = data.iter().map(|d| d.as_ref().len()).collect();
        let plen: Vec<usize> = parity.iter().map(|p| p.as_ref().len()).collect();
        let pptr: Vec<*mut u8> = parity.iter_mut().map(|p| p.as_mut().as_mut_ptr()).collect();
        check(unsafe {
            sys::cec_encode_sep(
                self.raw,
                dptr.as_ptr(),
                dlen.as_ptr(),
                dptr.len(),
                pptr.as_ptr(),
                plen.as_ptr(),
                pptr.len(),
            )
        })?;
        Ok(())
    }

    fn reconstruct_inner(&self, shards: &mut [Option<Vec<u8>>], data_only: bool) -> Result<(), Error> {
        // The crate allocates missing slots zeroed at the present length; do the same so the
        // engine writes straight into the caller's Vec.
        let len = shards.iter().flatten().map(|s| s.len()).find(|&l| l > 0).unwrap_or(0);
        let mut present: Vec<u8> = shards.iter().map(|s| s.is_some() as u8).collect();
        let d = self.data_shard_count();
        let mut scratch: Vec<Option<Vec<u8>>> = shards
            .iter()
            .enumerate()
            .map(|(i, s)| match s {
                None if !(data_only && i >= d) => Some(vec![0u8; len]),
                _ => None,
            })
            .collect();
        let ptrs: Vec<*mut u8> = shards
            .iter_mut()
            .zip(scratch.iter_mut())
            .map(|(s, t)| match (s, t) {
                (Some(v), _) => v.as_mut_ptr(),
                (None, Some(v)) => v.as_mut_ptr(),
                (None, None) => std::ptr::null_mut(),
            })
            .collect();
        let lens: Vec<usize> = shards
            .iter()
            .zip(scratch.iter())
            .map(|(s, t)| s.as_ref().or(t.as_ref()).map(|v| v.len()).unwrap_or(0))
            .collect();
        let f = if data_only { sys::cec_reconstruct_data } else { sys::cec_reconstruct };
        check(unsafe { f(self.raw, ptrs.as_ptr(), lens.as_ptr(), present.as_mut_ptr(), ptrs.len()) })?;
        for (i, slot) in shards.iter_mut().enumerate() {
            if slot.is_none() && present[i] != 0 {
                *slot = scratch[i].take();
            }
        }
        Ok(())
    }

    /// `reconstruct(&mut shards)`: rebuilds missing data and parity.
    pub fn reconstruct(&self, shards: &mut [Option<Vec<u8>>]) -> Result<(), Error> {
        self.reconstruct_inner(shards, false)
    }

    /// `reconstruct_data(&mut shards)`: rebuilds missing data only.
    pub fn reconstruct_data(&self, shards: &mut [Option<Vec<u8>>]) -> Result<(), Error> {
        self.reconstruct_inner(shards, true)
    }

    pub fn as_raw(&self) -> *const sys::cec_codec {
        self.raw
    }
}

/// `Sha256::digest(buf)` (sha256.rs:20-26) computed on the GPU.
pub fn sha256(buf: &[u8]) -> [u8; 32] {
    let mut out = [0u8; 32];
    check(unsafe { sys::cec_sha256(buf.as_ptr(), buf.len(), out.as_mut_ptr()) })
        .map_err(Error::from)
        .expect("cec_sha256");
    out
}

/// `FilePart::write_with_encoder`'s compute for one part: (chunksize, parity chunks, d+p digests).
pub fn part_encode(
    codec: &ReedSolomon,
    data_buf: &[u8],
    length: usize,
) -> Result<(usize, Vec<Vec<u8>>, Vec<[u8; 32]>), Error> {
    let d = codec.data_shard_count();
    let p = codec.parity_shard_count();
    let l = (length + d - 1) / d;
    let mut parity = vec![0u8; p * l];
    let mut digests = vec![0u8; 32 * (d + p)];
    let mut chunksize = 0usize;
    check(unsafe {
        sys::cec_part_encode(
            codec.raw,
            data_buf.as_ptr(),
            length,
            parity.as_mut_ptr(),
            digests.as_mut_ptr(),
            &mut chunksize,
        )
    })?;
    let parity = parity.chunks(l.max(1)).map(|c| c.to_vec()).take(p).collect();
    let digests = digests
        .chunks(32)
        .map(|c| {
            let mut a = [0u8; 32];
            a.copy_from_slice(c);
            a
        })
        .collect();
    Ok((chunksize, parity, digests))
}

/// Batched `FileWriteBuilder::write` compute (writer.rs:166-231): `depth` slots of
/// `parts_per_batch` parts each, pinned host buffers, one HIP stream per slot.  One thread
/// drives a pipeline (it is `Send`, not `Sync`).  Per slot: [`acquire`](Self::acquire) hands
/// out the pinned `[parts][d][chunk_len]` input area (each part's zero-padded `data_buf`,
/// writer.rs:172-197), [`submit`](Self::submit) queues H2D + fused encode/SHA-256 + D2H, and
/// [`wait`](Self::wait) returns the parity chunks and the d+p digests of every part, in order.
pub struct WritePipeline {
    raw: *mut sys::cec_pipeline,
    d: usize,
    p: usize,
    chunk_len: usize,
}

unsafe impl Send for WritePipeline {}

impl Drop for WritePipeline {
    fn drop(&mut self) {
        unsafe { sys::cec_pipeline_free(self.raw) }
    }
}

/// One completed batch: parity `[parts][p][chunk_len]` and digests `[parts][d+p][32]`
/// (pinned host memory owned by the pipeline slot until it is acquired again).
pub struct BatchResult<'a> {
    pub parity: &'a [u8],
    pub digests: &'a [u8],
    pub n_parts: usize,
}

impl WritePipeline {
    pub fn new(
        codec: &ReedSolomon,
        chunk_len: usize,
        parts_per_batch: usize,
        depth: usize,
    ) -> Result<WritePipeline, CecError> {
        let mut raw = std::ptr::null_mut();
        check_pipe(unsafe { sys::cec_pipeline_new(codec.raw, chunk_len, parts_per_batch, depth, &mut raw) })?;
        Ok(WritePipeline {
            raw,
            d: codec.data_shard_count(),
            p: codec.parity_shard_count(),
            chunk_len,
        })
    }

    pub fn depth(&self) -> usize {
        unsafe { sys::cec_pipeline_depth(self.raw) }
    }

    /// Next free slot (waits for its previous batch) and its pinned input area.
    pub fn acquire(&mut self, parts_per_batch: usize) -> Result<(usize, &mut [u8]), CecError> {
        let mut slot = 0usize;
        let mut data = std::ptr::null_mut();
        check_pipe(unsafe { sys::cec_pipeline_acquire(self.raw, &mut slot, &mut data) })?;
        let len = parts_per_batch * self.d * self.chunk_len;
        Ok((slot, unsafe { std::slice::from_raw_parts_mut(data, len) }))
    }

    /// Queue the first `n_parts` parts of `slot` (asynchronous).
    pub fn submit(&mut self, slot: usize, n_parts: usize) -> Result<(), CecError> {
        check_pipe(unsafe { sys::cec_pipeline_submit(self.raw, slot, n_parts) })
    }

    /// Wait for `slot`'s batch and borrow its parity and digests.
    pub fn wait(&mut self, slot: usize) -> Result<BatchResult<'_>, CecError> {
        let mut parity = std::ptr::null();
        let mut digests = std::ptr::null();
        let mut n_parts = 0usize;
        check_pipe(unsafe { sys::cec_pipeline_wait(self.raw, slot, &mut parity, &mut digests, &mut n_parts) })?;
        let plen = n_parts * self.p * self.chunk_len;
        let dlen = n_parts * (self.d + self.p) * 32;
        Ok(BatchResult {
            parity: unsafe { std::slice::from_raw_parts(parity, plen) },
            digests: unsafe { std::slice::from_raw_parts(digests, dlen) },
            n_parts,
        })
    }

    /// Wait for every submitted batch.
    pub fn drain(&mut self) -> Result<(), CecError> {
        check_pipe(unsafe { sys::cec_pipeline_drain(self.raw) })
    }
}

/// Batched `FileReadBuilder` / `FilePart::read_with_context` compute (reader.rs:40-75,
/// file_part.rs:73-135) over pinned slots: the caller writes the chunks it loaded, their
/// loaded flags and the metadata digests; the engine verifies every loaded chunk, rebuilds the
/// d data chunks from verified ones, and returns the part bytes, the flags and a per-part
/// status (`Error::TooFewShardsPresent` when fewer than d verify).
pub struct ReadPipeline {
    raw: *mut sys::cec_read_pipeline,
    d: usize,
    t: usize,
    chunk_len: usize,
    parts: usize,
}

unsafe impl Send for ReadPipeline {}

impl Drop for ReadPipeline {
    fn drop(&mut self) {
        unsafe { sys::cec_read_pipeline_free(self.raw) }
    }
}

/// A slot's input areas: chunks `[parts][d+p][chunk_len]`, present `[parts][d+p]`,
/// expected digests `[parts][d+p][32]`.
pub struct ReadSlotInput<'a> {
    pub slot: usize,
    pub chunks: &'a mut [u8],
    pub present: &'a mut [u8],
    pub expected: &'a mut [u8],
}

/// A completed read batch: data `[parts][d][chunk_len]`, verified `[parts][d+p]`, statuses.
pub struct ReadBatchResult<'a> {
    pub data: &'a [u8],
    pub verified: &'a [u8],
    pub part_status: Vec<Result<(), Error>>,
}

impl ReadPipeline {
    pub fn new(
        codec: &ReedSolomon,
        chunk_len: usize,
        parts_per_batch: usize,
        depth: usize,
    ) -> Result<ReadPipeline, CecError> {
        let mut raw = std::ptr::null_mut();
        check_pipe(unsafe {
            sys::cec_read_pipeline_new(codec.raw, chunk_len, parts_per_batch, depth, &mut raw)
        })?;
        Ok(ReadPipeline {
            raw,
            d: codec.data_shard_count(),
            t: codec.total_shard_count(),
            chunk_len,
            parts: parts_per_batch,
        })
    }

    pub fn depth(&self) -> usize {
        unsafe { sys::cec_read_pipeline_depth(self.raw) }
    }

    pub fn acquire(&mut self) -> Result<ReadSlotInput<'_>, CecError> {
        let (mut slot, mut c, mut p, mut e) =
            (0usize, std::ptr::null_mut(), std::ptr::null_mut(), std::ptr::null_mut());
        check_pipe(unsafe { sys::cec_read_pipeline_acquire(self.raw, &mut slot, &mut c, &mut p, &mut e) })?;
        let n = self.parts * self.t;
        Ok(ReadSlotInput {
            slot,
            chunks: unsafe { std::slice::from_raw_parts_mut(c, n * self.chunk_len) },
            present: unsafe { std::slice::from_raw_parts_mut(p, n) },
            expected: unsafe { std::slice::from_raw_parts_mut(e, n * 32) },
        })
    }

    pub fn submit(&mut self, slot: usize, n_parts: usize) -> Result<(), CecError> {
        check_pipe(unsafe { sys::cec_read_pipeline_submit(self.raw, slot, n_parts) })
    }

    pub fn wait(&mut self, slot: usize) -> Result<ReadBatchResult<'_>, CecError> {
        let (mut data, mut ver) = (std::ptr::null(), std::ptr::null());
        let mut status: *const c_int = std::ptr::null();
        let mut n = 0usize;
        check_pipe(unsafe {
            sys::cec_read_pipeline_wait(self.raw, slot, &mut data, &mut ver, &mut status, &mut n)
        })?;
        let codes = unsafe { std::slice::from_raw_parts(status, n) };
        Ok(ReadBatchResult {
            data: unsafe { std::slice::from_raw_parts(data, n * self.d * self.chunk_len) },
            verified: unsafe { std::slice::from_raw_parts(ver, n * self.t) },
            part_status: codes
                .iter()
                .map(|&c| check(c).map_err(Error::from))
                .collect(),
        })
    }

    pub fn drain(&mut self) -> Result<(), CecError> {
        check_pipe(unsafe { sys::cec_read_pipeline_drain(self.raw) })
    }

    /// As [`ReadPipeline::new`] with `CEC_READ_REBUILT_ONLY`: only the rebuilt data chunks come
    /// back over PCIe; read a part's bytes through [`ReadPipeline::data_chunks`].
    pub fn new_rebuilt_only(
        codec: &ReedSolomon,
        chunk_len: usize,
        parts_per_batch: usize,
        depth: usize,
    ) -> Result<ReadPipeline, CecError> {
        let mut raw = std::ptr::null_mut();
        check_pipe(unsafe {
            sys::cec_read_pipeline_new_ex(
                codec.raw,
                chunk_len,
                parts_per_batch,
                depth,
                sys::CEC_READ_REBUILT_ONLY,
                &mut raw,
            )
        })?;
        Ok(ReadPipeline {
            raw,
            d: codec.data_shard_count(),
            t: codec.total_shard_count(),
            chunk_len,
            parts: parts_per_batch,
        })
    }

    /// The d data chunks of each of the slot's `n_parts` parts (`[part][chunk]`), wherever they
    /// are (the slot's chunk buffer or the rebuilt buffer); valid until the slot is re-acquired.
    /// `read_with_context`'s output is their concatenation (file_part.rs:130-133).
    pub fn data_chunks(&mut self, slot: usize, n_parts: usize) -> Result<Vec<Vec<&[u8]>>, CecError> {
        let mut ptrs = vec![std::ptr::null::<u8>(); n_parts * self.d];
        check_pipe(unsafe { sys::cec_read_pipeline_data_chunks(self.raw, slot, ptrs.as_mut_ptr()) })?;
        Ok(ptrs
            .chunks(self.d)
            .map(|part| {
                part.iter()
                    .map(|&p| unsafe { std::slice::from_raw_parts(p, self.chunk_len) })
                    .collect()
            })
            .collect())
    }
}
