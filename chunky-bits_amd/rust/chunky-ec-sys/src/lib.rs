//! Rust side of the drop-in boundary (include/chunky_ec.h).
//!
//! `sys` mirrors the C-ABI one-to-one; [`ReedSolomon`] and [`sha256`] reproduce the surface of
//! `reed_solomon_erasure::ReedSolomon<galois_8::Field>` and `sha2::Sha256::digest` that
//! Chunky Bits calls (src/file/file_part.rs:77,128,161-165,185,302-304), returning the crate's
//! own `reed_solomon_erasure::Error` so `FileWriteError::Erasure` / `FileReadError::Erasure`
//! keep working unchanged.  Written against the header; compile-checked only where `cargo` is
//! available (not in the build container — see DESIGN.md).
use std::os::raw::{c_int, c_void};

pub mod batch;

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

    #[repr(C)]
    pub struct cec_multi {
        _private: [u8; 0],
    }

    pub const CEC_ABI_VERSION: c_int = 3;
    /// cec_read_pipeline_new_ex / cec_multi_read flag: only rebuilt data chunks come back.
    pub const CEC_READ_REBUILT_ONLY: std::os::raw::c_uint = 1;
    /// cec_read_pipeline_new_ex flag: FilePart::resilver's compute (data and parity rebuilt).
    pub const CEC_READ_RESILVER: std::os::raw::c_uint = 4;
    /// cec_read_pipeline_new_ex flag: FilePart::verify's compute (hash and compare only).
    pub const CEC_READ_VERIFY_ONLY: std::os::raw::c_uint = 8;
    /// cec_pipeline_new_ex / cec_read_pipeline_new_ex flag: batches come from caller buffers.
    pub const CEC_PIPE_EXTERNAL: std::os::raw::c_uint = 2;
    /// Present-flag value of a read retry: loaded and already verified (not hashed again).
    pub const CEC_PRESENT_VERIFIED: u8 = 0x80;
    /// Read-pipeline flag: keep retries' verified chunks on the device (carry pool).
    pub const CEC_READ_CARRY: std::os::raw::c_uint = 16;
    /// cec_read_submit flag: the chunks are packed back to back (one upload).
    pub const CEC_SUBMIT_PACKED: std::os::raw::c_uint = 32;
    /// cec_multi_new_ex job kinds.
    pub const CEC_MULTI_WRITE: std::os::raw::c_uint = 1;
    pub const CEC_MULTI_READ: std::os::raw::c_uint = 2;
    /// cec_multi_read(_carry) flag: the job goes ahead of the queued jobs not yet started.
    pub const CEC_MULTI_AHEAD: std::os::raw::c_uint = 64;
    /// Status of a part with fewer than d verified chunks (retry it with more).
    pub const CEC_TOO_FEW_SHARDS_PRESENT: c_int = 10;

    /// cec_read_pipeline_submit_ex's arguments (include/chunky_ec.h).
    #[repr(C)]
    #[derive(Clone, Copy, Debug)]
    pub struct cec_read_submit {
        pub chunks: *const u8,
        pub present: *const u8,
        pub expected: *const u8,
        pub n_parts: usize,
        pub data_out: *mut u8,
        pub carry_ids: *const i32,
        pub flags: std::os::raw::c_uint,
    }

    /// cec_multi_shard_stats's counters (include/chunky_ec.h).
    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default)]
    pub struct cec_multi_stats {
        pub device: c_int,
        pub numa_node: c_int,
        pub parts: u64,
        pub pipelines_made: u64,
        pub chunks_uploaded: u64,
        pub chunks_carried: u64,
        pub carry_held: u64,
    }

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
        pub fn cec_read_pipeline_acquire_idle(
            pipeline: *mut cec_read_pipeline,
            slot: *mut usize,
            chunks: *mut *mut u8,
            present: *mut *mut u8,
            expected: *mut *mut u8,
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
            capacity: usize,
        ) -> c_int;
        pub fn cec_coalesce_stats(calls: *mut u64, launches: *mut u64);
        pub fn cec_build_info() -> *const std::os::raw::c_char;
        pub fn cec_build_id() -> *const std::os::raw::c_char;
        pub fn cec_current_device(device: *mut c_int) -> c_int;
        pub fn cec_set_device(device: c_int) -> c_int;
        pub fn cec_device_numa_node(device: c_int) -> c_int;
        pub fn cec_codec_cached_patterns(codec: *const cec_codec) -> usize;
        pub fn cec_host_alloc(bytes: usize, device: c_int, out: *mut *mut c_void) -> c_int;
        pub fn cec_host_free(ptr: *mut c_void);
        pub fn cec_host_is_pinned(ptr: *const c_void, bytes: usize) -> c_int;
        pub fn cec_host_numa_node(ptr: *const c_void) -> c_int;
        pub fn cec_bind_thread_to_device_node(device: c_int) -> c_int;
        pub fn cec_pipeline_new_ex(
            codec: *const cec_codec,
            chunk_len: usize,
            parts_per_batch: usize,
            depth: usize,
            flags: std::os::raw::c_uint,
            out: *mut *mut cec_pipeline,
        ) -> c_int;
        pub fn cec_pipeline_submit_from(
            pipeline: *mut cec_pipeline,
            slot: usize,
            data: *const u8,
            n_parts: usize,
            parity_out: *mut u8,
            digests_out: *mut u8,
        ) -> c_int;
        pub fn cec_pipeline_query(pipeline: *mut cec_pipeline, slot: usize) -> c_int;
        pub fn cec_read_pipeline_submit_from(
            pipeline: *mut cec_read_pipeline,
            slot: usize,
            chunks: *const u8,
            present: *const u8,
            expected: *const u8,
            n_parts: usize,
            data_out: *mut u8,
        ) -> c_int;
        pub fn cec_read_pipeline_submit_packed(
            pipeline: *mut cec_read_pipeline,
            slot: usize,
            chunks: *const u8,
            present: *const u8,
            expected: *const u8,
            n_parts: usize,
            data_out: *mut u8,
        ) -> c_int;
        pub fn cec_read_pipeline_query(pipeline: *mut cec_read_pipeline, slot: usize) -> c_int;
        pub fn cec_read_pipeline_carry_ids(
            pipeline: *mut cec_read_pipeline,
            slot: usize,
            ids: *mut i32,
            capacity: usize,
        ) -> c_int;
        pub fn cec_read_pipeline_carry_held(pipeline: *const cec_read_pipeline) -> usize;
        pub fn cec_read_pipeline_submit_ex(
            pipeline: *mut cec_read_pipeline,
            slot: usize,
            submit: *const cec_read_submit,
        ) -> c_int;
        pub fn cec_pipelines_made() -> u64;
        pub fn cec_multi_new_ex(
            codec: *const cec_codec,
            chunk_len: usize,
            parts_per_batch: usize,
            depth: usize,
            devices: *const c_int,
            n_devices: usize,
            flags: std::os::raw::c_uint,
            out: *mut *mut cec_multi,
        ) -> c_int;
        pub fn cec_multi_read_carry(
            multi: *mut cec_multi,
            chunks: *const u8,
            present: *const u8,
            expected: *const u8,
            n_parts: usize,
            data: *mut u8,
            verified: *mut u8,
            part_status: *mut c_int,
            data_ptrs: *mut *const u8,
            flags: std::os::raw::c_uint,
            carry_in: *const i32,
            carry_out: *mut i32,
            job: *mut u64,
        ) -> c_int;
        pub fn cec_multi_carry_release(multi: *mut cec_multi, id: i32) -> c_int;
        pub fn cec_multi_shard_stats(multi: *mut cec_multi, g: usize, out: *mut cec_multi_stats) -> c_int;
        pub fn cec_read_pipeline_submit_carried(
            pipeline: *mut cec_read_pipeline,
            slot: usize,
            n_parts: usize,
            carry_ids: *const i32,
        ) -> c_int;
        pub fn cec_read_pipeline_carry_release(pipeline: *mut cec_read_pipeline, id: i32) -> c_int;
        pub fn cec_multi_new(
            codec: *const cec_codec,
            chunk_len: usize,
            parts_per_batch: usize,
            depth: usize,
            devices: *const c_int,
            n_devices: usize,
            out: *mut *mut cec_multi,
        ) -> c_int;
        pub fn cec_multi_free(multi: *mut cec_multi);
        pub fn cec_multi_shards(multi: *const cec_multi) -> usize;
        pub fn cec_multi_shard_info(
            multi: *mut cec_multi,
            g: usize,
            device: *mut c_int,
            numa_node: *mut c_int,
            parts: *mut u64,
        ) -> c_int;
        pub fn cec_multi_encode_hash(
            multi: *mut cec_multi,
            data: *const u8,
            n_parts: usize,
            parity: *mut u8,
            digests: *mut u8,
            job: *mut u64,
        ) -> c_int;
        pub fn cec_multi_read(
            multi: *mut cec_multi,
            chunks: *const u8,
            present: *const u8,
            expected: *const u8,
            n_parts: usize,
            data: *mut u8,
            verified: *mut u8,
            part_status: *mut c_int,
            data_ptrs: *mut *const u8,
            flags: std::os::raw::c_uint,
            job: *mut u64,
        ) -> c_int;
        pub fn cec_multi_resilver(
            multi: *mut cec_multi,
            chunks: *const u8,
            present: *const u8,
            expected: *const u8,
            n_parts: usize,
            rebuilt: *mut u8,
            verified: *mut u8,
            part_status: *mut c_int,
            chunk_ptrs: *mut *const u8,
            job: *mut u64,
        ) -> c_int;
        pub fn cec_multi_verify(
            multi: *mut cec_multi,
            chunks: *const u8,
            present: *const u8,
            expected: *const u8,
            n_parts: usize,
            verified: *mut u8,
            job: *mut u64,
        ) -> c_int;
        pub fn cec_multi_wait(multi: *mut cec_multi, job: u64) -> c_int;
        pub fn cec_multi_query(multi: *mut cec_multi, job: u64) -> c_int;
        pub fn cec_multi_last_error() -> *const std::os::raw::c_char;
        pub fn cec_fill_synthetic(
            batch: *const cec_part_batch,
            n_chunks: usize,
            seed: u64,
            stream: *mut c_void,
        ) -> c_int;
        pub fn cec_synth_byte(seed: u64, part: u64, chunk: u64, offset: u64) -> u8;
        pub fn cec_reload_knobs();
        pub fn cec_release_cached(device: c_int) -> usize;
    }
}

pub use reed_solomon_erasure::Error;

/// Engine failures with no crate equivalent (no GPU, HIP error, allocation failure).
#[derive(Debug)]
pub struct EngineError {
    pub code: c_int,
    pub message: String,
}

impl std::fmt::Display for EngineError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "chunky_ec engine error {}: {}", self.code, self.message)
    }
}

impl std::error::Error for EngineError {}

/// Error of a call through the boundary: a crate error (codes 1..13) or an engine error.
/// Every fallible call returns it; nothing in this crate panics on an engine failure (a HIP
/// out-of-memory inside a tokio part task surfaces as an error of that part).  The reference
/// side gains one variant per error type it returns:
/// `FileWriteError::Engine(EngineError)` / `FileReadError::Engine(EngineError)` with
/// `From<CecError>`, so `?` keeps working at every call site.
#[derive(Debug)]
pub enum CecError {
    Erasure(Error),
    Engine(EngineError),
}

impl std::fmt::Display for CecError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        match self {
            CecError::Erasure(e) => write!(f, "{:?}", e),
            CecError::Engine(e) => e.fmt(f),
        }
    }
}

impl std::error::Error for CecError {}

impl From<Error> for CecError {
    fn from(e: Error) -> CecError {
        CecError::Erasure(e)
    }
}

impl CecError {
    /// The crate error, if this is one (engine errors have no crate variant).
    pub fn erasure(&self) -> Option<Error> {
        match self {
            CecError::Erasure(e) => Some(*e),
            CecError::Engine(_) => None,
        }
    }
}

pub(crate) fn check(code: c_int) -> Result<(), CecError> {
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
    pub fn new(data_shards: usize, parity_shards: usize) -> Result<ReedSolomon, CecError> {
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
    ) -> Result<(), CecError> {
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

    fn reconstruct_inner(
        &self,
        shards: &mut [Option<Vec<u8>>],
        data_only: bool,
    ) -> Result<(), CecError> {
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
    pub fn reconstruct(&self, shards: &mut [Option<Vec<u8>>]) -> Result<(), CecError> {
        self.reconstruct_inner(shards, false)
    }

    /// `reconstruct_data(&mut shards)`: rebuilds missing data only.
    pub fn reconstruct_data(&self, shards: &mut [Option<Vec<u8>>]) -> Result<(), CecError> {
        self.reconstruct_inner(shards, true)
    }

    pub fn as_raw(&self) -> *const sys::cec_codec {
        self.raw
    }
}

/// `Sha256::digest(buf)` (sha256.rs:20-26) computed on the GPU.  Fallible where the CPU digest
/// is not: an engine failure is returned, never panicked on.
pub fn sha256(buf: &[u8]) -> Result<[u8; 32], CecError> {
    let mut out = [0u8; 32];
    check(unsafe { sys::cec_sha256(buf.as_ptr(), buf.len(), out.as_mut_ptr()) })?;
    Ok(out)
}

/// Many `Sha256::digest` calls in one launch (`cec_sha256_many`): the digest of every buffer, in
/// order.  Concurrent callers are coalesced like [`sha256`]'s.
pub fn sha256_many(bufs: &[&[u8]]) -> Result<Vec<[u8; 32]>, CecError> {
    if bufs.is_empty() {
        return Ok(Vec::new());
    }
    let ptrs: Vec<*const u8> = bufs.iter().map(|b| b.as_ptr()).collect();
    let lens: Vec<usize> = bufs.iter().map(|b| b.len()).collect();
    let mut out = vec![0u8; 32 * bufs.len()];
    check(unsafe { sys::cec_sha256_many(ptrs.as_ptr(), lens.as_ptr(), bufs.len(), out.as_mut_ptr()) })?;
    Ok(out
        .chunks(32)
        .map(|c| {
            let mut a = [0u8; 32];
            a.copy_from_slice(c);
            a
        })
        .collect())
}

/// `FilePart::write_with_encoder`'s compute for one part: (chunksize, parity chunks, d+p digests).
pub fn part_encode(
    codec: &ReedSolomon,
    data_buf: &[u8],
    length: usize,
) -> Result<(usize, Vec<Vec<u8>>, Vec<[u8; 32]>), CecError> {
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
    pub part_status: Vec<Result<(), CecError>>,
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

    /// A batch whose loaded chunks the reader appended back to back (part by part, ascending
    /// chunk index): `chunks` holds exactly the chunks whose `present` flag is nonzero, each
    /// `chunk_len` bytes, and goes up as one copy (`cec_read_pipeline_submit_packed`).
    ///
    /// # Safety
    /// `chunks` must stay alive and unmodified until `slot` is acquired again: the copy is
    /// asynchronous and `data_chunks` may point into it.
    pub unsafe fn submit_packed(
        &mut self,
        slot: usize,
        chunks: &[u8],
        present: &[u8],
        expected: &[u8],
        n_parts: usize,
    ) -> Result<(), CecError> {
        let n = n_parts * self.t;
        let loaded = present.iter().take(n).filter(|&&f| f != 0).count();
        if present.len() < n || expected.len() < n * 32 || chunks.len() < loaded * self.chunk_len {
            return Err(too_small("submit_packed"));
        }
        check_pipe(sys::cec_read_pipeline_submit_packed(
            self.raw,
            slot,
            chunks.as_ptr(),
            present.as_ptr(),
            expected.as_ptr(),
            n_parts,
            std::ptr::null_mut(),
        ))
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
                .map(|&c| check(c))
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
        // room for the largest batch a slot can hold, whatever n_parts says (the library writes
        // one pointer per chunk of the slot's batch, and checks the capacity)
        let mut ptrs = vec![std::ptr::null::<u8>(); self.parts * self.t];
        check_pipe(unsafe {
            sys::cec_read_pipeline_data_chunks(self.raw, slot, ptrs.as_mut_ptr(), ptrs.len())
        })?;
        ptrs.truncate(n_parts.min(self.parts) * self.d);
        Ok(ptrs
            .chunks(self.d)
            .map(|part| {
                part.iter()
                    .map(|&p| unsafe { std::slice::from_raw_parts(p, self.chunk_len) })
                    .collect()
            })
            .collect())
    }

    /// As [`ReadPipeline::new_rebuilt_only`] with `CEC_READ_CARRY`: the verified chunks of a
    /// part that comes back `TooFewShardsPresent` stay on the device for its retry
    /// ([`ReadPipeline::carry_ids`], [`ReadPipeline::submit_carried`]), so the loader fetches and
    /// uploads only the retry's new chunks -- the reference keeps them in memory the same way
    /// while it draws another chunk (file_part.rs:92-107).
    pub fn new_carry(
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
                sys::CEC_READ_REBUILT_ONLY | sys::CEC_READ_CARRY,
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

    /// After [`ReadPipeline::wait`]: each of the slot's `n_parts` parts' carry entry (`None`: its
    /// verified chunks were not kept; it resends them flagged `CEC_PRESENT_VERIFIED`).
    pub fn carry_ids(&mut self, slot: usize, n_parts: usize) -> Result<Vec<Option<i32>>, CecError> {
        // room for the largest batch a slot can hold (the library checks the capacity)
        let mut ids = vec![-1i32; self.parts];
        check_pipe(unsafe {
            sys::cec_read_pipeline_carry_ids(self.raw, slot, ids.as_mut_ptr(), ids.len())
        })?;
        Ok(ids.into_iter().take(n_parts).map(|id| if id >= 0 { Some(id) } else { None }).collect())
    }

    /// [`ReadPipeline::submit`] where the parts with `Some(id)` take their
    /// `CEC_PRESENT_VERIFIED` chunks from that carry entry (the slot need not hold them).  An
    /// entry is used once.
    pub fn submit_carried(
        &mut self,
        slot: usize,
        n_parts: usize,
        carry: &[Option<i32>],
    ) -> Result<(), CecError> {
        if carry.len() < n_parts {
            return Err(too_small("submit_carried"));
        }
        let ids: Vec<i32> = carry.iter().take(n_parts).map(|c| c.unwrap_or(-1)).collect();
        check_pipe(unsafe { sys::cec_read_pipeline_submit_carried(self.raw, slot, n_parts, ids.as_ptr()) })
    }

    /// Hands back the entry of a part the caller gives up on (undecodable: no chunk left).
    pub fn carry_release(&mut self, id: i32) -> Result<(), CecError> {
        check_pipe(unsafe { sys::cec_read_pipeline_carry_release(self.raw, id) })
    }
}

/// Page-locked host memory (`cec_host_alloc`) placed on `device`'s NUMA node: use it for the
/// part buffers the reference allocates with `vec![0; d * chunk_size]` (writer.rs:172) and the
/// parity `Vec`s (file_part.rs:158), and the engine DMAs them directly (no staging copy).
pub struct HostBuffer {
    ptr: *mut u8,
    len: usize,
}

unsafe impl Send for HostBuffer {}
unsafe impl Sync for HostBuffer {}

impl HostBuffer {
    /// `len` bytes, zeroed like the reference's `vec![0; n]`; `device` < 0: no NUMA preference.
    pub fn zeroed(len: usize, device: c_int) -> Result<HostBuffer, CecError> {
        let mut p: *mut c_void = std::ptr::null_mut();
        check(unsafe { sys::cec_host_alloc(len.max(1), device, &mut p) })?;
        unsafe { std::ptr::write_bytes(p as *mut u8, 0, len) };
        Ok(HostBuffer { ptr: p as *mut u8, len })
    }
}

impl Drop for HostBuffer {
    fn drop(&mut self) {
        unsafe { sys::cec_host_free(self.ptr as *mut c_void) }
    }
}

impl std::ops::Deref for HostBuffer {
    type Target = [u8];
    fn deref(&self) -> &[u8] {
        unsafe { std::slice::from_raw_parts(self.ptr, self.len) }
    }
}

impl std::ops::DerefMut for HostBuffer {
    fn deref_mut(&mut self) -> &mut [u8] {
        unsafe { std::slice::from_raw_parts_mut(self.ptr, self.len) }
    }
}

impl AsRef<[u8]> for HostBuffer {
    fn as_ref(&self) -> &[u8] {
        self
    }
}

impl AsMut<[u8]> for HostBuffer {
    fn as_mut(&mut self) -> &mut [u8] {
        self
    }
}

/// Multi-GPU part scheduler (`cec_multi_*`): `FileWriteBuilder::write`'s part loop
/// (writer.rs:117-255) and `FileReadBuilder`'s (reader.rs:32-74) over several GPUs in one
/// process.  One worker thread per entry of `devices`; a job of n parts in file order gives
/// shard g the contiguous range [g*n/G, (g+1)*n/G) and every result lands at its part's own
/// position.  The blocking forms below submit one job and wait for it; the buffers are the
/// caller's (page-locked ones, e.g. [`HostBuffer`], are DMA'd directly).
pub struct Multi {
    raw: *mut sys::cec_multi,
    d: usize,
    t: usize,
    chunk_len: usize,
}

pub(crate) fn too_small(what: &str) -> CecError {
    CecError::Engine(EngineError { code: 101, message: format!("{} buffer too small", what) })
}

unsafe impl Send for Multi {}
unsafe impl Sync for Multi {}

impl Drop for Multi {
    fn drop(&mut self) {
        unsafe { sys::cec_multi_free(self.raw) }
    }
}

fn check_multi(code: c_int) -> Result<(), CecError> {
    match check(code) {
        Err(CecError::Engine(mut e)) => {
            e.message = unsafe { std::ffi::CStr::from_ptr(sys::cec_multi_last_error()) }
                .to_string_lossy()
                .into_owned();
            Err(CecError::Engine(e))
        },
        other => other,
    }
}

impl Multi {
    /// A scheduler for both job kinds (write and read / resilver / verify).
    pub fn new(
        codec: &ReedSolomon,
        chunk_len: usize,
        parts_per_batch: usize,
        depth: usize,
        devices: &[c_int],
    ) -> Result<Multi, CecError> {
        Multi::with_kinds(codec, chunk_len, parts_per_batch, depth, devices,
                          sys::CEC_MULTI_WRITE | sys::CEC_MULTI_READ)
    }

    /// A scheduler for the job kinds in `kinds` (`CEC_MULTI_WRITE`, `CEC_MULTI_READ`): every
    /// shard makes those pipelines here, once (`cec_multi_new_ex`).
    pub fn with_kinds(
        codec: &ReedSolomon,
        chunk_len: usize,
        parts_per_batch: usize,
        depth: usize,
        devices: &[c_int],
        kinds: std::os::raw::c_uint,
    ) -> Result<Multi, CecError> {
        let mut raw = std::ptr::null_mut();
        check_multi(unsafe {
            sys::cec_multi_new_ex(
                codec.raw,
                chunk_len,
                parts_per_batch,
                depth,
                devices.as_ptr(),
                devices.len(),
                kinds,
                &mut raw,
            )
        })?;
        Ok(Multi {
            raw,
            d: codec.data_shard_count(),
            t: codec.total_shard_count(),
            chunk_len,
        })
    }

    /// write_with_encoder's compute for `n_parts` parts: `data` `[n][d][L]` ->
    /// `parity` `[n][p][L]`, `digests` `[n][d+p][32]` (chunks in order).
    pub fn encode_hash(
        &self,
        data: &[u8],
        n_parts: usize,
        parity: &mut [u8],
        digests: &mut [u8],
    ) -> Result<(), CecError> {
        let (d, p, l) = (self.d, self.t - self.d, self.chunk_len);
        if data.len() < n_parts * d * l {
            return Err(too_small("data"));
        }
        if parity.len() < n_parts * p * l {
            return Err(too_small("parity"));
        }
        if digests.len() < n_parts * self.t * 32 {
            return Err(too_small("digests"));
        }
        let mut job = 0u64;
        check_multi(unsafe {
            sys::cec_multi_encode_hash(
                self.raw,
                data.as_ptr(),
                n_parts,
                parity.as_mut_ptr(),
                digests.as_mut_ptr(),
                &mut job,
            )
        })?;
        check_multi(unsafe { sys::cec_multi_wait(self.raw, job) })
    }

    /// read_with_context's compute for `n_parts` parts: `chunks` `[n][d+p][L]` (loaded chunk
    /// bytes), `present` `[n][d+p]` (0 not loaded, 1 loaded, `CEC_PRESENT_VERIFIED` already
    /// verified by an earlier pass), `expected` `[n][d+p][32]` -> `data` `[n][d][L]`,
    /// `verified` `[n][d+p]`; per part `Ok(())` or `Err(TooFewShardsPresent)` (load more
    /// chunks and read that part again, file_part.rs:92-107).
    pub fn read(
        &self,
        chunks: &[u8],
        present: &[u8],
        expected: &[u8],
        n_parts: usize,
        data: &mut [u8],
        verified: &mut [u8],
    ) -> Result<Vec<Result<(), CecError>>, CecError> {
        let (d, t, l) = (self.d, self.t, self.chunk_len);
        if chunks.len() < n_parts * t * l || data.len() < n_parts * d * l {
            return Err(too_small("chunk / data"));
        }
        if present.len() < n_parts * t || verified.len() < n_parts * t {
            return Err(too_small("present / verified"));
        }
        if expected.len() < n_parts * t * 32 {
            return Err(too_small("expected"));
        }
        let mut status = vec![0 as c_int; n_parts];
        let mut job = 0u64;
        check_multi(unsafe {
            sys::cec_multi_read(
                self.raw,
                chunks.as_ptr(),
                present.as_ptr(),
                expected.as_ptr(),
                n_parts,
                data.as_mut_ptr(),
                verified.as_mut_ptr(),
                status.as_mut_ptr(),
                std::ptr::null_mut(),
                0,
                &mut job,
            )
        })?;
        check_multi(unsafe { sys::cec_multi_wait(self.raw, job) })?;
        Ok(status.into_iter().map(check).collect())
    }

    /// Asynchronous [`Multi::encode_hash`]: queues the job and returns its id for
    /// [`Multi::wait`], so the caller can fill its next window while this one runs.
    ///
    /// # Safety
    /// `data` (`n_parts * d * L` bytes), `parity` (`n_parts * p * L`) and `digests`
    /// (`n_parts * (d + p) * 32`) must stay valid, and `data` unmodified, until the job has been
    /// waited for.
    pub unsafe fn submit_encode_hash(
        &self,
        data: *const u8,
        n_parts: usize,
        parity: *mut u8,
        digests: *mut u8,
    ) -> Result<u64, CecError> {
        let mut job = 0u64;
        check_multi(sys::cec_multi_encode_hash(self.raw, data, n_parts, parity, digests, &mut job))?;
        Ok(job)
    }

    /// Asynchronous [`Multi::read`] (data of every part back, no `data_ptrs`): queues the job
    /// and returns its id for [`Multi::wait`].
    ///
    /// # Safety
    /// `chunks` (`n_parts * (d + p) * L` bytes), `present` / `verified` (`n_parts * (d + p)`),
    /// `expected` (`n_parts * (d + p) * 32`), `data` (`n_parts * d * L`) and `status`
    /// (`n_parts`) must stay valid, and the inputs unmodified, until the job has been waited for.
    #[allow(clippy::too_many_arguments)]
    pub unsafe fn submit_read(
        &self,
        chunks: *const u8,
        present: *const u8,
        expected: *const u8,
        n_parts: usize,
        data: *mut u8,
        verified: *mut u8,
        status: *mut c_int,
    ) -> Result<u64, CecError> {
        let mut job = 0u64;
        check_multi(sys::cec_multi_read(
            self.raw,
            chunks,
            present,
            expected,
            n_parts,
            data,
            verified,
            status,
            std::ptr::null_mut(),
            0,
            &mut job,
        ))?;
        Ok(job)
    }

    /// Asynchronous [`Multi::read`] that keeps retries' verified chunks on the GPUs
    /// (`cec_multi_read_carry`): `carry_out[k]` receives, at [`Multi::wait`], an id for each part
    /// reported `TooFewShardsPresent` whose verified chunks its shard kept (-1: none);
    /// `carry_in[k]` (-1: none) hands such an id to the part's retry, whose
    /// `CEC_PRESENT_VERIFIED` chunks then come from that GPU, not from `chunks`.  An id is used
    /// once; ids that will not be used go back with [`Multi::carry_release`].  `data_ptrs`
    /// (`n_parts * d` entries, nullable): `CEC_READ_REBUILT_ONLY` -- only the rebuilt data chunks
    /// come back into `data`, and `data_ptrs[k * d + j]` receives, at [`Multi::wait`], where data
    /// chunk j of part k is (in `chunks` where it was loaded, else in `data`).  `ahead`
    /// (`CEC_MULTI_AHEAD`): the job goes ahead of the queued jobs not yet started -- a reader's
    /// retry round, which the window being emitted waits for.
    ///
    /// # Safety
    /// As [`Multi::submit_read`]; `carry_in`, `carry_out` (`n_parts` each) and `data_ptrs`, any of
    /// them null, must stay valid until the job has been waited for.
    #[allow(clippy::too_many_arguments)]
    pub unsafe fn submit_read_carry(
        &self,
        chunks: *const u8,
        present: *const u8,
        expected: *const u8,
        n_parts: usize,
        data: *mut u8,
        verified: *mut u8,
        status: *mut c_int,
        carry_in: *const i32,
        carry_out: *mut i32,
        data_ptrs: *mut *const u8,
        ahead: bool,
    ) -> Result<u64, CecError> {
        let mut job = 0u64;
        let rebuilt_only = if data_ptrs.is_null() { 0 } else { sys::CEC_READ_REBUILT_ONLY };
        check_multi(sys::cec_multi_read_carry(
            self.raw,
            chunks,
            present,
            expected,
            n_parts,
            data,
            verified,
            status,
            data_ptrs,
            rebuilt_only | if ahead { sys::CEC_MULTI_AHEAD } else { 0 },
            carry_in,
            carry_out,
            &mut job,
        ))?;
        Ok(job)
    }

    /// Gives back a carry id the caller will not use (`cec_multi_carry_release`).
    pub fn carry_release(&self, id: i32) -> Result<(), CecError> {
        check_multi(unsafe { sys::cec_multi_carry_release(self.raw, id) })
    }

    /// Shard `g`'s counters (`cec_multi_shard_stats`).
    pub fn stats(&self, g: usize) -> Result<sys::cec_multi_stats, CecError> {
        let mut st = sys::cec_multi_stats::default();
        check_multi(unsafe { sys::cec_multi_shard_stats(self.raw, g, &mut st) })?;
        Ok(st)
    }

    /// `FilePart::verify`'s compute (file_part.rs:228-251) for `n_parts` rows of d + p items:
    /// `verified[x] = 1` iff item x (`present[x] != 0`) hashes to `expected[x]`.  The rows need
    /// not be parts: any d + p copies per row, whatever chunk each belongs to (one item per
    /// location, [`crate::batch::BatchChecker`]).
    pub fn verify(
        &self,
        chunks: &[u8],
        present: &[u8],
        expected: &[u8],
        n_parts: usize,
        verified: &mut [u8],
    ) -> Result<(), CecError> {
        let (t, l) = (self.t, self.chunk_len);
        if chunks.len() < n_parts * t * l {
            return Err(too_small("chunks"));
        }
        if present.len() < n_parts * t || verified.len() < n_parts * t {
            return Err(too_small("present / verified"));
        }
        if expected.len() < n_parts * t * 32 {
            return Err(too_small("expected"));
        }
        let job = unsafe {
            self.submit_verify(chunks.as_ptr(), present.as_ptr(), expected.as_ptr(), n_parts,
                               verified.as_mut_ptr())
        }?;
        self.wait(job)
    }

    /// Asynchronous [`Multi::verify`].
    ///
    /// # Safety
    /// `chunks` (`n_parts * (d + p) * L` bytes), `present` / `verified` (`n_parts * (d + p)`)
    /// and `expected` (`n_parts * (d + p) * 32`) must stay valid, and the inputs unmodified, until
    /// the job has been waited for.
    pub unsafe fn submit_verify(
        &self,
        chunks: *const u8,
        present: *const u8,
        expected: *const u8,
        n_parts: usize,
        verified: *mut u8,
    ) -> Result<u64, CecError> {
        let mut job = 0u64;
        check_multi(sys::cec_multi_verify(self.raw, chunks, present, expected, n_parts, verified,
                                          &mut job))?;
        Ok(job)
    }

    /// `FilePart::resilver`'s compute (file_part.rs:266-308), asynchronous: every chunk of the
    /// `n_parts` parts whose `present` flag is 0, or whose copy does not verify, rebuilt (data
    /// and parity) into `rebuilt` `[n][d+p][L]`; `verified` and `status` as [`Multi::read`].
    ///
    /// # Safety
    /// `chunks` / `rebuilt` (`n_parts * (d + p) * L` bytes), `present` / `verified`
    /// (`n_parts * (d + p)`), `expected` (`n_parts * (d + p) * 32`) and `status` (`n_parts`) must
    /// stay valid, and the inputs unmodified, until the job has been waited for.
    #[allow(clippy::too_many_arguments)]
    pub unsafe fn submit_resilver(
        &self,
        chunks: *const u8,
        present: *const u8,
        expected: *const u8,
        n_parts: usize,
        rebuilt: *mut u8,
        verified: *mut u8,
        status: *mut c_int,
    ) -> Result<u64, CecError> {
        let mut job = 0u64;
        check_multi(sys::cec_multi_resilver(
            self.raw,
            chunks,
            present,
            expected,
            n_parts,
            rebuilt,
            verified,
            status,
            std::ptr::null_mut(),
            &mut job,
        ))?;
        Ok(job)
    }

    /// Waits for a job queued with one of the `submit_*` calls.
    pub fn wait(&self, job: u64) -> Result<(), CecError> {
        check_multi(unsafe { sys::cec_multi_wait(self.raw, job) })
    }

    /// Whether a job is done ([`Multi::wait`] then returns at once); never blocks
    /// (`cec_multi_query`).
    pub fn query(&self, job: u64) -> Result<bool, CecError> {
        match unsafe { sys::cec_multi_query(self.raw, job) } {
            0 => Ok(false),
            1 => Ok(true),
            code => Err(check_multi(code).err().unwrap_or_else(|| crate::too_small("query"))),
        }
    }
}

/// Visible HIP devices (0 when none; never fails).
pub fn device_count() -> c_int {
    unsafe { sys::cec_device_count() }
}

/// Hash of the sources the linked library was built from (`cec_build_id`): a `build.rs` or a
/// service's startup log can compare it with the engine checkout it expects.
pub fn build_id() -> String {
    unsafe { std::ffi::CStr::from_ptr(sys::cec_build_id()) }.to_string_lossy().into_owned()
}

/// Frees the engine's idle per-call staging on `device` (every device when < 0); returns the
/// device bytes released (`cec_release_cached`).
pub fn release_cached(device: c_int) -> usize {
    unsafe { sys::cec_release_cached(device) }
}
