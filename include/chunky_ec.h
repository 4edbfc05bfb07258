/*
 * chunky_ec.h — C-ABI of the MI355X (gfx950) erasure-coding + chunk-hashing engine for Chunky Bits.
 *
 * This is the drop-in boundary.  It replaces the two third-party crates the
 * reference's part layer calls (neither is vendored in /root/reference):
 *
 *   reed_solomon_erasure 4.0.2 (Cargo.lock:1031-1037), galois_8 field:
 *     ReedSolomon::new            src/file/file_part.rs:77,302   src/file/writer.rs:131
 *                                 src/bin/chunky-bits/main.rs:557          -> cec_codec_new
 *     ReedSolomon::encode_sep     src/file/file_part.rs:161-165  main.rs:289 -> cec_encode_sep
 *     ReedSolomon::reconstruct_data  src/file/file_part.rs:128  main.rs:263 -> cec_reconstruct_data
 *     ReedSolomon::reconstruct    src/file/file_part.rs:304                 -> cec_reconstruct
 *     reed_solomon_erasure::Error (wrapped by FileWriteError::Erasure / FileReadError::Erasure,
 *                                 src/error.rs:44,55)                       -> cec_status 1..13
 *   sha2 0.9.9 (Cargo.lock:1221-1231):
 *     Sha256Hash::from_buf        src/file/hash/sha256.rs:20-26 (DataHasher, any.rs:17-25)
 *                                                                           -> cec_sha256
 *     DataVerifier::verify        src/file/hash/any.rs:27-52                -> cec_sha256 + compare
 *
 * and adds the batched, device-resident forms the GPU needs (many parts per launch):
 *     FilePart::write_with_encoder compute (file_part.rs:150-185: ceil(len/d) slicing, encode_sep,
 *       sha256 of the d+p chunks in order)                 -> cec_part_encode, cec_encode_hash_batch
 *     FilePart::read_with_context compute (file_part.rs:86-133: verify, reconstruct_data)
 *                                                          -> cec_reconstruct_batch, cec_sha256_batch
 *     FilePart::resilver compute (file_part.rs:266-308)    -> cec_reconstruct_batch (data_only = 0)
 *     FilePart::verify (file_part.rs:228-251)              -> cec_sha256_batch
 *
 * Conventions
 *   - Plain pointers and sizes only; every buffer is owned by the caller.
 *   - Functions return int status codes (cec_status).  1..13 map 1:1 onto the variants of
 *     reed_solomon_erasure::Error in declaration order, so a Rust shim can rebuild the crate
 *     error.  Codes >= 100 are engine errors with no crate equivalent.
 *   - Thread-safety: a cec_codec is immutable after cec_codec_new and may be shared by any
 *     number of threads (like the Arc<ReedSolomon> at writer.rs:131,200).  Host-buffer calls use a
 *     per-thread HIP stream and staging area on the calling thread's current HIP device.
 *   - Device-batch calls take a hipStream_t as `void* stream` (NULL = the null stream) and are
 *     asynchronous with respect to the host; device pointers must live on the current device.
 *   - All computation runs on the GPU.  There is no CPU fallback: without a usable HIP device
 *     the compute entry points return CEC_ERR_NO_DEVICE.
 */
#ifndef CHUNKY_EC_H
#define CHUNKY_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CEC_ABI_VERSION 3  /* 2: CEC_PRESENT_VERIFIED moved from 2 to 0x80; 3: read-pipeline
                              * modes per submit, output capacities, scheduler carry */

typedef enum cec_status {
    CEC_OK = 0,
    /* reed_solomon_erasure::Error (4.0.2), declaration order */
    CEC_TOO_FEW_SHARDS = 1,
    CEC_TOO_MANY_SHARDS = 2,
    CEC_TOO_FEW_DATA_SHARDS = 3,
    CEC_TOO_MANY_DATA_SHARDS = 4,
    CEC_TOO_FEW_PARITY_SHARDS = 5,
    CEC_TOO_MANY_PARITY_SHARDS = 6,
    CEC_TOO_FEW_BUFFER_SHARDS = 7,   /* no entry point of this ABI can raise it */
    CEC_TOO_MANY_BUFFER_SHARDS = 8,  /* no entry point of this ABI can raise it */
    CEC_INCORRECT_SHARD_SIZE = 9,
    CEC_TOO_FEW_SHARDS_PRESENT = 10,
    CEC_EMPTY_SHARD = 11,
    CEC_INVALID_SHARD_FLAGS = 12,    /* no entry point of this ABI can raise it */
    CEC_INVALID_INDEX = 13,          /* no entry point of this ABI can raise it */
    /* engine errors */
    CEC_ERR_INVALID_ARGUMENT = 101,
    CEC_ERR_HIP = 102,
    CEC_ERR_NO_DEVICE = 103,
    CEC_ERR_OUT_OF_MEMORY = 104
} cec_status;

/* ---------------------------------------------------------------------------------------- */
/* Library                                                                                   */
/* ---------------------------------------------------------------------------------------- */

int cec_abi_version(void);
/* Static description of a status code ("TooFewShardsPresent", ...). */
const char* cec_status_name(int status);
/* Message of the last CEC_ERR_HIP on the calling thread (empty string if none). */
const char* cec_last_error(void);
/* Number of visible HIP devices (0 when none; never fails). */
int cec_device_count(void);
/* The calling thread's current HIP device / make `device` current (host threads that drive
 * several GPUs; every call below works on the calling thread's current device). */
int cec_current_device(int* device);
int cec_set_device(int device);
/* NUMA node of a device's PCIe root (-1 when unknown). */
int cec_device_numa_node(int device);
/* Static build description, e.g. "chunky_ec gfx950 ab_tools=0".  The product library is always
 * ab_tools=0: the timing-attribution kernels (wrong outputs by design) exist only in the
 * separate A/B build used by tools/ (DESIGN.md §6.1). */
const char* cec_build_info(void);
/* Provenance: 16 hex digits, the hash of the sources the library was built from
 * (chunky-bits_amd/csrc/source_hash.py: every .cpp, .hip and .hpp file of csrc, its Makefile
 * and this header).  The Python binding refuses a library whose id differs from its shipped sources. */
const char* cec_build_id(void);
/* Environment knobs (CEC_APPLY_*, CEC_FUSED*, CEC_SHA_VARIANT, CEC_COALESCE_*, CEC_READ_*, ...;
 * DESIGN.md §4) are read ONCE, on the first call that needs one, into an immutable snapshot;
 * no launch path calls getenv (the reference drives the hot path from tokio worker threads,
 * where getenv racing a setenv is undefined behaviour).  Test-only: re-read them now (a test
 * that sets a knob calls this after setting it and again after restoring it).  No Rust binding
 * is needed for the reference's calls. */
void cec_reload_knobs(void);
/* Frees the engine's idle per-call staging (stream + device buffer contexts kept between
 * cec_encode_sep / cec_part_encode / ... calls: at most 8 per device holding at most
 * CEC_IDLE_STAGING_MIB, default 1024, of HBM) on `device`, or on every device when device < 0.
 * Staging leased by calls in progress is untouched.  Returns the device bytes released. */
size_t cec_release_cached(int device);

/* ---------------------------------------------------------------------------------------- */
/* Codec: ReedSolomon<galois_8::Field>                                                       */
/* ---------------------------------------------------------------------------------------- */

typedef struct cec_codec cec_codec;

/* ReedSolomon::new(data_shards, parity_shards).  Errors: TooFewDataShards (d == 0),
 * TooFewParityShards (p == 0), TooManyShards (d + p > 256).  Host-only; needs no GPU. */
int cec_codec_new(size_t data_shards, size_t parity_shards, cec_codec** out);
void cec_codec_free(cec_codec* codec);
size_t cec_codec_data_shards(const cec_codec* codec);
size_t cec_codec_parity_shards(const cec_codec* codec);
size_t cec_codec_total_shards(const cec_codec* codec);
/* Copies the (d+p) x d coding matrix (row major; top d x d = identity) into out[out_len]. */
int cec_codec_matrix(const cec_codec* codec, uint8_t* out, size_t out_len);
/* Decode matrices cached in the codec (one per erasure pattern and mode; least recently used
 * evicted past 4096 - the crate also bounds its decode-matrix cache). */
size_t cec_codec_cached_patterns(const cec_codec* codec);

/* ---------------------------------------------------------------------------------------- */
/* Page-locked host memory                                                                   */
/* ---------------------------------------------------------------------------------------- */

/* The reference allocates every part's data buffer with vec![0; d*chunk_size] (writer.rs:172)
 * and parity with vec![vec![0; L]; p] (file_part.rs:158).  Buffers from cec_host_alloc instead
 * are page-locked and portable (any device may DMA them), with pages on the NUMA node of
 * `device` (-1: no preference): every entry point below that takes host buffers DMAs straight
 * from / into them and skips its staging copy.  Contents are undefined (not zeroed). */
int cec_host_alloc(size_t bytes, int device, void** out);
void cec_host_free(void* ptr);
/* 1 if [ptr, ptr + bytes) lies in one page-locked allocation (cec_host_alloc, hipHostMalloc,
 * hipHostRegister), else 0. */
int cec_host_is_pinned(const void* ptr, size_t bytes);
/* NUMA node holding the page at ptr (-1 when unknown). */
int cec_host_numa_node(const void* ptr);
/* Restrict the calling thread to the CPUs of `device`'s NUMA node (∩ the CPUs it may use);
 * 1 if done, 0 if not possible (node unknown, or outside this process's cpuset).  The pinned
 * buffers the engine allocates itself (pipeline slots, scheduler staging) are placed on that
 * node whatever the caller's affinity. */
int cec_bind_thread_to_device_node(int device);

/* ---------------------------------------------------------------------------------------- */
/* Host-buffer API: one call per part, staged through the GPU (drop-in for the crate calls) */
/* ---------------------------------------------------------------------------------------- */

/* ReedSolomon::encode_sep(&data, &mut parity): data[n_data] slices of data_lens[i] bytes,
 * parity[n_parity] caller-allocated slices of parity_lens[i] bytes, overwritten. */
int cec_encode_sep(const cec_codec* codec,
                   const uint8_t* const* data, const size_t* data_lens, size_t n_data,
                   uint8_t* const* parity, const size_t* parity_lens, size_t n_parity);

/* ReedSolomon::reconstruct / reconstruct_data on &mut [Option<Vec<u8>>].
 * present[i] != 0 <=> Some(shard) of shard_lens[i] bytes at shards[i].  For every missing slot
 * the crate would fill (all missing slots for reconstruct; missing DATA slots only for
 * reconstruct_data) shards[i] must point to caller memory of shard_lens[i] >= the present shard
 * length (else CEC_ERR_INVALID_ARGUMENT).  On success those slots are written and present[i] is
 * set to 1; slots the crate would leave None keep present[i] == 0. */
int cec_reconstruct(const cec_codec* codec, uint8_t* const* shards, const size_t* shard_lens,
                    uint8_t* present, size_t n_shards);
int cec_reconstruct_data(const cec_codec* codec, uint8_t* const* shards,
                         const size_t* shard_lens, uint8_t* present, size_t n_shards);

/* Sha256Hash::from_buf: out[32] = SHA-256(buf[0..len]). */
int cec_sha256(const uint8_t* buf, size_t len, uint8_t* out32);
/* n independent digests in one launch: out[i*32..] = SHA-256(bufs[i][0..lens[i]]). */
int cec_sha256_many(const uint8_t* const* bufs, const size_t* lens, size_t n, uint8_t* out);

/* FilePart::write_with_encoder compute (file_part.rs:150-185) for one part:
 * L = ceil(length / d); data chunk j = data_buf[j*L .. (j+1)*L] (data_buf holds d*L bytes,
 * zero padded past `length` like writer.rs:172); parity_out receives p*L bytes (chunk i at
 * parity_out + i*L); digests_out receives (d+p)*32 bytes, chunks in order (d data then p
 * parity); *chunksize = L.  length == 0 -> CEC_EMPTY_SHARD (as encode_sep on empty slices). */
int cec_part_encode(const cec_codec* codec, const uint8_t* data_buf, size_t length,
                    uint8_t* parity_out, uint8_t* digests_out, size_t* chunksize);

/* Per-call coalescing.  Concurrent cec_part_encode calls with the same codec and chunk length
 * (and concurrent cec_sha256 / cec_sha256_many calls) on the same device are gathered into one
 * launch: the first caller waits up to CEC_COALESCE_US microseconds (environment, default 200,
 * 0 = off) for others, runs the whole batch and wakes them with their results.  A lone GPU
 * SHA-256 lane hashes ~25 MB/s (a serial chain), so the reference's per-part calls only pay off
 * when their concurrency becomes batch width.  Results are identical either way.
 * cec_coalesce_stats: calls made and launches issued through this path since load. */
void cec_coalesce_stats(uint64_t* calls, uint64_t* launches);

/* ---------------------------------------------------------------------------------------- */
/* Device-resident batch API (inputs already in HBM; asynchronous on `stream`)              */
/* ---------------------------------------------------------------------------------------- */

/* Part k's chunk i (0 <= i < d+p, d data then p parity, in order) lives at
 *   base + k*part_stride + i*chunk_stride
 * and is chunk_len (= FilePart::chunksize) bytes long.  Fast path: base, part_stride and
 * chunk_stride multiples of 16; any other layout is supported at lower speed. */
typedef struct cec_part_batch {
    uint8_t* base;
    size_t part_stride;
    size_t chunk_stride;
    size_t n_parts;
    size_t chunk_len;
} cec_part_batch;

/* encode_sep for every part: writes the p parity chunks of each part from its d data chunks. */
int cec_encode_batch(const cec_codec* codec, const cec_part_batch* batch, void* stream);

/* encode_sep + SHA-256 of all d+p chunks of every part (write_with_encoder's compute).
 * digests: device buffer of n_parts*(d+p)*32 bytes, part-major, chunks in order. */
int cec_encode_hash_batch(const cec_codec* codec, const cec_part_batch* batch, uint8_t* digests,
                          void* stream);

/* SHA-256 of chunks [first_chunk, first_chunk + n_chunks) of every part.
 * digests: device buffer, digest of (part k, chunk first_chunk + c) at (k*n_chunks + c)*32. */
int cec_sha256_batch(const cec_part_batch* batch, size_t first_chunk, size_t n_chunks,
                     uint8_t* digests, void* stream);

/* reconstruct (data_only = 0) / reconstruct_data (data_only = 1) for every part.
 * present: HOST array of n_parts*(d+p) flags (part-major).  Every part must have >= d present
 * chunks (else CEC_TOO_FEW_SHARDS_PRESENT, nothing launched).  Missing chunks are rebuilt in
 * place from the first d present chunks of their part (the crate's choice); parts with nothing
 * missing are skipped.  Parts are grouped by erasure pattern on the host; decode matrices are
 * inverted once per pattern and cached in the codec. */
int cec_reconstruct_batch(const cec_codec* codec, const cec_part_batch* batch,
                          const uint8_t* present, int data_only, void* stream);

/* DataVerifier::verify (src/file/hash/any.rs:27-52, called per chunk at file_part.rs:102,239)
 * for chunks [first_chunk, first_chunk + n_chunks) of every part:
 * ok[k*n_chunks + c] = 1 iff SHA-256(chunk) == expected[(k*n_chunks + c)*32 .. +32]; chunks
 * whose present flag is 0 are not read and get ok = 0.  present (nullable: all present),
 * expected and ok are DEVICE buffers. */
int cec_verify_batch(const cec_part_batch* batch, size_t first_chunk, size_t n_chunks,
                     const uint8_t* present, const uint8_t* expected, uint8_t* ok, void* stream);

/* Present-flag value for read retries.  The reference's read drops a chunk whose hash fails and
 * samples another (file_part.rs:92-107) until d chunks verified or none are left.  The batched
 * reads (cec_read_batch, cec_read_pipeline_*, cec_multi_read) report such a part
 * CEC_TOO_FEW_SHARDS_PRESENT with its verified flags; the caller loads more chunks for just
 * those parts and submits them again, marking the chunks already verified CEC_PRESENT_VERIFIED
 * (they are used but not hashed again) and the new ones 1.  Any other nonzero flag = loaded and
 * hashed.  ABI 2 moved the value from 2 to 0x80: in ABI 1 a caller passing 2 for "loaded" (or
 * summing / OR-ing small flags) silently skipped verification; 0x80 does not arise that way. */
#define CEC_PRESENT_VERIFIED 0x80

/* FilePart::read_with_context compute (file_part.rs:86-129) for every part: verify the loaded
 * chunks (present: HOST flags, n_parts*(d+p)) against expected (DEVICE digests, part-major,
 * chunks in order), then reconstruct_data from the first d verified chunks.  Outputs (HOST):
 * verified[k*(d+p)+i] = verification result; part_status[k] = CEC_OK, or
 * CEC_TOO_FEW_SHARDS_PRESENT when fewer than d chunks verified (its loaded chunks are left
 * untouched; its other chunks are unspecified).  The decode runs speculatively from the first d
 * LOADED chunks, concurrently with the verification, and parts with a loaded chunk that failed
 * are decoded again from their verified chunks, so the result is always the verified decode.
 * Waits on `stream` once, for the verification flags; the re-decode (if any) is queued on it. */
int cec_read_batch(const cec_codec* codec, const cec_part_batch* batch, const uint8_t* present,
                   const uint8_t* expected, uint8_t* verified, int* part_status, void* stream);
/* FilePart::resilver compute (file_part.rs:266-308): as cec_read_batch over all d+p chunks,
 * then reconstruct (missing data AND parity) in place. */
int cec_resilver_batch(const cec_codec* codec, const cec_part_batch* batch,
                       const uint8_t* present, const uint8_t* expected, uint8_t* verified,
                       int* part_status, void* stream);

/* ---------------------------------------------------------------------------------------- */
/* Host-staged write pipeline (FileWriteBuilder::write's part loop, writer.rs:166-231)      */
/* ---------------------------------------------------------------------------------------- */

/* `depth` slots on the current device, each with pinned host buffers for parts_per_batch parts
 * of d chunks of chunk_len bytes, a device batch and its own HIP stream.  One thread drives a
 * pipeline.  Per slot: acquire (waits for the slot's previous batch; *data = pinned
 * [parts][d][chunk_len] buffer the caller fills, i.e. each part's zero-padded d*L data_buf),
 * submit (H2D, encode + SHA-256 of all d+p chunks, D2H parity + digests, asynchronously),
 * wait (*parity = pinned [parts][p][L], *digests = pinned [parts][d+p][32]). */
typedef struct cec_pipeline cec_pipeline;
int cec_pipeline_new(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                     size_t depth, cec_pipeline** out);
/* Pipeline flag: no pinned part-data slot buffers; batches come from the caller's own buffers
 * through *_submit_from (zero-copy when they are page-locked, e.g. cec_host_alloc). */
#define CEC_PIPE_EXTERNAL 2u
int cec_pipeline_new_ex(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                        size_t depth, unsigned flags, cec_pipeline** out);
/* As cec_pipeline_submit, with the data read from the caller's data [n_parts][d][chunk_len] and
 * the results written to parity_out [n_parts][p][chunk_len] and digests_out [n_parts][d+p][32]
 * (NULL: the slot's own buffers).  The buffers must stay valid until the slot's wait. */
int cec_pipeline_submit_from(cec_pipeline* pipeline, size_t slot, const uint8_t* data,
                             size_t n_parts, uint8_t* parity_out, uint8_t* digests_out);
void cec_pipeline_free(cec_pipeline* pipeline);
size_t cec_pipeline_depth(const cec_pipeline* pipeline);
int cec_pipeline_acquire(cec_pipeline* pipeline, size_t* slot, uint8_t** data);
int cec_pipeline_submit(cec_pipeline* pipeline, size_t slot, size_t n_parts);
int cec_pipeline_wait(cec_pipeline* pipeline, size_t slot, const uint8_t** parity,
                      const uint8_t** digests, size_t* n_parts);
int cec_pipeline_drain(cec_pipeline* pipeline);
/* 1 when the slot's batch is complete (or none is in flight), 0 while it is running; never
 * blocks (for callers that multiplex pipelines).  Same for cec_read_pipeline_query. */
int cec_pipeline_query(cec_pipeline* pipeline, size_t slot);
const char* cec_pipeline_last_error(void);

/* Host-staged READ pipeline (FileReadBuilder's part loop, reader.rs:40-75, over
 * FilePart::read_with_context, file_part.rs:73-135).  `depth` slots; per slot the caller fills
 * (acquire): chunks = pinned [parts][d+p][chunk_len] (the chunk bytes it could load), present =
 * pinned [parts][d+p] (1 = loaded; every slot starts all-0 and keeps what the caller wrote),
 * expected = pinned [parts][d+p][32] (the metadata digests).  submit: loaded chunks H2D,
 * SHA-256 verification of every loaded chunk, speculative reconstruct_data from the first d
 * loaded chunks, D2H of the d data chunks - all asynchronous.  wait: *data = pinned
 * [parts][d][chunk_len] (the part's bytes, as read_with_context returns them), *verified =
 * [parts][d+p] flags, *part_status = [parts] (CEC_OK or CEC_TOO_FEW_SHARDS_PRESENT); parts
 * whose loaded chunks did not all verify are decoded again from their verified chunks before
 * wait returns.  Errors: cec_pipeline_last_error(). */
typedef struct cec_read_pipeline cec_read_pipeline;
int cec_read_pipeline_new(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                          size_t depth, cec_read_pipeline** out);
void cec_read_pipeline_free(cec_read_pipeline* pipeline);
size_t cec_read_pipeline_depth(const cec_read_pipeline* pipeline);
int cec_read_pipeline_acquire(cec_read_pipeline* pipeline, size_t* slot, uint8_t** chunks,
                              uint8_t** present, uint8_t** expected);
int cec_read_pipeline_submit(cec_read_pipeline* pipeline, size_t slot, size_t n_parts);
/* As cec_read_pipeline_acquire, but takes the first slot (from the round-robin position on)
 * whose batch has completed or that has none, and waits only when every slot is busy: a small
 * retry batch submitted while the other slots run starts at once.  The slot's previous results
 * are no longer valid. */
int cec_read_pipeline_acquire_idle(cec_read_pipeline* pipeline, size_t* slot, uint8_t** chunks,
                                   uint8_t** present, uint8_t** expected);
int cec_read_pipeline_wait(cec_read_pipeline* pipeline, size_t slot, const uint8_t** data,
                           const uint8_t** verified, const int** part_status, size_t* n_parts);
int cec_read_pipeline_drain(cec_read_pipeline* pipeline);
int cec_read_pipeline_query(cec_read_pipeline* pipeline, size_t slot);
/* As cec_read_pipeline_new with flags: the default MODE of the submits above (mode bits
 * CEC_READ_REBUILT_ONLY / CEC_READ_RESILVER / CEC_READ_VERIFY_ONLY, below), CEC_PIPE_EXTERNAL and
 * CEC_READ_CARRY.  The device buffers are the same for every mode, so any submit may pick
 * another mode (cec_read_pipeline_submit_ex): one pipeline serves verify, resilver and read in
 * turn (FilePart::verify / resilver / read_with_context on the same parts, file_part.rs:73-390).
 * Mode CEC_READ_REBUILT_ONLY: submit copies back only the data chunks it rebuilt (RS(10,4) with
 * d random chunks loaded: 2.9 of 10 per part), since the loaded ones are already in the caller's
 * pinned chunk buffer; wait's *data then holds only those, and cec_read_pipeline_data_chunks
 * says where each data chunk is. */
#define CEC_READ_REBUILT_ONLY 1u
int cec_read_pipeline_new_ex(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                             size_t depth, unsigned flags, cec_read_pipeline** out);
/* Mode: FilePart::resilver's compute (file_part.rs:253-308) instead of read_with_context's.
 * Every chunk that does not verify (data AND parity: missing, or loaded with a bad hash) is
 * rebuilt from the first d verified chunks (reconstruct, not reconstruct_data) and comes back
 * into the output, which is then [parts][d+p][chunk_len] (only the rebuilt chunks are written);
 * cec_read_pipeline_data_chunks gives d+p pointers per part (a verified chunk where it was read,
 * a rebuilt one in the output): what resilver writes back to storage is every chunk whose
 * verified flag is 0. */
#define CEC_READ_RESILVER 4u
/* Mode: FilePart::verify's compute (file_part.rs:228-251): every loaded chunk is hashed and
 * compared with its metadata digest; nothing is decoded or copied back (wait gives the verified
 * flags; part_status is CEC_OK; data_out may be NULL). */
#define CEC_READ_VERIFY_ONLY 8u
/* Pipeline flag: keep retries' verified chunks on the device (read modes only; a resilver or
 * verify submit keeps nothing).  The reference keeps a chunk that verified in memory while it
 * draws another for the one that failed (file_part.rs:92-107); without this flag the retry of a
 * part sends its verified chunks up again (CEC_PRESENT_VERIFIED).  With it, each batch keeps the
 * verified chunks of every part it will report CEC_TOO_FEW_SHARDS_PRESENT in a device carry pool,
 * on the device right after the verification (up to max(8, parts_per_batch/4) parts per batch,
 * in part order; the pool holds depth+1 times that many entries of (d+p) chunks and is made with
 * the pipeline).  After wait, cec_read_pipeline_carry_ids gives each such part its entry (-1:
 * none kept) and hands the entries to the caller; entries of a batch whose ids were not taken go
 * back when its slot is submitted again.  The retry passes the ids with its submit (carry_ids of
 * cec_read_submit): a part with an id takes its CEC_PRESENT_VERIFIED chunks from the pool (the
 * caller need not supply them) and its data chunks among them come back like rebuilt ones
 * (REBUILT_ONLY data_chunks point at the data output for them).  An id is only accepted for the
 * part it was kept for (same metadata digests, and every CEC_PRESENT_VERIFIED chunk one the
 * entry holds): CEC_ERR_INVALID_ARGUMENT otherwise.  An id is used once; one the caller will not
 * use (an undecodable part) goes back with cec_read_pipeline_carry_release. */
#define CEC_READ_CARRY 16u
/* After wait: ids[k] = the carry entry of part k of the slot's batch, or -1; capacity = the
 * entries ids holds (CEC_ERR_INVALID_ARGUMENT when the batch has more parts). */
int cec_read_pipeline_carry_ids(cec_read_pipeline* pipeline, size_t slot, int32_t* ids,
                                size_t capacity);
/* As cec_read_pipeline_submit, with carry_ids[n_parts] (-1 = none) for the parts whose verified
 * chunks come from the carry pool. */
int cec_read_pipeline_submit_carried(cec_read_pipeline* pipeline, size_t slot, size_t n_parts,
                                     const int32_t* carry_ids);
/* Hands an unused carry entry back. */
int cec_read_pipeline_carry_release(cec_read_pipeline* pipeline, int32_t id);
/* Carry entries the caller holds (taken with carry_ids, not yet submitted or released). */
size_t cec_read_pipeline_carry_held(const cec_read_pipeline* pipeline);
/* After (or instead of) wait: ptrs[k*out + j] = the chunk_len bytes of output chunk j of part k
 * (out = d, or d+p for a resilver batch) -- in the chunk buffer (loaded and verified,
 * REBUILT_ONLY / resilver) or in the data output (rebuilt, re-decoded, or without REBUILT_ONLY).
 * capacity = the pointers ptrs holds (CEC_ERR_INVALID_ARGUMENT when the batch has more).  Valid
 * until the slot is acquired again; undefined for parts whose status is not CEC_OK. */
int cec_read_pipeline_data_chunks(cec_read_pipeline* pipeline, size_t slot,
                                  const uint8_t** ptrs, size_t capacity);
/* As cec_read_pipeline_submit, with the loaded chunk bytes read from the caller's chunks
 * [n_parts][d+p][chunk_len] and the data written to data_out [n_parts][d][chunk_len] (NULL: the
 * slot's own buffer); present / expected (NULL: the slot's arrays as filled after acquire) are
 * copied in at submit.  chunks and data_out must stay valid until the slot is acquired again
 * (REBUILT_ONLY data_chunks pointers may point into chunks). */
int cec_read_pipeline_submit_from(cec_read_pipeline* pipeline, size_t slot, const uint8_t* chunks,
                                  const uint8_t* present, const uint8_t* expected, size_t n_parts,
                                  uint8_t* data_out);
/* As cec_read_pipeline_submit_from with the loaded chunks PACKED: `chunks` holds exactly the
 * chunks whose present flag is nonzero (CEC_PRESENT_VERIFIED included), chunk_len bytes each,
 * back to back — part by part, ascending chunk index within a part — the order a reader that
 * fetches a part's chunks one after the other produces them (file_part.rs:86-107).  The batch
 * then goes up as ONE copy (per-run copies of randomly loaded chunks cost the copy engines
 * ~11 us each) and a device kernel places each chunk.  Outputs, data_chunks pointers (which may
 * point into `chunks`) and lifetimes as cec_read_pipeline_submit_from. */
int cec_read_pipeline_submit_packed(cec_read_pipeline* pipeline, size_t slot,
                                    const uint8_t* chunks, const uint8_t* present,
                                    const uint8_t* expected, size_t n_parts, uint8_t* data_out);
/* The general submit: every form above is this with the pipeline's default mode.
 *   chunks    -- NULL: the slot's pinned chunk buffer (not for CEC_PIPE_EXTERNAL pipelines);
 *   present, expected -- NULL: the slot's arrays as filled after acquire; else copied in;
 *   data_out  -- NULL: the slot's own output (CEC_ERR_INVALID_ARGUMENT when it is smaller than
 *                the mode writes, or absent); [n][d][L], or [n][d+p][L] for CEC_READ_RESILVER;
 *   carry_ids -- NULL, or [n_parts] carry ids (-1 = none) of a CEC_READ_CARRY pipeline;
 *   flags     -- the mode bits (0 = read_with_context) | CEC_SUBMIT_PACKED (`chunks` holds
 *                back to back exactly the chunks that go up: present != 0, except the
 *                CEC_PRESENT_VERIFIED chunks of parts with a carry id). */
#define CEC_SUBMIT_PACKED 32u
typedef struct cec_read_submit {
    const uint8_t* chunks;
    const uint8_t* present;
    const uint8_t* expected;
    size_t n_parts;
    uint8_t* data_out;
    const int32_t* carry_ids;
    unsigned flags;
} cec_read_submit;
int cec_read_pipeline_submit_ex(cec_read_pipeline* pipeline, size_t slot,
                                const cec_read_submit* submit);
/* Write and read pipelines made by this process so far (a scheduler makes its own once, in
 * cec_multi_new: tests check that no job makes another). */
uint64_t cec_pipelines_made(void);

/* ---------------------------------------------------------------------------------------- */
/* Multi-GPU part scheduler (one process, several GPUs: SURVEY.md §8e)                       */
/* ---------------------------------------------------------------------------------------- */

/* The reference writes and reads a file from one process (FileWriteBuilder::write's part loop,
 * writer.rs:117-255; FileReadBuilder, reader.rs:32-74).  A cec_multi runs one worker thread per
 * entry of devices[n_devices] (an ordinal may repeat: several shards on one GPU); each worker
 * binds to its device's NUMA node and streams its share through its own pipelines of `depth`
 * slots of parts_per_batch parts.  A job of n parts in file order gives shard g the contiguous
 * range [g*n/G, (g+1)*n/G); every result lands at its part's own position (file order).  Jobs
 * are asynchronous (wait with cec_multi_wait; buffers stay the caller's and must live until
 * then) and run in submission order (CEC_MULTI_AHEAD below excepted).  Page-locked caller
 * buffers (cec_host_alloc) are DMA'd directly; others go through the workers' NUMA-local pinned
 * staging. */
typedef struct cec_multi cec_multi;
int cec_multi_new(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch, size_t depth,
                  const int* devices, size_t n_devices, cec_multi** out);
/* As cec_multi_new for the job kinds in flags: CEC_MULTI_WRITE (cec_multi_encode_hash),
 * CEC_MULTI_READ (read / resilver / verify); cec_multi_new = both.  Each shard makes its
 * pipelines for those kinds (one write pipeline; one read pipeline with a carry pool, whose mode
 * is picked per job) before this returns -- no job ever makes or frees a pipeline, so no stream
 * or device buffer is created while other shards' batches run -- and an allocation failure is
 * reported here.  A job of a kind the scheduler was not made for: CEC_ERR_INVALID_ARGUMENT. */
#define CEC_MULTI_WRITE 1u
#define CEC_MULTI_READ 2u
int cec_multi_new_ex(const cec_codec* codec, size_t chunk_len, size_t parts_per_batch,
                     size_t depth, const int* devices, size_t n_devices, unsigned flags,
                     cec_multi** out);
void cec_multi_free(cec_multi* multi);
size_t cec_multi_shards(const cec_multi* multi);
/* Shard g's device ordinal, its NUMA node, and the parts it has processed. */
int cec_multi_shard_info(cec_multi* multi, size_t g, int* device, int* numa_node, uint64_t* parts);
/* write_with_encoder's compute for n_parts parts: data [n][d][L] (each part's zero-padded
 * data_buf) -> parity [n][p][L], digests [n][d+p][32] (chunks in order). */
int cec_multi_encode_hash(cec_multi* multi, const uint8_t* data, size_t n_parts, uint8_t* parity,
                          uint8_t* digests, uint64_t* job);
/* read_with_context's compute for n_parts parts: chunks [n][d+p][L] (loaded chunk bytes; only
 * chunks with present != 0 are read), present [n][d+p], expected [n][d+p][32] -> data [n][d][L]
 * (the part bytes), verified [n][d+p], part_status [n] (CEC_OK / CEC_TOO_FEW_SHARDS_PRESENT).
 * flags = CEC_READ_REBUILT_ONLY: data receives only the rebuilt data chunks and data_ptrs[n*d]
 * (required then; optional otherwise) says where each data chunk of each part is (null for a
 * part that is not CEC_OK when its bytes went through the scheduler's own staging). */
/* flags |= CEC_MULTI_AHEAD (read and read_carry): the job goes ahead of every queued job that has
 * not started (behind earlier AHEAD jobs) -- a reader's retry round, a few parts that the window
 * being emitted waits for, need not wait behind whole windows queued after it. */
#define CEC_MULTI_AHEAD 64u
int cec_multi_read(cec_multi* multi, const uint8_t* chunks, const uint8_t* present,
                   const uint8_t* expected, size_t n_parts, uint8_t* data, uint8_t* verified,
                   int* part_status, const uint8_t** data_ptrs, unsigned flags, uint64_t* job);
/* As cec_multi_read, keeping retries' verified chunks on the devices (file_part.rs:92-107 keeps
 * them in memory while it draws another chunk).  carry_out[n] (nullable): for each part reported
 * CEC_TOO_FEW_SHARDS_PRESENT, an id under which its shard keeps the part's verified chunks on its
 * GPU (-1: none kept, e.g. the shard's carry pool is full; every other part gets -1).
 * carry_in[n] (nullable): per part, -1 or an id from an earlier job's carry_out.  A part with an
 * id runs on the shard that holds its chunks (the others split as usual) and takes its
 * CEC_PRESENT_VERIFIED chunks from there: `chunks` need not hold them and they are not sent
 * again.  An id is accepted only for the part it was kept for (same expected digests, its
 * CEC_PRESENT_VERIFIED chunks among the kept ones) and used once; the job fails with
 * CEC_ERR_INVALID_ARGUMENT otherwise.  Ids the caller will not use go back with
 * cec_multi_carry_release. */
int cec_multi_read_carry(cec_multi* multi, const uint8_t* chunks, const uint8_t* present,
                         const uint8_t* expected, size_t n_parts, uint8_t* data,
                         uint8_t* verified, int* part_status, const uint8_t** data_ptrs,
                         unsigned flags, const int32_t* carry_in, int32_t* carry_out,
                         uint64_t* job);
int cec_multi_carry_release(cec_multi* multi, int32_t id);
/* Shard g's counters: device, NUMA node, parts processed, pipelines made (1 per job kind, at
 * cec_multi_new), chunks sent to the GPU by read jobs, chunks read jobs took from the carry pool
 * instead, carry entries the caller holds. */
typedef struct cec_multi_stats {
    int device;
    int numa_node;
    uint64_t parts;
    uint64_t pipelines_made;
    uint64_t chunks_uploaded;
    uint64_t chunks_carried;
    uint64_t carry_held;
} cec_multi_stats;
int cec_multi_shard_stats(cec_multi* multi, size_t g, cec_multi_stats* out);
/* FilePart::resilver's compute (file_part.rs:253-308) for n_parts parts: as cec_multi_read, but
 * every chunk that does not verify (data AND parity) is rebuilt (reconstruct) into
 * rebuilt [n][d+p][L] (the verified ones are not written there); chunk_ptrs[n*(d+p)] (nullable)
 * says where each chunk of each part is.  What resilver writes back to storage: each chunk of a
 * CEC_OK part whose verified flag is 0. */
int cec_multi_resilver(cec_multi* multi, const uint8_t* chunks, const uint8_t* present,
                       const uint8_t* expected, size_t n_parts, uint8_t* rebuilt,
                       uint8_t* verified, int* part_status, const uint8_t** chunk_ptrs,
                       uint64_t* job);
/* FilePart::verify's compute for n_parts parts: verified[n][d+p] = every loaded chunk
 * (present != 0) hashed and compared with expected; nothing is decoded. */
int cec_multi_verify(cec_multi* multi, const uint8_t* chunks, const uint8_t* present,
                     const uint8_t* expected, size_t n_parts, uint8_t* verified, uint64_t* job);
/* Blocks until the job is done; returns its first error (message: cec_multi_last_error). */
int cec_multi_wait(cec_multi* multi, uint64_t job);
/* Never blocks: 1 when the job is done (cec_multi_wait then returns at once), 0 while it runs;
 * CEC_ERR_INVALID_ARGUMENT for a job not submitted or already waited for.  A reader polls its
 * windows' jobs with it, so a window's retry starts as soon as its job is done. */
int cec_multi_query(cec_multi* multi, uint64_t job);
const char* cec_multi_last_error(void);

/* ---------------------------------------------------------------------------------------- */
/* Utilities for benchmarks and tests                                                        */
/* ---------------------------------------------------------------------------------------- */

/* Deterministic synthetic bytes: for every part k, bytes [0, n_chunks*chunk_len) of chunks
 * 0..n_chunks-1 are filled from a counter-based generator keyed by (seed, k, chunk, offset).
 * Byte value = cec_synth_byte(seed, k, chunk, offset) (see below). */
int cec_fill_synthetic(const cec_part_batch* batch, size_t n_chunks, uint64_t seed, void* stream);
/* Host reference of the generator (same bytes), for checking sampled parts. */
uint8_t cec_synth_byte(uint64_t seed, uint64_t part, uint64_t chunk, uint64_t offset);

#ifdef __cplusplus
}
#endif

#endif /* CHUNKY_EC_H */
