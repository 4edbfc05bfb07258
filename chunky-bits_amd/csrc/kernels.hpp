// kernels.hpp — launch interface of the gfx950 kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace cec {

// One launch of the GF(2^8) matrix-apply kernel over a set of parts that share the output-row
// count.  Part `lp` of the launch is batch part part_ids[lp] (or lp), uses the pattern record at
// pat + part_pat[lp] (or pat + 0); see gf256.hpp for the record layout.  For each part:
//   chunk[out_idx[r]] = XOR_j coef[r][j] (x) chunk[in_idx[j]]     (bytes [0, len))
struct ApplyParams {
    uint8_t* base;
    uint64_t part_stride;
    uint64_t chunk_stride;
    uint64_t len;
    const uint32_t* pat;
    const uint32_t* part_ids;
    const uint32_t* part_pat;
    uint32_t n_parts;
    uint32_t d;
    uint32_t n_rows;  // n_out shared by every pattern of this launch (var launch: the largest)
    // Dynamic LDS each workgroup reserves (never touched; 0 = none).  Above 64 KiB a block
    // cannot share a CU with a SHA-256 lane-kernel workgroup (>= 64 KiB reserved each), which
    // keeps a decode running beside a verification off the SHA waves' SIMDs.
    uint32_t lds_reserve;
    // Nonzero: `pat` is the codec's encode record (inputs 0..d-1, outputs d..d+p-1) and its
    // matrix equals gfc::Shape<d, p> (bs_encode_matches), so launch_rs_encode may take the
    // bit-sliced kernel of that shape.
    uint32_t std_encode;
};

// SHA-256 of n_parts * n_chunks chunks.  Strided mode: chunk (k, first_chunk + c) at
// base + k*part_stride + (first_chunk + c)*chunk_stride, len bytes, digest at (k*n_chunks+c)*32.
// List mode (ptrs != nullptr): item i hashes lens[i] bytes at ptrs[i] (n_parts = items,
// n_chunks = 1).
struct ShaParams {
    const uint8_t* base;
    uint64_t part_stride;
    uint64_t chunk_stride;
    uint64_t len;
    const uint64_t* ptrs;
    const uint64_t* lens;
    uint32_t n_parts;
    uint32_t first_chunk;
    uint32_t n_chunks;
    uint8_t* digests;     // may be null when only verifying
    // Verify mode (DataVerifier::verify): items with present[item] == 0 are skipped (ok = 0);
    // ok[item] = digest == expected[item*32 .. +32].  All three optional (device pointers).
    const uint8_t* present;
    const uint8_t* expected;
    uint8_t* ok;
    // Compacted item list (nullable, lane kernel only): lane g hashes item items[g] of the
    // strided batch, g < n_items; present is ignored and unlisted items are not touched.  Packs
    // the loaded chunks of a read into full waves (RS(10,4), d of 14 loaded: 640 waves, not 896).
    const uint32_t* items;
    uint32_t n_items;
};

struct FillParams {
    uint8_t* base;
    uint64_t part_stride;
    uint64_t chunk_stride;
    uint64_t len;
    uint64_t seed;
    uint32_t n_parts;
    uint32_t n_chunks;
};

// Fused encode_sep + SHA-256 of all d+p chunks (fused_kernels.hip).  Encode tables come from
// the codec's encode pattern record `pat`; digests as in ShaParams ((k*(d+p) + i) * 32).
struct FusedParams {
    uint8_t* base;
    uint64_t part_stride;
    uint64_t chunk_stride;
    uint64_t len;
    const uint32_t* pat;
    uint8_t* digests;
    uint32_t n_parts;
    uint32_t d;
    uint32_t p;
    uint32_t parts_per_wg;  // set by launch_encode_hash
    uint32_t enc_prio;      // set by launch_encode_hash: 1 = encoder waves, 2 = SHA waves at s_setprio 1
};

hipError_t launch_rs_apply(const ApplyParams& a, bool vec16, hipStream_t s);
// encode_sep over a batch: the bit-sliced kernel of the shape when a.std_encode, the layout is
// 16-byte aligned and (d, p) is one of the compiled shapes; launch_rs_apply otherwise.
hipError_t launch_rs_encode(const ApplyParams& a, bool vec16, hipStream_t s);
// Whether a codec's parity rows (p x d bytes, row-major) are those of a compiled bit-sliced
// shape (the compile-time construction of gf_const.hpp, compared byte for byte).
bool bs_encode_matches(uint32_t d, uint32_t p, const uint8_t* parity_rows);
// Listed parts whose patterns carry their own row count (1..max_var_rows()), one launch.
// a.n_rows selects the kernel's row class (2, 4 or 8 rows) and MUST be at least the widest
// listed pattern's row count, or 0 (unknown: the 8-row class); a pattern wider than its class is
// skipped in the kernel (its chunks are not written).  The caller (capi.cpp reconstruct_batch)
// checks this against the host records before every launch.
hipError_t launch_rs_apply_var(const ApplyParams& a, bool vec16, hipStream_t s);
uint32_t max_var_rows();
bool fused_supported(uint32_t d, uint32_t p);
bool fused_covers(uint32_t d, uint32_t p, uint64_t len);
hipError_t launch_encode_hash(const FusedParams& a, bool vec16, hipStream_t s);
hipError_t launch_sha256(const ShaParams& a, bool vec16, hipStream_t s);
// Whether launch_sha256 takes the split producer/rounds kernel for `chunks` chunks (small
// launches: lower latency per chain); callers pick separate encode + SHA over the fused kernel
// when it does.
bool use_split(uint64_t chunks);
int device_cus();  // CUs of the current device
hipError_t launch_fill(const FillParams& a, hipStream_t s);

// Packed <-> batch chunk moves (move_kernels.hip): packed chunk j (len bytes at packed + j*len)
// is batch chunk ids[j] = k*t + i (at batch + k*part_stride + i*chunk_stride); to_batch = 1
// scatters packed -> batch, 0 gathers batch -> packed.  Device memory on both sides.
struct MoveParams {
    uint8_t* batch;
    uint64_t part_stride;
    uint64_t chunk_stride;
    uint32_t t;
    uint8_t* packed;
    uint64_t len;
    const uint32_t* ids;
    uint32_t n;
    uint32_t to_batch;
    // nullable: chunk j of the packed side is at packed + packed_ids[j] * len (else j * len)
    const uint32_t* packed_ids = nullptr;
};
hipError_t launch_move_chunks(const MoveParams& a, hipStream_t s);

// CEC_READ_CARRY's stash, queued in the batch's own stream after the verification: every part
// with 0 < verified chunks < d (the parts wait() will report CEC_TOO_FEW_SHARDS_PRESENT) gets the
// next of the `n_reserved` pool entries the host reserved for this batch, in part order, and its
// verified chunks (present == CEC_PRESENT_VERIFIED, or loaded and ok) are copied to
// pool + (entry * t + i) * len.  map[k] = the entry of part k, or -1 (none needed, or the
// reservation ran out).
struct CarryStashParams {
    const uint8_t* batch;
    uint64_t part_stride;
    uint64_t chunk_stride;
    uint32_t t;
    uint32_t d;
    uint32_t n_parts;
    uint8_t* pool;
    uint64_t len;             // bytes per chunk copied (the pool's chunk stride)
    const uint8_t* present;   // device [n_parts][t]: the caller's loaded flags
    const uint8_t* ok;        // device [n_parts][t]: verification of the freshly loaded chunks
    const uint32_t* reserved;
    uint32_t n_reserved;
    int32_t* map;             // device [n_parts]
};
hipError_t launch_carry_stash(const CarryStashParams& a, hipStream_t s);

// Host mirror of the device generator (cec_synth_byte).
uint8_t synth_byte(uint64_t seed, uint64_t part, uint64_t chunk, uint64_t offset);

}  // namespace cec
