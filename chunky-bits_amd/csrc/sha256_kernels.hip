// sha256_kernels.hip — FIPS 180-4 SHA-256 of many chunks on gfx950 (Sha256Hash::from_buf,
// reference src/file/hash/sha256.rs:20-26, called per chunk at src/file/file_part.rs:185 and
// through DataVerifier::verify_async at file_part.rs:102,239,280).
//
// A chunk is a serial chain of 64-byte compressions, so the parallelism is the number of chunks
// (C2: 4096 parts x 14 = 57 344 streams, i.e. under one wave per SIMD).  Measured on MI355X, a
// lone wave issues a VALU op every ~5 cycles at best and a dependent op every ~10-11, and the
// rotate (v_alignbit_b32) and 3-input add (v_add3_u32) that SHA-256 lives on are half-rate ops:
// one wave per SIMD is issue-bound.  Two kernels:
//
//  sha256_lane_kernel   (v1, default) one lane = one chunk, one wave per SIMD.  Message
//                       load, byte swap, message schedule and the 64 rounds all in one wave;
//                       T1 = (h + K[t]+W[t] + Ch) + Sigma1 adds the long-latency Sigma1 last, and
//                       Ch/Maj are single full-rate v_bitop3 (1482 VALU per block, ~4.2 cycles
//                       per instruction per wave measured: near the lone-wave issue floor).
//  sha256_split_kernel  (v2) one 128-thread workgroup = 64 chunks and TWO waves:
//                       wave 0 (producer) loads the block, byte-swaps, expands the message
//                       schedule and writes K[t]+W[t] for block b into an LDS ring slot;
//                       wave 1 (rounds) runs the 64 rounds of block b-1 from the other slot.
//                       One __syncthreads per block hands the slot over.  Doubles the waves
//                       per SIMD, but the half-rate rotate/add3 ops then saturate the shared
//                       SIMDs and the lock-step barrier costs more than it saves (measured
//                       slower than v1; kept as the reference for the producer/consumer split).
#include <cstdlib>

#include "device_common.hpp"
#include "kernels.hpp"
#include "knobs.hpp"
#include "sha256_device.hpp"

namespace cec {
namespace {

using namespace sha;

// Chunk `item` of the launch: pointer and length (strided or list mode).
__device__ __forceinline__ void item_source(const ShaParams& a, uint32_t item, const uint8_t*& p,
                                            uint64_t& len) {
    if (a.ptrs) {
        p = reinterpret_cast<const uint8_t*>(a.ptrs[item]);
        len = a.lens[item];
    } else {
        const uint32_t k = item / a.n_chunks;
        const uint32_t c = item - k * a.n_chunks;
        p = a.base + uint64_t(k) * a.part_stride + uint64_t(a.first_chunk + c) * a.chunk_stride;
        len = a.len;
    }
}

// Digest out and/or compare with the expected digest (verify mode).
__device__ __forceinline__ void finish_item(const ShaParams& a, uint32_t item,
                                            const uint32_t st[8]) {
    if (a.digests) store_digest(a.digests + uint64_t(item) * 32u, st);
    if (a.expected && a.ok) {
        const uint4* e = reinterpret_cast<const uint4*>(a.expected + uint64_t(item) * 32u);
        const uint4 e0 = e[0], e1 = e[1];
        const bool eq = e0.x == bswap32(st[0]) && e0.y == bswap32(st[1]) &&
                        e0.z == bswap32(st[2]) && e0.w == bswap32(st[3]) &&
                        e1.x == bswap32(st[4]) && e1.y == bswap32(st[5]) &&
                        e1.z == bswap32(st[6]) && e1.w == bswap32(st[7]);
        a.ok[item] = eq ? 1 : 0;
    }
}

// ------------------------------------------------------------------------------------------
// v1: one lane per chunk, everything in one wave
// ------------------------------------------------------------------------------------------

// 256-thread workgroups: the four waves of a workgroup land on the four SIMDs of a CU, and
// launch_sha256 reserves enough (otherwise unused) LDS that at most one such workgroup fits on
// a CU.  The waves of this kernel live for the whole launch, so this pins exactly one wave per
// SIMD whatever ran before: without it, launched behind the encode kernel the dispatcher stacked
// two waves on some SIMDs and the launch took 80 ms instead of 42 ms (C2, MI355X).
constexpr int kLaneThreads = 256;

template <bool VEC>
__global__ __launch_bounds__(kLaneThreads) void sha256_lane_kernel(ShaParams a) {
    extern __shared__ uint32_t cu_reservation[];  // never touched: occupancy control only
    uint32_t item = blockIdx.x * uint32_t(kLaneThreads) + threadIdx.x;
    if (a.items) {
        if (item >= a.n_items) return;
        item = a.items[item];
    } else {
        if (item >= a.n_parts * a.n_chunks) return;
        if (a.present && !a.present[item]) {
            if (a.ok) a.ok[item] = 0;
            return;
        }
    }
    const uint8_t* p;
    uint64_t len;
    item_source(a, item, p, len);
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = kH0[i];
    const uint64_t nfull = len >> 6;
    uint32_t w[16];
    if (nfull) {
        // Blocks are loaded in pairs (one 128-byte line of an aligned chunk), both halves
        // together: every lane streams its own 1 MiB-apart chunk, so the lines of a wave share
        // L2 sets, and a line's second half loaded one block (~2.5 us) later was re-fetched from
        // HBM about half the time (PMC: 1.44-1.72x the algorithmic bytes).  The pair after the
        // current one is in flight while its second block compresses.
        uint4 q[8];
        load_block<VEC>(p, q);
        if (nfull > 1) load_block<VEC>(p + 64, q + 4);
        uint64_t b = 0;
#pragma unroll 1
        for (; b + 1 < nfull; b += 2) {
            block_words(q, w);
            compress(st, w);
            block_words(q + 4, w);
            if (b + 2 < nfull) load_block<VEC>(p + 64 * (b + 2), q);
            if (b + 3 < nfull) load_block<VEC>(p + 64 * (b + 3), q + 4);
            compress(st, w);
        }
        if (b < nfull) {  // odd block count: the last full block is in q[0..3]
            block_words(q, w);
            compress(st, w);
        }
    }
    const uint32_t rem = uint32_t(len - 64 * nfull);
    const uint32_t tb = tail_blocks(rem);
#pragma unroll 1
    for (uint32_t blk = 0; blk < tb; ++blk) {
        tail_words(p + 64 * nfull, rem, blk, tb, len * 8, w);
        compress(st, w);
    }
    finish_item(a, item, st);
}

// ------------------------------------------------------------------------------------------
// v2: producer (schedule) wave + rounds wave per 64 chunks, K+W handed over through LDS
// ------------------------------------------------------------------------------------------

// One lane's K+W row: 64 words + 4 pad words -> 272-byte stride, so the 16 lanes of each
// ds_read_b128 / ds_write_b128 lane group cover all 64 banks exactly once.
constexpr int kKwRow = 68;

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = max(v, uint32_t(__shfl_xor(int(v), m, 64)));
    return v;
}

// SPW = streams per wave.
template <bool VEC, int SPW>
__global__ __launch_bounds__(128) void sha256_split_kernel(ShaParams a) {
    __shared__ __attribute__((aligned(16))) uint32_t kw[2][SPW * kKwRow];
    const uint32_t lane = threadIdx.x & 63u;
    const bool producer = threadIdx.x < 64u;  // wave-uniform
    const uint32_t idx = blockIdx.x * uint32_t(SPW) + lane;
    bool valid = lane < uint32_t(SPW) &&
                 idx < (a.items ? a.n_items : a.n_parts * a.n_chunks);
    const uint32_t item = valid && a.items ? a.items[idx] : idx;
    bool skipped = false;  // verify mode, chunk not loaded: no blocks, ok = 0
    if (valid && !a.items && a.present && !a.present[item]) {
        skipped = true;
        valid = false;
    }
    const uint8_t* p = nullptr;
    uint64_t len = 0;
    if (valid) item_source(a, item, p, len);
    const uint64_t nfull = len >> 6;
    const uint32_t rem = uint32_t(len - 64 * nfull);
    const uint32_t nb = valid ? uint32_t(nfull) + tail_blocks(rem) : 0u;
    // Both waves hold the same 64 items, so both compute the same trip count: every lane of
    // the workgroup reaches the same number of barriers.
    const uint32_t nb_max = wave_max_u32(nb);

    if (producer) {
        // Blocks loaded in pairs, both halves of a 128-byte line together (see the lane kernel).
        uint4 q[8];
        if (nfull) load_block<VEC>(p, q);
        if (nfull > 1) load_block<VEC>(p + 64, q + 4);
#pragma unroll 1
        for (uint32_t b = 0; b <= nb_max; ++b) {
            if (b < nb) {
                uint32_t w[16];
                if (b < nfull) {
                    if (b & 1) {  // wave-uniform: static register indexing in both arms
                        block_words(q + 4, w);
                        if (b + 1 < nfull) load_block<VEC>(p + 64 * uint64_t(b + 1), q);
                        if (b + 2 < nfull) load_block<VEC>(p + 64 * uint64_t(b + 2), q + 4);
                    } else {
                        block_words(q, w);
                    }
                } else {
                    tail_words(p + 64 * nfull, rem, b - uint32_t(nfull), tail_blocks(rem),
                               len * 8, w);
                }
                uint32_t* row = &kw[b & 1][(lane % SPW) * kKwRow];
#pragma unroll
                for (int i = 0; i < 64; i += 4) {
                    uint32_t v[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        v[k] = (i + k < 16 ? w[i + k] : schedule_next(w, i + k)) + kK[i + k];
                    *reinterpret_cast<uint4*>(row + i) = make_uint4(v[0], v[1], v[2], v[3]);
                }
            }
            __syncthreads();
        }
    } else {
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = kH0[i];
#pragma unroll 1
        for (uint32_t b = 0; b <= nb_max; ++b) {
            if (b >= 1 && b - 1 < nb) {
                const uint32_t* row = &kw[(b - 1) & 1][(lane % SPW) * kKwRow];
                uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
                uint32_t x4 = st[4], x5 = st[5], x6 = st[6], x7 = st[7];
#pragma unroll
                for (int i = 0; i < 64; i += 4) {
                    const uint4 v = *reinterpret_cast<const uint4*>(row + i);
                    round_step(x0, x1, x2, x3, x4, x5, x6, x7, v.x);
                    round_step(x0, x1, x2, x3, x4, x5, x6, x7, v.y);
                    round_step(x0, x1, x2, x3, x4, x5, x6, x7, v.z);
                    round_step(x0, x1, x2, x3, x4, x5, x6, x7, v.w);
                }
                st[0] += x0;
                st[1] += x1;
                st[2] += x2;
                st[3] += x3;
                st[4] += x4;
                st[5] += x5;
                st[6] += x6;
                st[7] += x7;
            }
            __syncthreads();
        }
        if (valid) finish_item(a, item, st);
        else if (skipped && a.ok) a.ok[item] = 0;
    }
}

#ifdef CEC_AB_TOOLS
// ------------------------------------------------------------------------------------------
// v3: split with balanced placement.  512-thread workgroup, one per CU (LDS ring > 80 KiB):
// waves 0-3 producers, waves 4-7 rounds, so every SIMD carries exactly one rounds wave and one
// producer wave (waves of a workgroup are dealt to the 4 SIMDs round-robin).  224 streams per
// workgroup (56 per wave pair): C2's 57 344 chunks fill the 256 CUs in one pass.
// Strided mode with one chunk length (every lane has the same block count).
// ------------------------------------------------------------------------------------------
constexpr uint32_t kS4Spw = 56;
constexpr uint32_t kS4Streams = 4 * kS4Spw;
constexpr size_t kS4Lds = size_t(2) * 256 * kKwRow * 4;  // 2 slots x 256 rows

__device__ __forceinline__ void round_split(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                            uint32_t& e, uint32_t& f, uint32_t& g, uint32_t& h,
                                            uint32_t kw) {
    const uint32_t x = h + kw + ch(e, f, g);
    const uint32_t y = x + big_s1(e);
    const uint32_t na = y + big_s0(a) + maj(a, b, c);
    h = g;
    g = f;
    f = e;
    e = d + y;
    d = c;
    c = b;
    b = a;
    a = na;
}

// MODE (timing experiments only): 0 = normal, 1 = producers only hand over (no schedule work),
// 2 = rounds waves only hand over (no rounds work).
template <bool PRIO, int MODE = 0>
__global__ __launch_bounds__(512) void sha256_split4_kernel(ShaParams a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t kw4[];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const bool producer = wave < 4u;
    // Ring row = wave pair * 64 + lane.  Lanes without a stream of their own (lanes 56-63, past
    // the last chunk) hash a copy of the workgroup's first chunk and store nothing: no lane
    // branches, so the waitcnt that guards each prefetch is exact.
    const uint32_t slot_lane = (wave & 3u) * 64u + lane;
    const uint32_t item = blockIdx.x * kS4Streams + (wave & 3u) * kS4Spw + lane;
    const bool valid = lane < kS4Spw && item < a.n_parts * a.n_chunks;
    const uint32_t src_item = valid ? item : blockIdx.x * kS4Streams;
    const uint64_t len = a.len;
    const uint64_t nfull = len >> 6;
    const uint32_t rem = uint32_t(len - 64 * nfull);
    const uint32_t tb = tail_blocks(rem);
    const uint32_t nb = uint32_t(nfull) + tb;
    const uint8_t* p = nullptr;
    uint64_t dummy;
    item_source(a, src_item, p, dummy);
    if (producer) {
        // K[t]+W[t] of one block into ring slot `slot`
        auto produce = [&](uint32_t w[16], uint32_t slot) {
            if (MODE == 1) return;
            uint32_t* row = &kw4[(slot * 256u + slot_lane) * kKwRow];
#pragma unroll
            for (int i = 0; i < 64; i += 4) {
                uint32_t v[4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    v[k] = (i + k < 16 ? w[i + k] : schedule_next(w, i + k)) + kK[i + k];
                *reinterpret_cast<uint4*>(row + i) = make_uint4(v[0], v[1], v[2], v[3]);
            }
        };
        auto load = [&](uint4 q[4], uint64_t blk) {
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = gload16(p + 64 * blk + 16 * i);
        };
        // Full blocks, unrolled by two with two register sets so the next block's load stays
        // in flight across the barrier (no copy back into a loop-carried set).
        uint4 qa[4], qb[4];
        const uint32_t nf = uint32_t(nfull);
        // loads past the last full block re-read it (no branch around the prefetch)
        if (nf) load(qa, 0);
#pragma unroll 1
        for (uint32_t b = 0; b < nf; b += 2) {
            load(qb, min(b + 1, nf - 1));
            {
                uint32_t w[16];
                block_words(qa, w);
                produce(w, b & 1u);
            }
            lds_barrier();
            if (b + 1 < nf) {
                load(qa, min(b + 2, nf - 1));
                uint32_t w[16];
                block_words(qb, w);
                produce(w, (b + 1) & 1u);
                lds_barrier();
            }
        }
#pragma unroll 1
        for (uint32_t t = 0; t < tb; ++t) {
            uint32_t w[16];
            tail_words(p + 64 * nfull, rem, t, tb, len * 8, w);
            produce(w, (nf + t) & 1u);
            lds_barrier();
        }
        lds_barrier();  // matches the rounds waves' last hand-over
    } else {
        // The rounds waves carry the serial chain: let them win VALU arbitration (they are
        // the younger half and would otherwise get the producers' leftover issue slots).
        if (PRIO && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = kH0[i];
        lds_barrier();
#pragma unroll 1
        for (uint32_t b = 0; b < nb; ++b) {
            if (MODE != 2) {
                const uint32_t* row = &kw4[((b & 1u) * 256u + slot_lane) * kKwRow];
                uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
                uint32_t x4 = st[4], x5 = st[5], x6 = st[6], x7 = st[7];
#pragma unroll
                for (int i = 0; i < 64; i += 4) {
                    const uint4 v = *reinterpret_cast<const uint4*>(row + i);
                    round_split(x0, x1, x2, x3, x4, x5, x6, x7, v.x);
                    round_split(x0, x1, x2, x3, x4, x5, x6, x7, v.y);
                    round_split(x0, x1, x2, x3, x4, x5, x6, x7, v.z);
                    round_split(x0, x1, x2, x3, x4, x5, x6, x7, v.w);
                }
                st[0] += x0;
                st[1] += x1;
                st[2] += x2;
                st[3] += x3;
                st[4] += x4;
                st[5] += x5;
                st[6] += x6;
                st[7] += x7;
            }
            lds_barrier();
        }
        if (valid) finish_item(a, item, st);
    }
}

template <bool PRIO, int MODE = 0>
hipError_t launch_split4(const ShaParams& a, hipStream_t s) {
    static const bool attr_ok =
        hipFuncSetAttribute(reinterpret_cast<const void*>(&sha256_split4_kernel<PRIO, MODE>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(kS4Lds)) == hipSuccess;
    if (!attr_ok) return hipErrorInvalidValue;
    const uint64_t total = uint64_t(a.n_parts) * a.n_chunks;
    dim3 grid(uint32_t((total + kS4Streams - 1) / kS4Streams));
    clear_stale_error();
    hipLaunchKernelGGL((sha256_split4_kernel<PRIO, MODE>), grid, dim3(512), kS4Lds, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// v5: the v3 split with per-pair hand-over counters in LDS instead of workgroup barriers.  A
// rounds wave waits only for ITS producer's block (produced[pair] > b) and a producer only for
// its slot to be consumed (consumed[pair] >= b - 1, two slots), so the four pairs of a CU no
// longer lock-step each other at every block.  Waits spin with s_sleep and give up after
// ~2^20 polls (a wave that gave up stops waiting and runs to its end: wrong digests, never a
// hang); in a correct run a wait lasts at most about one block.
// ------------------------------------------------------------------------------------------
constexpr size_t kS5Ring = size_t(2) * 256 * kKwRow;  // words
constexpr size_t kS5Lds = kS5Ring * 4 + 64;

__device__ __forceinline__ void s5_wait_ge(const uint32_t* c, uint32_t target, bool& dead) {
    uint32_t spins = 0;
    while (!dead) {
        const uint32_t v = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const volatile uint32_t*>(c));
        if (v >= target) break;
        if (++spins > (1u << 20)) dead = true;
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void s5_publish(uint32_t* c, uint32_t v) {
    // this wave's ring writes / reads are done before the counter moves (LDS only: global
    // prefetches stay in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    *reinterpret_cast<volatile uint32_t*>(c) = v;
}

template <bool PRIO>
__global__ __launch_bounds__(512) void sha256_split5_kernel(ShaParams a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s5[];
    uint32_t* cnt = s5 + kS5Ring;  // [0, 4) produced blocks per pair, [4, 8) consumed
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t pair = wave & 3u;
    const bool producer = wave < 4u;
    if (threadIdx.x < 8u) cnt[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t slot_lane = pair * 64u + lane;
    const uint32_t item = blockIdx.x * kS4Streams + pair * kS4Spw + lane;
    const bool valid = lane < kS4Spw && item < a.n_parts * a.n_chunks;
    const uint32_t src_item = valid ? item : blockIdx.x * kS4Streams;
    const uint64_t len = a.len;
    const uint64_t nfull = len >> 6;
    const uint32_t rem = uint32_t(len - 64 * nfull);
    const uint32_t tb = tail_blocks(rem);
    const uint32_t nb = uint32_t(nfull) + tb;
    const uint8_t* p = nullptr;
    uint64_t dummy;
    item_source(a, src_item, p, dummy);
    bool dead = false;
    if (producer) {
        auto produce = [&](uint32_t w[16], uint32_t b) {
            if (b >= 2) s5_wait_ge(&cnt[4 + pair], b - 1, dead);
            uint32_t* row = &s5[((b & 1u) * 256u + slot_lane) * kKwRow];
#pragma unroll
            for (int i = 0; i < 64; i += 4) {
                uint32_t v[4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    v[k] = (i + k < 16 ? w[i + k] : schedule_next(w, i + k)) + kK[i + k];
                *reinterpret_cast<uint4*>(row + i) = make_uint4(v[0], v[1], v[2], v[3]);
            }
            s5_publish(&cnt[pair], b + 1);
        };
        auto load = [&](uint4 q[4], uint64_t blk) {
#pragma unroll
            for (int i = 0; i < 4; ++i) q[i] = gload16(p + 64 * blk + 16 * i);
        };
        uint4 qa[4], qb[4];
        const uint32_t nf = uint32_t(nfull);
        if (nf) load(qa, 0);
#pragma unroll 1
        for (uint32_t b = 0; b < nf; b += 2) {
            load(qb, min(b + 1, nf - 1));
            {
                uint32_t w[16];
                block_words(qa, w);
                produce(w, b);
            }
            if (b + 1 < nf) {
                load(qa, min(b + 2, nf - 1));
                uint32_t w[16];
                block_words(qb, w);
                produce(w, b + 1);
            }
        }
#pragma unroll 1
        for (uint32_t t = 0; t < tb; ++t) {
            uint32_t w[16];
            tail_words(p + 64 * nfull, rem, t, tb, len * 8, w);
            produce(w, nf + t);
        }
    } else {
        if (PRIO) __builtin_amdgcn_s_setprio(1);
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = kH0[i];
#pragma unroll 1
        for (uint32_t b = 0; b < nb; ++b) {
            s5_wait_ge(&cnt[pair], b + 1, dead);
            const uint32_t* row = &s5[((b & 1u) * 256u + slot_lane) * kKwRow];
            uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
            uint32_t x4 = st[4], x5 = st[5], x6 = st[6], x7 = st[7];
#pragma unroll
            for (int i = 0; i < 64; i += 4) {
                const uint4 v = *reinterpret_cast<const uint4*>(row + i);
                round_split(x0, x1, x2, x3, x4, x5, x6, x7, v.x);
                round_split(x0, x1, x2, x3, x4, x5, x6, x7, v.y);
                round_split(x0, x1, x2, x3, x4, x5, x6, x7, v.z);
                round_split(x0, x1, x2, x3, x4, x5, x6, x7, v.w);
            }
            st[0] += x0;
            st[1] += x1;
            st[2] += x2;
            st[3] += x3;
            st[4] += x4;
            st[5] += x5;
            st[6] += x6;
            st[7] += x7;
            s5_publish(&cnt[4 + pair], b + 1);
        }
        if (valid) finish_item(a, item, st);
    }
}

template <bool PRIO>
hipError_t launch_split5(const ShaParams& a, hipStream_t s) {
    static const bool attr_ok =
        hipFuncSetAttribute(reinterpret_cast<const void*>(&sha256_split5_kernel<PRIO>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(kS5Lds)) == hipSuccess;
    if (!attr_ok) return hipErrorInvalidValue;
    const uint64_t total = uint64_t(a.n_parts) * a.n_chunks;
    dim3 grid(uint32_t((total + kS4Streams - 1) / kS4Streams));
    clear_stale_error();
    hipLaunchKernelGGL((sha256_split5_kernel<PRIO>), grid, dim3(512), kS5Lds, s, a);
    return hipGetLastError();
}

#endif  // CEC_AB_TOOLS

// CEC_SHA_VARIANT: 1 = lane kernel, 2 = split kernel (both correct; by size when unset).  The
// experiment kernels 3-5, 7, 8 (7/8 timing attribution with wrong outputs by design) exist only
// in the A/B build (-DCEC_AB_TOOLS): the product library treats them as unset.
int sha_variant() {
    const int v = knobs().sha_variant;
#ifdef CEC_AB_TOOLS
    return v;
#else
    return v == 1 || v == 2 ? v : 0;
#endif
}

// Dynamic LDS requested per lane-kernel workgroup: more than half of the 160 KiB of a CU, so
// two workgroups never share a CU.
constexpr size_t kCuReservation = 96 * 1024;
// ... and at most two (grids larger than one workgroup per CU).
constexpr size_t kCuReservation2 = 64 * 1024;


hipError_t launch_lane(const ShaParams& a, bool vec16, hipStream_t s, bool one_per_cu = false) {
    static const bool attr_ok = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&sha256_lane_kernel<true>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   int(kCuReservation)) == hipSuccess &&
               hipFuncSetAttribute(reinterpret_cast<const void*>(&sha256_lane_kernel<false>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                   int(kCuReservation)) == hipSuccess;
    }();
    if (!attr_ok) return hipErrorInvalidValue;
    const uint64_t total = a.items ? a.n_items : uint64_t(a.n_parts) * a.n_chunks;
    dim3 grid(uint32_t((total + kLaneThreads - 1) / kLaneThreads));
    // One workgroup (one wave per SIMD) per CU while the grid fits the chip in one pass.  When
    // it does not, a second co-resident wave per SIMD turns the lone wave's issue-bound ~6000
    // cycles per block into a shared SIMD-bound ~5100 per wave: every wave starts at once
    // instead of a second, partly empty pass.
    const size_t lds =
        (!one_per_cu && grid.x > uint32_t(device_cus())) ? kCuReservation2 : kCuReservation;
    clear_stale_error();
    if (vec16)
        hipLaunchKernelGGL((sha256_lane_kernel<true>), grid, dim3(kLaneThreads), lds, s, a);
    else
        hipLaunchKernelGGL((sha256_lane_kernel<false>), grid, dim3(kLaneThreads), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_split(const ShaParams& a, bool vec16, hipStream_t s) {
    const uint64_t total = a.items ? a.n_items : uint64_t(a.n_parts) * a.n_chunks;
    dim3 grid(uint32_t((total + 63) / 64));
    clear_stale_error();
    if (vec16) hipLaunchKernelGGL((sha256_split_kernel<true, 64>), grid, dim3(128), 0, s, a);
    else hipLaunchKernelGGL((sha256_split_kernel<false, 64>), grid, dim3(128), 0, s, a);
    return hipGetLastError();
}

}  // namespace

// CUs of the current device (cached per device ordinal).
int device_cus() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cache[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

// Chunks up to which a launch takes the split kernel: its 2 waves per 64 chunks then fill at
// most a quarter of the SIMDs (4 x CUs), leaving room for the other launches in flight (write /
// read pipeline slots, coalesced per-call batches: 4 each).  Past it the chip fills and the lane
// kernel's one wave per 64 chunks wins (C2: split 50.6 ms vs lane 42.1 ms).
uint64_t split_max_chunks() { return uint64_t(device_cus()) * 32; }

bool use_split(uint64_t chunks) {
    const int v = sha_variant();
    if (v) return v == 2;
    return chunks <= split_max_chunks();
}

// CEC_SHA_VARIANT (tuning knob, read per launch): unset = by size (use_split), 1 = one lane per
// chunk, 2 = split producer/rounds waves, 3/4/5/7/8 = experiments.  A lone 1 MiB chain: lane
// kernel ~42 ms, split kernel ~31 ms (rounds wave alone on its SIMD; tools/sha_ab.py,
// profiles/r1z_sha_ab_small.log).
hipError_t launch_sha256(const ShaParams& a, bool vec16, hipStream_t s) {
    const uint64_t total = a.items ? a.n_items : uint64_t(a.n_parts) * a.n_chunks;
    if (total == 0) return hipSuccess;
    const int v = sha_variant();
    if (use_split(total)) return launch_split(a, vec16, s);
    if (a.items) return launch_lane(a, vec16, s);
#ifdef CEC_AB_TOOLS
    if (v == 3 && !a.present && !a.ptrs && vec16) return launch_split4<false>(a, s);
    if (v == 4 && !a.present && !a.ptrs && vec16) return launch_split4<true>(a, s);
    if (v == 7 && !a.present && !a.ptrs && vec16) return launch_split4<true, 1>(a, s);
    if (v == 8 && !a.present && !a.ptrs && vec16) return launch_split4<true, 2>(a, s);
    if (v == 5) return launch_lane(a, vec16, s, true);
    if (v == 9 && !a.present && !a.ptrs && vec16) return launch_split5<false>(a, s);
    if (v == 10 && !a.present && !a.ptrs && vec16) return launch_split5<true>(a, s);
#else
    (void)v;
#endif
    return launch_lane(a, vec16, s);
}

}  // namespace cec
