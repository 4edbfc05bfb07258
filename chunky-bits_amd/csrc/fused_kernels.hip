// fused_kernels.hip — encode_hash_kernel: FilePart::write_with_encoder's compute for many parts
// in one launch (reference src/file/file_part.rs:150-185): encode_sep of the p parity chunks and
// SHA-256 of all d+p chunks, with every data byte read from HBM once and every parity byte
// written once and hashed from LDS (never re-read).
//
// Workgroup = 512 threads, one per CU:
//   waves 0-3  SHA lanes: lane = one chunk of one of the workgroup's G parts (G*(d+p) <= 256;
//              RS(10,4): 16 parts = 224 lanes), so each SIMD carries exactly one SHA wave —
//              the long-lived, issue-bound wave that sets the pace (sha256_kernels.hip).
//   waves 4-7  encoders: per pipeline step of STEP bytes, load the G*d data columns (16 B per
//              lane) from HBM into an LDS slot, compute the G*p parity columns with the v_perm
//              GF(2^8) multiply (gf_device.hpp), write them to the slot and to HBM.
// Double-buffered LDS ring [2][G*(d+p)][STEP+16]: while the SHA waves hash slot s%2 the
// encoders fill slot (s+1)%2; one barrier per step hands the slots over.  The encoders hold the
// next step's d inputs in registers (loads issued right after the current step's compute) and
// hand over with lgkmcnt(0) + s_barrier, so HBM latency never sits on the step.  The ring
// (≈122 KB for RS(10,4)) also keeps a second workgroup off the CU.  The encoder waves share each
// SIMD with a SHA wave and use the issue slots it leaves (it runs ~4.2 cycles per VALU op,
// below the SIMD's rate).
#include <algorithm>
#include <cstdlib>

#include "device_common.hpp"
#include "gf256.hpp"
#include "gf_device.hpp"
#include "kernels.hpp"
#include "knobs.hpp"
#include "sha256_device.hpp"

namespace cec {
namespace {

using namespace gf;
using namespace sha;

constexpr uint32_t kShaLanes = 256;   // SHA lanes of the one-wave-per-SIMD build (SW = 4)
constexpr uint32_t kEncThreads = 256;  // 4 encoder waves in every build
constexpr int kMaxFusedData = 16;  // generic build: d <= 16 (RS(20,p) has its own build)

// 4x4 byte transpose: r_k byte i = a_i byte k.  acc words hold, per data byte position, the
// products of all parity rows (row r in byte r); the transpose turns 4 byte positions into one
// output word per row.  8 v_perm per 4 words.
__device__ __forceinline__ void transpose4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                           uint32_t r[4]) {
    const uint32_t t01 = perm(a1, a0, 0x05010400u), t23 = perm(a3, a2, 0x05010400u);
    const uint32_t u01 = perm(a1, a0, 0x07030602u), u23 = perm(a3, a2, 0x07030602u);
    r[0] = perm(t23, t01, 0x05040100u);
    r[1] = perm(t23, t01, 0x07060302u);
    r[2] = perm(u23, u01, 0x05040100u);
    r[3] = perm(u23, u01, 0x07060302u);
}

// Byte k of w times E (E = 4 or 8): one SDWA shift (src1_sel picks the byte, zero-extended).
// The compiler's own form is v_bfe + v_lshl_add (two ops, one of them half-rate).
template <int E>
__device__ __forceinline__ uint32_t byte_scaled(uint32_t w, int k) {
    static_assert(E == 4 || E == 8, "entry size");
    uint32_t r;
    if (E == 4) {
        switch (k) {
            case 0: asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(w)); break;
            case 1: asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(w)); break;
            case 2: asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(w)); break;
            default: asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(w)); break;
        }
    } else {
        switch (k) {
            case 0: asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(w)); break;
            case 1: asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(w)); break;
            case 2: asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(w)); break;
            default: asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(w)); break;
        }
    }
    return r;
}

constexpr int col_width(int dmax) { return dmax > kMaxFusedData ? 8 : 16; }

// NW words (NW*4 bytes) of one column: a full 16- or 8-byte load, or the n < NW*4 bytes of a
// ragged chunk's last column (zero-filled).
template <int NW, bool RAGGED>
__device__ __forceinline__ void load_words(const uint8_t* src, uint64_t n, uint32_t w[NW]) {
    if (!RAGGED || n == NW * 4) {
        if (NW == 4) {
            const uint4 q = *reinterpret_cast<const uint4*>(src);
            w[0] = q.x; w[1] = q.y; w[2 % NW] = q.z; w[3 % NW] = q.w;
        } else {
            const uint2 q = *reinterpret_cast<const uint2*>(src);
            w[0] = q.x; w[1] = q.y;
        }
    } else {
        const uint4 q = load_partial(src, n);
        w[0] = q.x; w[1] = q.y;
        if (NW == 4) { w[2 % NW] = q.z; w[3 % NW] = q.w; }
    }
}

template <int NW, bool RAGGED>
__device__ __forceinline__ void store_words(uint8_t* dst, uint64_t n, const uint32_t w[NW]) {
    if (!RAGGED || n == NW * 4) {
        if (NW == 4) *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2 % NW], w[3 % NW]);
        else *reinterpret_cast<uint2*>(dst) = make_uint2(w[0], w[1]);
    } else {
        const uint32_t o4[4] = {w[0], w[1], NW == 4 ? w[2 % NW] : 0u, NW == 4 ? w[3 % NW] : 0u};
        store_partial(dst, o4, n);
    }
}

// BE builds keep every chunk in the LDS ring as big-endian 32-bit words (SHA-256's message word
// order): the encoder waves byte-swap while storing, so the SHA waves read message words
// directly (16 fewer half-rate v_perm per 64-byte block).  GF(2^8) arithmetic is byte-wise, so
// the encoders compute parity on their native words.  See fused_be() for where it pays.
template <int NW, bool BE = true>
__device__ __forceinline__ void lds_store_words(uint8_t* dst, const uint32_t w[NW]) {
    if (!BE) {
        if (NW == 4) *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2 % NW], w[3 % NW]);
        else *reinterpret_cast<uint2*>(dst) = make_uint2(w[0], w[1]);
    } else if (NW == 4)
        *reinterpret_cast<uint4*>(dst) = make_uint4(bswap32(w[0]), bswap32(w[1]),
                                                    bswap32(w[2 % NW]), bswap32(w[3 % NW]));
    else
        *reinterpret_cast<uint2*>(dst) = make_uint2(bswap32(w[0]), bswap32(w[1]));
}

// block_words for a ring row that already holds big-endian words.
__device__ __forceinline__ void ring_block_words(const uint4 q[4], uint32_t w[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w[4 * i + 0] = q[i].x;
        w[4 * i + 1] = q[i].y;
        w[4 * i + 2] = q[i].z;
        w[4 * i + 3] = q[i].w;
    }
}

// tail_words over a ring row of big-endian words: message byte pos sits at row byte pos ^ 3.
__device__ __forceinline__ void ring_tail_words(const uint8_t* tp, uint32_t rem, uint32_t blk,
                                                uint32_t tb, uint64_t bits, uint32_t w[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        uint32_t word = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t pos = blk * 64 + uint32_t(i * 4 + k);
            const uint32_t byte = pos < rem ? uint32_t(tp[pos ^ 3u]) : (pos == rem ? 0x80u : 0u);
            word = (word << 8) | byte;
        }
        w[i] = word;
    }
    if (blk == tb - 1) {
        w[14] = uint32_t(bits >> 32);
        w[15] = uint32_t(bits);
    }
}

// PMAX: parity rows (exact when a.p == PMAX; rows r >= a.p skipped by uniform guards).
// Up to kMaxFusedData data inputs are held in registers per encoder thread (next step's
// prefetch).  Aligned (16-byte) layouts only; others use the separate kernels.
// MODE (timing attribution only, CEC_FUSED_MODE): 0 = the product; 1 = encoders skip the GF
// multiply (parity = data chunk 0); 2 = encoders only join the barriers (SHA hashes whatever the
// ring holds).  Modes 1 and 2 produce wrong parity/digests by design.
// DT: data chunk count fixed at compile time (0 = a.d at run time, <= kMaxFusedData).
// SW: SHA waves per workgroup, 4 (one per SIMD) or 8 (two per SIMD: batches with more chunks
// than one wave per SIMD can hold, where two co-resident SHA waves turn the lone wave's
// issue-bound ~6000 cycles per block into a SIMD-bound ~5800 each).
// ENC3 (SW == 8 only): the column tasks run on SIMD 3 only.  Waves are dealt to the 4 SIMDs
// round-robin (wave w on SIMD w % 4), so with at most 7 SHA waves (G*(d+p) <= 448) SIMD 3
// carries ONE SHA wave where SIMDs 0-2 carry two: its spare issue slots absorb all the encoder
// work, as waves 7 (an otherwise empty SHA slot) and 11 (tasks 0-63 and 64-127; needs
// G*STEP/CW <= 128), while encoder waves 8-10 only build the product tables and join the
// barriers.  The SIMDs with two SHA waves then carry no encoder work at all.
template <int PMAX, int STEP, int MODE, int DT, int SW = 4, bool ENC3 = false, bool BE = false>
__global__ __launch_bounds__(64 * (SW + 4)) void encode_hash_kernel(FusedParams a) {
    static_assert(!ENC3 || SW == 8, "ENC3 needs the two-SHA-wave build");
    constexpr uint32_t kSha = 64u * SW;
    constexpr int DMAX = DT ? DT : kMaxFusedData;
    constexpr int kEntry = PMAX <= 4 ? 4 : 8;
    // Column width per encoder task: 16 bytes, or 8 for builds with more than 16 inputs so the
    // prefetched inputs plus accumulators stay in registers.
    constexpr int CW = col_width(DMAX);
    constexpr int NW = CW / 4;  // words per column
    // Shape builds (DT != 0) run only when len is a multiple of CW (launch_step): no ragged
    // last column, whose byte-wise path would cost the wide builds their registers.
    constexpr bool RAGGED = DT == 0;
    // LDS: product tables in static LDS (fixed addresses: input j's table base folds into the
    // ds_read instruction offset), the ring in dynamic LDS behind them.
    __shared__ __attribute__((aligned(16))) uint8_t tabs[DMAX * 256 * kEntry];
    extern __shared__ __attribute__((aligned(16))) uint8_t ring[];
    constexpr uint32_t kRow = STEP + 16;  // 16-byte pad: conflict-free 16 B per lane accesses
    constexpr uint32_t kCols = STEP / CW;
    // d is a compile-time constant only in the 4-byte-entry shape builds: with 8-byte entries
    // the per-input uniform branches of a run-time d are what keep the scheduler from hoisting
    // every input's lookups at once (fully unrolled, the RS(20,8) build spills).
    const uint32_t d = (DT && kEntry == 4) ? uint32_t(DT) : a.d, P = a.p, t = d + a.p;
    const uint32_t G = a.parts_per_wg;
    const uint32_t rows = G * t;
    const uint32_t part0 = blockIdx.x * G;
    const uint32_t g_here = min(G, a.n_parts - part0);
    const uint64_t L = a.len;
    const uint64_t cs = a.chunk_stride;
    const uint32_t n_steps = uint32_t((L + STEP - 1) / STEP);

    const uint32_t wave = threadIdx.x >> 6;
    if (threadIdx.x >= kSha || (ENC3 && wave == 7u)) {
        // ------------------------------ encoders ------------------------------
        // Each encoder thread owns one CW-byte column (g, col) of every step
        // (launch_encode_hash guarantees G*kCols <= kEncThreads).  Per step: multiply the d
        // inputs already in registers, write data + parity into the LDS slot, store parity to
        // HBM, then issue the next step's d loads (all in flight at once) before the barrier.
        // Two SHA waves saturate their SIMD: without priority the encoders would get no issue
        // slots until the SHA waves park at the step barrier, which then waits for them.
        if (a.enc_prio == 1u) __builtin_amdgcn_s_setprio(1);
        cu32* pat = as_const(a.pat);
        cu32* tab = pat + 1 + d + P;  // input j, row r at (j*P + r) * 5
        const uint32_t et = threadIdx.x - kSha;  // table builders: et < kEncThreads
        // Fewer column tasks than encoder threads (wide stripes, 128-byte steps): deal them
        // round-robin over the 4 encoder waves so every SIMD's SHA wave shares its issue slots
        // with the same amount of encoder work (the step barrier waits for the slowest SIMD).
        // ENC3: waves 7 and 11 (SIMD 3) take every task.
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t task = ENC3 ? (wave == 7u ? lane : (wave == 11u ? 64u + lane : ~0u))
                              : G * kCols < kEncThreads ? (et & 63u) * 4u + (et >> 6) : et;
        const bool has_task = task < g_here * kCols;
        const uint32_t g = task / kCols, col = task - g * kCols;
        uint8_t* pb = a.base + uint64_t(part0 + g) * a.part_stride;
        uint32_t v[DMAX][NW];
        auto load_step = [&](uint32_t s) {
            const uint64_t x = uint64_t(s) * STEP + col * CW;
            if (!has_task || x >= L || MODE == 2) return;
            const uint64_t n = (L - x) < CW ? (L - x) : CW;
            const uint8_t* src = pb + x;  // per-lane pointer walked by chunk_stride: no
                                          // per-input 64-bit base held in SGPRs
#pragma unroll
            for (int j = 0; j < DMAX; ++j) {
                if (uint32_t(j) < d) {
                    load_words<NW, RAGGED>(src, n, v[j]);
                    src += cs;
                }
            }
        };
        // Product tables in static LDS: for input j and byte value x, one entry packs c[r][j]*x
        // for every parity row r (row r in byte r; 4 B per entry for p <= 4, 8 B for p <= 8).
        // A data byte then costs one ds_read + half an xor3 for all rows, instead of three
        // half-rate v_perm per row: the GF multiply moves off the VALU the SHA waves saturate.
        if (threadIdx.x >= kSha) {
            const uint32_t x = et;  // 256 encoder threads = 256 byte values
            const Sel sx = selectors(x);
#pragma unroll 1
            for (uint32_t j = 0; j < d; ++j) {
                uint32_t lo = 0u, hi = 0u;
                cu32* tj = tab + size_t(j) * P * kTabWords;
#pragma unroll
                for (int r = 0; r < PMAX; ++r) {
                    if (uint32_t(r) >= P) break;
                    cu32* c = tj + r * kTabWords;
                    const uint32_t prod = gmul(sx, c[0], c[1], c[2], c[3], c[4]) & 0xFFu;
                    if (r < 4) lo |= prod << (8 * r);
                    else hi |= prod << (8 * (r - 4));
                }
                uint32_t* e = reinterpret_cast<uint32_t*>(tabs + (size_t(j) * 256 + x) * kEntry);
                e[0] = lo;
                if (kEntry == 8) e[1] = hi;
            }
        }
        auto emit_step = [&](uint32_t s, uint32_t slot) {
            const uint64_t x = uint64_t(s) * STEP + col * CW;
            if (!has_task || x >= L || MODE == 2) return;
            const uint64_t n = (L - x) < CW ? (L - x) : CW;
            uint8_t* lrow = ring + (size_t(slot) * rows + size_t(g) * t) * kRow + col * CW;
            uint32_t acc_lo[4 * NW], acc_hi[4 * NW];
#pragma unroll
            for (int b = 0; b < 4 * NW; ++b) acc_lo[b] = acc_hi[b] = 0u;
#pragma unroll
            for (int j = 0; j < DMAX; ++j)
                if (uint32_t(j) < d) lds_store_words<NW, BE>(lrow + size_t(j) * kRow, v[j]);
            if (MODE == 1) {
#pragma unroll
                for (int q = 0; q < NW; ++q) acc_lo[4 * q] = v[0][q];
            } else {
                // Inputs in pairs: two lookups folded into the accumulator by one full-rate
                // xor3.  Table j sits at LDS offset j*256*kEntry (an instruction offset); the
                // entry index is one byte of the data word (byte select + scale: one SDWA op).
#pragma unroll
                for (int j = 0; j < DMAX; j += 2) {
                    if (j + 1 < DMAX && uint32_t(j + 1) < d) {
                        const int j1 = j + 1 < DMAX ? j + 1 : j;
                        const uint8_t* t0 = tabs + size_t(j) * 256 * kEntry;
                        const uint8_t* t1 = tabs + size_t(j1) * 256 * kEntry;
#pragma unroll
                        for (int q = 0; q < NW; ++q) {
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                const uint32_t i0 = byte_scaled<kEntry>(v[j][q], k);
                                const uint32_t i1 = byte_scaled<kEntry>(v[j1][q], k);
                                if (kEntry == 4) {
                                    acc_lo[4 * q + k] = xor3(
                                        acc_lo[4 * q + k],
                                        *reinterpret_cast<const uint32_t*>(t0 + i0),
                                        *reinterpret_cast<const uint32_t*>(t1 + i1));
                                } else {
                                    const uint2 e0 = *reinterpret_cast<const uint2*>(t0 + i0);
                                    const uint2 e1 = *reinterpret_cast<const uint2*>(t1 + i1);
                                    acc_lo[4 * q + k] = xor3(acc_lo[4 * q + k], e0.x, e1.x);
                                    acc_hi[4 * q + k] = xor3(acc_hi[4 * q + k], e0.y, e1.y);
                                }
                            }
                        }
                    } else if (uint32_t(j) < d) {
                        const uint8_t* t0 = tabs + size_t(j) * 256 * kEntry;
#pragma unroll
                        for (int q = 0; q < NW; ++q) {
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                const uint32_t i0 = byte_scaled<kEntry>(v[j][q], k);
                                if (kEntry == 4) {
                                    acc_lo[4 * q + k] ^=
                                        *reinterpret_cast<const uint32_t*>(t0 + i0);
                                } else {
                                    const uint2 e0 = *reinterpret_cast<const uint2*>(t0 + i0);
                                    acc_lo[4 * q + k] ^= e0.x;
                                    acc_hi[4 * q + k] ^= e0.y;
                                }
                            }
                        }
                    }
                }
            }
            // rows 0..3 from acc_lo, rows 4..7 from acc_hi: out[r][q] = word q of parity row r
            uint32_t out[8][NW];
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                uint32_t r4[4];
                transpose4(acc_lo[4 * q], acc_lo[4 * q + 1], acc_lo[4 * q + 2], acc_lo[4 * q + 3],
                           r4);
                out[0][q] = r4[0];
                out[1][q] = r4[1];
                out[2][q] = r4[2];
                out[3][q] = r4[3];
                if (PMAX > 4) {
                    transpose4(acc_hi[4 * q], acc_hi[4 * q + 1], acc_hi[4 * q + 2],
                               acc_hi[4 * q + 3], r4);
                    out[4][q] = r4[0];
                    out[5][q] = r4[1];
                    out[6][q] = r4[2];
                    out[7][q] = r4[3];
                }
            }
#pragma unroll
            for (int r = 0; r < PMAX; ++r) {
                if (uint32_t(r) >= P) break;
                lds_store_words<NW, BE>(lrow + size_t(d + r) * kRow, out[r]);
                store_words<NW, RAGGED>(pb + uint64_t(d + r) * cs + x, n, out[r]);
            }
        };
        __syncthreads();  // tables built (the SHA waves join this barrier too)
        load_step(0);
        emit_step(0, 0);
        if (n_steps > 1) load_step(1);
        lds_barrier();
#pragma unroll 1
        for (uint32_t s = 0; s < n_steps; ++s) {
            if (s + 1 < n_steps) {
                emit_step(s + 1, (s + 1) & 1u);
                if (s + 2 < n_steps) load_step(s + 2);
            }
            lds_barrier();
        }
    } else {
        // ------------------------------ SHA lanes ------------------------------
        if (a.enc_prio == 2u) __builtin_amdgcn_s_setprio(1);  // A/B: SHA waves first
        const uint32_t lane = threadIdx.x;
        const bool valid = lane < g_here * t;
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = kH0[i];
        const uint64_t nfull = L >> 6;
        uint32_t w[16];
        __syncthreads();  // encoders' product tables built
        __syncthreads();  // slot 0 filled
#pragma unroll 1
        for (uint32_t s = 0; s < n_steps; ++s) {
            if (valid) {
                const uint8_t* row = ring + (size_t(s & 1u) * rows + lane) * kRow;
                const uint64_t b0 = uint64_t(s) * (STEP / 64);
                const uint64_t b1 = (b0 + STEP / 64) < nfull ? (b0 + STEP / 64) : nfull;
#pragma unroll 1
                for (uint64_t b = b0; b < b1; ++b) {
                    const uint4* q = reinterpret_cast<const uint4*>(row + (b - b0) * 64);
                    const uint4 qq[4] = {q[0], q[1], q[2], q[3]};
                    if (BE) ring_block_words(qq, w);
                    else block_words(qq, w);
                    compress(st, w);
                }
                if (s + 1 == n_steps) {
                    const uint32_t rem = uint32_t(L - 64 * nfull);
                    const uint32_t tb = tail_blocks(rem);
                    const uint8_t* tp = row + (64 * nfull - uint64_t(s) * STEP);
#pragma unroll 1
                    for (uint32_t blk = 0; blk < tb; ++blk) {
                        if (BE) ring_tail_words(tp, rem, blk, tb, L * 8, w);
                        else tail_words(tp, rem, blk, tb, L * 8, w);
                        compress(st, w);
                    }
                }
            }
            __syncthreads();
        }
        if (valid) {
            const uint32_t g = lane / t, i = lane - g * t;
            store_digest(a.digests + (uint64_t(part0 + g) * t + i) * 32u, st);
        }
    }
}

template <int PMAX, int STEP, int MODE, int DT, int SW = 4, bool ENC3 = false, bool BE = false>
hipError_t launch_p(const FusedParams& a, hipStream_t s) {
    const size_t lds = size_t(2) * a.parts_per_wg * (a.d + a.p) * (STEP + 16);  // ring
    const size_t tabs = size_t(DT ? DT : kMaxFusedData) * 256 * (PMAX <= 4 ? 4 : 8);
    if (lds + tabs > 160 * 1024) return hipErrorInvalidValue;
    static const bool attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&encode_hash_kernel<PMAX, STEP, MODE, DT, SW, ENC3, BE>),
        hipFuncAttributeMaxDynamicSharedMemorySize,
        int(160 * 1024 - size_t(DT ? DT : kMaxFusedData) * 256 * (PMAX <= 4 ? 4 : 8))) ==
        hipSuccess;
    if (!attr) return hipErrorInvalidValue;
    const uint32_t grid = (a.n_parts + a.parts_per_wg - 1) / a.parts_per_wg;
    clear_stale_error();
    hipLaunchKernelGGL((encode_hash_kernel<PMAX, STEP, MODE, DT, SW, ENC3, BE>), dim3(grid),
                       dim3(64 * (SW + 4)), lds, s, a);
    return hipGetLastError();
}

// Wave priorities: 0 = none, 1 = encoder waves at s_setprio 1, 2 = SHA waves at s_setprio 1.
// The build's default, or CEC_FUSED_PRIO=0/1/2 (dev knob, A/B).
uint32_t fused_prio(uint32_t dflt) {
    const int v = knobs().fused_prio;
    return v >= 0 ? uint32_t(v) : dflt;
}

// Byte order of the LDS ring (BE = encoders store big-endian words, the SHA waves skip their
// 16 byte-swaps per block).  It pays where the encoders run on a SIMD with spare issue slots
// (the ENC3 build: C4 21.06 -> 20.47 ms) and costs where they share a saturated SIMD with a SHA
// wave (RS(10,4) build: C2 42.63 -> 42.97 ms), so it is on for ENC3 only.  CEC_FUSED_BE=0/1
// overrides (A/B).
bool fused_be(bool dflt) {
    const int v = knobs().fused_be;
    return v >= 0 ? v == 1 : dflt;
}

// CEC_FUSED_ENC3=0 turns the SIMD-3 encoder placement of the two-SHA-wave build off (A/B).
bool fused_enc3() { return knobs().fused_enc3; }

// CEC_FUSED_MODE: 3 = the generic-d build on every shape it covers (correct output; A/B and
// tests against the shape builds).  Modes 1 and 2 (timing attribution, wrong outputs by design)
// exist only in the A/B build (-DCEC_AB_TOOLS, `make ab`): the product library ignores them.
int fused_mode() {
    const int m = knobs().fused_mode;
#ifdef CEC_AB_TOOLS
    return m;
#else
    return m == 3 ? 3 : 0;
#endif
}

template <int STEP>
hipError_t launch_step(const FusedParams& a, hipStream_t s) {
    const int mode = fused_mode();
    if constexpr (STEP == 256) {
#ifdef CEC_AB_TOOLS
        if (mode == 1)
            return a.p == 4 ? launch_p<4, STEP, 1, 0>(a, s) : launch_p<8, STEP, 1, 0>(a, s);
        if (mode == 2)
            return a.p == 4 ? launch_p<4, STEP, 2, 0>(a, s) : launch_p<8, STEP, 2, 0>(a, s);
#endif
        // mode 3: the generic-d build on every shape it covers (A/B and tests against the
        // shape builds)
        if (mode != 3 && a.d == 10 && a.p == 4 && a.len % col_width(10) == 0)
            return fused_be(false) ? launch_p<4, STEP, 0, 10, 4, false, true>(a, s)
                                   : launch_p<4, STEP, 0, 10, 4, false, false>(a, s);
    }
    if constexpr (STEP == 128) {
        if (a.d == 20) {  // RS(20, p <= 8); launch_encode_hash checked len % col_width(20)
            return launch_p<8, STEP, 0, 20>(a, s);
        }
    }
    return a.p <= 4 ? launch_p<4, STEP, 0, 0>(a, s) : launch_p<8, STEP, 0, 0>(a, s);
}

}  // namespace

bool fused_supported(uint32_t d, uint32_t p) {
    return p >= 1 && p <= 8 && ((d >= 1 && d <= uint32_t(kMaxFusedData)) || d == 20);
}

// The fused kernel covers this (d, p, len): the RS(20,p) build has no ragged-column path.
bool fused_covers(uint32_t d, uint32_t p, uint64_t len) {
    return fused_supported(d, p) && (d != 20 || len % uint64_t(col_width(20)) == 0);
}

// Parts per workgroup for a STEP: every SHA lane holds one chunk (G*(d+p) <= 256) and every
// encoder thread gets at most one 16-byte column per step (G*STEP/16 <= 256): one extra task
// round on one encoder wave would stall the whole workgroup at each step's barrier while its
// SIMD also carries a SHA wave.  RS(10,4), STEP 256: G = 16 (not 18), 4096 parts = 256 groups.
uint32_t parts_per_group(uint32_t t, uint32_t step, uint32_t cw = 16) {
    return std::min(kShaLanes / t, kEncThreads / (step / cw));
}

// 256-byte steps: the ring (≈122 KB for RS(10,4)) admits one workgroup per CU.  Grids larger
// than the CU count run in passes, as the separate SHA kernel does; a second workgroup per CU
// would need <= 128 VGPRs per wave and could gain at most ~16% (one SHA wave already keeps its
// SIMD ~86% busy).
hipError_t launch_encode_hash(const FusedParams& in, bool vec16, hipStream_t s) {
    if (in.n_parts == 0 || in.len == 0) return hipSuccess;
    if (!fused_covers(in.d, in.p, in.len) || !vec16) return hipErrorInvalidValue;
    FusedParams a = in;
    const uint32_t t = a.d + a.p;
    // RS(20,p) batches with more chunks than one SHA wave per SIMD holds: two SHA waves per
    // SIMD (8 + 4 waves per workgroup), one workgroup per CU, 64-byte steps (the ring for 16
    // parts x 28 chunks then fits beside the 40 KB of tables), parts spread over every CU.
    if (a.d == 20 && fused_mode() != 3) {
        const uint32_t cus = uint32_t(device_cus());
        if (uint64_t(a.n_parts) * t > uint64_t(cus) * kShaLanes) {
            const uint32_t cap = std::min(2 * kShaLanes / t, kEncThreads / (64u / 8u));
            const uint32_t want = uint32_t((uint64_t(a.n_parts) + cus - 1) / cus);
            a.parts_per_wg = std::min(cap, want);
            a.enc_prio = fused_prio(1u);
            if (size_t(2) * a.parts_per_wg * t * (64 + 16) + size_t(20) * 256 * 8 <= 160 * 1024) {
                if (fused_enc3() && a.parts_per_wg * t <= 7 * 64 &&
                    a.parts_per_wg * (64u / 8u) <= 128)
                    return fused_be(true) ? launch_p<8, 64, 0, 20, 8, true, true>(a, s)
                                          : launch_p<8, 64, 0, 20, 8, true, false>(a, s);
                return launch_p<8, 64, 0, 20, 8>(a, s);
            }
        }
    }
    // 256-byte steps when the ring and the (generic-size) product tables fit the CU's LDS,
    // else 128-byte steps (wide p = 8 stripes).
    const size_t tabs = size_t(a.d > uint32_t(kMaxFusedData) ? a.d : kMaxFusedData) * 256 *
                        (a.p <= 4 ? 4 : 8);
    a.enc_prio = fused_prio(0u);
    a.parts_per_wg = parts_per_group(t, 256);
    if (a.d <= uint32_t(kMaxFusedData) &&
        size_t(2) * a.parts_per_wg * t * (256 + 16) + tabs <= 160 * 1024)
        return launch_step<256>(a, s);
    a.parts_per_wg = parts_per_group(t, 128, uint32_t(col_width(int(a.d))));
    return launch_step<128>(a, s);
}

}  // namespace cec
