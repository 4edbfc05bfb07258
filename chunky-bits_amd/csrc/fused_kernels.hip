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

#include "device_common.hpp"
#include "gf256.hpp"
#include "gf_device.hpp"
#include "kernels.hpp"
#include "sha256_device.hpp"

namespace cec {
namespace {

using namespace gf;
using namespace sha;

constexpr int kFusedThreads = 512;
constexpr uint32_t kShaLanes = 256;
constexpr uint32_t kEncThreads = 256;
constexpr int kMaxFusedData = 16;  // d > 16: separate encode + SHA kernels

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

// Byte k of w, scaled to a table entry offset of 1 << SHIFT bytes (k constant after unroll).
template <int SHIFT>
__device__ __forceinline__ uint32_t entry_off(uint32_t w, int k) {
    constexpr uint32_t mask = 0xFFu << SHIFT;
    const int sh = 8 * k - SHIFT;
    return sh >= 0 ? ((w >> sh) & mask) : ((w << -sh) & mask);
}

// LDS hand-over barrier that does not drain vector memory: the encoders keep next step's
// global loads in flight across it (a __syncthreads() would wait for them: vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// PMAX: parity rows (exact when a.p == PMAX; rows r >= a.p skipped by uniform guards).
// Up to kMaxFusedData data inputs are held in registers per encoder thread (next step's
// prefetch).  Aligned (16-byte) layouts only; others use the separate kernels.
template <int PMAX, int STEP>
__global__ __launch_bounds__(kFusedThreads) void encode_hash_kernel(FusedParams a) {
    constexpr bool VEC = true;
    constexpr int DMAX = kMaxFusedData;
    extern __shared__ __attribute__((aligned(16))) uint8_t ring[];
    constexpr uint32_t kRow = STEP + 16;  // 16-byte pad: conflict-free 16 B per lane accesses
    constexpr uint32_t kCols = STEP / 16;
    const uint32_t d = a.d, P = a.p, t = a.d + a.p;
    const uint32_t G = a.parts_per_wg;
    const uint32_t rows = G * t;
    const uint32_t part0 = blockIdx.x * G;
    const uint32_t g_here = min(G, a.n_parts - part0);
    const uint64_t L = a.len;
    const uint64_t cs = a.chunk_stride;
    const uint32_t n_steps = uint32_t((L + STEP - 1) / STEP);

    if (threadIdx.x >= kShaLanes) {
        // ------------------------------ encoders ------------------------------
        // Each encoder thread owns one 16-byte column (g, col) of every step (launch_encode_hash
        // guarantees G*kCols <= kEncThreads).  Per step: multiply the d inputs already in
        // registers, write data + parity into the LDS slot, store parity to HBM, then issue the
        // next step's d loads (all in flight at once) before the barrier.
        cu32* pat = as_const(a.pat);
        cu32* tab = pat + 1 + d + P;  // input j, row r at (j*P + r) * 5
        const uint32_t et = threadIdx.x - kShaLanes;
        const bool has_task = et < g_here * kCols;
        const uint32_t g = et / kCols, col = et - g * kCols;
        uint8_t* pb = a.base + uint64_t(part0 + g) * a.part_stride;
        uint4 v[DMAX];
        auto load_step = [&](uint32_t s) {
            const uint64_t x = uint64_t(s) * STEP + col * 16u;
            if (!has_task || x >= L) return;
            const uint64_t n = (L - x) < 16 ? (L - x) : 16;
            const uint8_t* src = pb + x;  // per-lane pointer walked by chunk_stride: no
                                          // per-input 64-bit base held in SGPRs
#pragma unroll
            for (int j = 0; j < DMAX; ++j) {
                if (uint32_t(j) < d) {
                    v[j] = (VEC && n == 16) ? *reinterpret_cast<const uint4*>(src)
                                            : load_partial(src, n);
                    src += cs;
                }
            }
        };
        // Product tables in LDS behind the ring: for input j and byte value x, one entry packs
        // c[r][j] * x for every parity row r (row r in byte r; 4 B per entry for p <= 4, 8 B for
        // p <= 8).  A data byte then costs one ds_read + one xor for all rows, instead of three
        // half-rate v_perm per row: the GF multiply moves off the VALU the SHA waves saturate.
        constexpr int kEntry = PMAX <= 4 ? 4 : 8;
        uint8_t* tabs = ring + size_t(2) * rows * kRow;
        {
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
            const uint64_t x = uint64_t(s) * STEP + col * 16u;
            if (!has_task || x >= L) return;
            const uint64_t n = (L - x) < 16 ? (L - x) : 16;
            uint8_t* lrow = ring + (size_t(slot) * rows + size_t(g) * t) * kRow + col * 16u;
            uint32_t acc_lo[16], acc_hi[16];
#pragma unroll
            for (int b = 0; b < 16; ++b) acc_lo[b] = acc_hi[b] = 0u;
#pragma unroll
            for (int j = 0; j < DMAX; ++j) {
                if (uint32_t(j) < d) {
                    *reinterpret_cast<uint4*>(lrow + size_t(j) * kRow) = v[j];
                    const uint8_t* tj = tabs + size_t(j) * 256 * kEntry;
                    const uint32_t wq[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            if (kEntry == 4) {
                                acc_lo[4 * q + k] ^= *reinterpret_cast<const uint32_t*>(
                                    tj + entry_off<2>(wq[q], k));
                            } else {
                                const uint2 e = *reinterpret_cast<const uint2*>(
                                    tj + entry_off<3>(wq[q], k));
                                acc_lo[4 * q + k] ^= e.x;
                                acc_hi[4 * q + k] ^= e.y;
                            }
                        }
                    }
                }
            }
            // rows 0..3 from acc_lo, rows 4..7 from acc_hi: out[r][q] = word q of parity row r
            uint32_t out[8][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
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
                const uint4 o = make_uint4(out[r][0], out[r][1], out[r][2], out[r][3]);
                *reinterpret_cast<uint4*>(lrow + size_t(d + r) * kRow) = o;
                uint8_t* dst = pb + uint64_t(d + r) * cs + x;
                if (VEC && n == 16) {
                    *reinterpret_cast<uint4*>(dst) = o;
                } else {
                    const uint32_t o4[4] = {o.x, o.y, o.z, o.w};
                    store_partial(dst, o4, n);
                }
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
                    block_words(qq, w);
                    compress(st, w);
                }
                if (s + 1 == n_steps) {
                    const uint32_t rem = uint32_t(L - 64 * nfull);
                    const uint32_t tb = tail_blocks(rem);
                    const uint8_t* tp = row + (64 * nfull - uint64_t(s) * STEP);
#pragma unroll 1
                    for (uint32_t blk = 0; blk < tb; ++blk) {
                        tail_words(tp, rem, blk, tb, L * 8, w);
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

template <int PMAX, int STEP>
hipError_t launch_p(const FusedParams& a, hipStream_t s) {
    const size_t lds = size_t(2) * a.parts_per_wg * (a.d + a.p) * (STEP + 16) +
                       size_t(a.d) * 256 * (PMAX <= 4 ? 4 : 8);
    static const bool attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&encode_hash_kernel<PMAX, STEP>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (!attr) return hipErrorInvalidValue;
    const uint32_t grid = (a.n_parts + a.parts_per_wg - 1) / a.parts_per_wg;
    hipLaunchKernelGGL((encode_hash_kernel<PMAX, STEP>), dim3(grid), dim3(kFusedThreads), lds, s,
                       a);
    return hipGetLastError();
}

template <int STEP>
hipError_t launch_step(const FusedParams& a, hipStream_t s) {
    return a.p == 4 ? launch_p<4, STEP>(a, s) : launch_p<8, STEP>(a, s);
}

}  // namespace

bool fused_supported(uint32_t d, uint32_t p) {
    return p >= 1 && p <= 8 && d >= 1 && d <= uint32_t(kMaxFusedData) && d + p <= kShaLanes;
}

// Parts per workgroup for a STEP: every SHA lane holds one chunk (G*(d+p) <= 256) and every
// encoder thread gets at most one 16-byte column per step (G*STEP/16 <= 256): one extra task
// round on one encoder wave would stall the whole workgroup at each step's barrier while its
// SIMD also carries a SHA wave.  RS(10,4), STEP 256: G = 16 (not 18), 4096 parts = 256 groups.
uint32_t parts_per_group(uint32_t t, uint32_t step) {
    return std::min(kShaLanes / t, kEncThreads / (step / 16));
}

// 256-byte steps: the ring (≈122 KB for RS(10,4)) admits one workgroup per CU.  Grids larger
// than the CU count run in passes, as the separate SHA kernel does; a second workgroup per CU
// would need <= 128 VGPRs per wave and could gain at most ~16% (one SHA wave already keeps its
// SIMD ~86% busy).
hipError_t launch_encode_hash(const FusedParams& in, bool vec16, hipStream_t s) {
    if (in.n_parts == 0 || in.len == 0) return hipSuccess;
    if (!fused_supported(in.d, in.p) || !vec16) return hipErrorInvalidValue;
    FusedParams a = in;
    a.parts_per_wg = parts_per_group(a.d + a.p, 256);
    return launch_step<256>(a, s);
}

}  // namespace cec
