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
// encoders fill slot (s+1)%2; one __syncthreads per step hands the slots over.  The ring
// (≈139 KB for STEP=256) also keeps a second workgroup off the CU.  The encoder waves share
// each SIMD with a SHA wave and use the issue slots the SHA wave leaves (it runs ~4.2 cycles per
// VALU op, below the SIMD's rate).
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

template <int P, bool VEC, int STEP>
__global__ __launch_bounds__(kFusedThreads) void encode_hash_kernel(FusedParams a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t ring[];
    constexpr uint32_t kRow = STEP + 16;  // 16-byte pad: conflict-free 16 B per lane accesses
    constexpr uint32_t kCols = STEP / 16;
    const uint32_t d = a.d, t = a.d + P;
    const uint32_t G = a.parts_per_wg;
    const uint32_t rows = G * t;
    const uint32_t part0 = blockIdx.x * G;
    const uint32_t g_here = min(G, a.n_parts - part0);
    const uint64_t L = a.len;
    const uint64_t cs = a.chunk_stride;
    const uint32_t n_steps = uint32_t((L + STEP - 1) / STEP);

    if (threadIdx.x >= kShaLanes) {
        // ------------------------------ encoders ------------------------------
        cu32* pat = as_const(a.pat);
        cu32* tab = pat + 1 + d + P;  // input j, row r at (j*P + r) * 5
        const uint32_t et = threadIdx.x - kShaLanes;
        const uint32_t tasks = g_here * kCols;
        auto fill = [&](uint32_t s, uint32_t slot) {
            uint8_t* sl = ring + size_t(slot) * rows * kRow;
#pragma unroll 1
            for (uint32_t task = et; task < tasks; task += kEncThreads) {
                const uint32_t g = task / kCols, col = task - g * kCols;
                const uint64_t x = uint64_t(s) * STEP + col * 16u;
                if (x >= L) continue;
                const uint64_t n = (L - x) < 16 ? (L - x) : 16;
                const bool full = VEC && n == 16;
                uint8_t* pb = a.base + uint64_t(part0 + g) * a.part_stride;
                uint8_t* lrow = sl + size_t(g) * t * kRow + col * 16u;
                uint32_t acc[P][4];
#pragma unroll
                for (int r = 0; r < P; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
#pragma unroll 2
                for (uint32_t j = 0; j < d; ++j) {
                    const uint8_t* src = pb + uint64_t(j) * cs + x;
                    const uint4 v = full ? *reinterpret_cast<const uint4*>(src)
                                         : load_partial(src, n);
                    *reinterpret_cast<uint4*>(lrow + size_t(j) * kRow) = v;
                    const Sel s0 = selectors(v.x), s1 = selectors(v.y), s2 = selectors(v.z),
                              s3 = selectors(v.w);
                    cu32* tj = tab + size_t(j) * P * kTabWords;
#pragma unroll
                    for (int r = 0; r < P; ++r) {
                        cu32* c = tj + r * kTabWords;
                        const uint32_t t0 = c[0], t1 = c[1], t2 = c[2], t3 = c[3], t4 = c[4];
                        acc[r][0] ^= gmul(s0, t0, t1, t2, t3, t4);
                        acc[r][1] ^= gmul(s1, t0, t1, t2, t3, t4);
                        acc[r][2] ^= gmul(s2, t0, t1, t2, t3, t4);
                        acc[r][3] ^= gmul(s3, t0, t1, t2, t3, t4);
                    }
                }
#pragma unroll
                for (int r = 0; r < P; ++r) {
                    const uint4 o = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
                    *reinterpret_cast<uint4*>(lrow + size_t(d + r) * kRow) = o;
                    uint8_t* dst = pb + uint64_t(d + r) * cs + x;
                    if (full) *reinterpret_cast<uint4*>(dst) = o;
                    else store_partial(dst, acc[r], n);
                }
            }
        };
        fill(0, 0);
        __syncthreads();
#pragma unroll 1
        for (uint32_t s = 0; s < n_steps; ++s) {
            if (s + 1 < n_steps) fill(s + 1, (s + 1) & 1u);
            __syncthreads();
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

template <int P, bool VEC, int STEP>
hipError_t launch_p(const FusedParams& a, hipStream_t s) {
    const size_t lds = size_t(2) * a.parts_per_wg * (a.d + P) * (STEP + 16);
    static const bool attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&encode_hash_kernel<P, VEC, STEP>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    if (!attr) return hipErrorInvalidValue;
    const uint32_t grid = (a.n_parts + a.parts_per_wg - 1) / a.parts_per_wg;
    hipLaunchKernelGGL((encode_hash_kernel<P, VEC, STEP>), dim3(grid), dim3(kFusedThreads), lds,
                       s, a);
    return hipGetLastError();
}

template <bool VEC, int STEP>
hipError_t launch_step(const FusedParams& a, uint32_t p, hipStream_t s) {
    switch (p) {
        case 1: return launch_p<1, VEC, STEP>(a, s);
        case 2: return launch_p<2, VEC, STEP>(a, s);
        case 3: return launch_p<3, VEC, STEP>(a, s);
        case 4: return launch_p<4, VEC, STEP>(a, s);
        case 5: return launch_p<5, VEC, STEP>(a, s);
        case 6: return launch_p<6, VEC, STEP>(a, s);
        case 7: return launch_p<7, VEC, STEP>(a, s);
        case 8: return launch_p<8, VEC, STEP>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

bool fused_supported(uint32_t d, uint32_t p) { return p >= 1 && p <= 8 && d + p <= kShaLanes; }

// Parts per workgroup for a STEP: every SHA lane holds one chunk (G*(d+p) <= 256) and every
// encoder thread gets at most one 16-byte column per step (G*STEP/16 <= 256): one extra task
// round on one encoder wave would stall the whole workgroup at each step's barrier while its
// SIMD also carries a SHA wave.  RS(10,4), STEP 256: G = 16 (not 18), 4096 parts = 256 groups.
uint32_t parts_per_group(uint32_t t, uint32_t step) {
    return std::min(kShaLanes / t, kEncThreads / (step / 16));
}

// STEP: 256-byte steps (ring ≈ 139 KB: one workgroup per CU) when the grid fits the CUs in one
// pass; 128-byte steps (ring < 80 KB: two workgroups per CU, two SHA waves per SIMD) when it
// would otherwise take two passes.
hipError_t launch_encode_hash(const FusedParams& in, bool vec16, hipStream_t s) {
    if (in.n_parts == 0 || in.len == 0) return hipSuccess;
    if (!fused_supported(in.d, in.p)) return hipErrorInvalidValue;
    FusedParams a = in;
    const uint32_t t = a.d + a.p;
    int cus = 256;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    a.parts_per_wg = parts_per_group(t, 256);
    const uint32_t grid = (a.n_parts + a.parts_per_wg - 1) / a.parts_per_wg;
    const bool two_per_cu = grid > uint32_t(cus);
    if (two_per_cu) a.parts_per_wg = parts_per_group(t, 128);
    if (vec16)
        return two_per_cu ? launch_step<true, 128>(a, a.p, s) : launch_step<true, 256>(a, a.p, s);
    return two_per_cu ? launch_step<false, 128>(a, a.p, s) : launch_step<false, 256>(a, a.p, s);
}

}  // namespace cec
