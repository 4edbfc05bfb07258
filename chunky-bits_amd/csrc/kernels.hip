// kernels.hip — gfx950 (MI355X, CDNA4) kernels of the erasure-coding + chunk-hashing engine.
//
//  rs_apply_kernel   GF(2^8) matrix x chunk-set multiply.  One kernel serves
//                    ReedSolomon::encode_sep (rows = parity rows of M, inputs = the d data chunks)
//                    and reconstruct / reconstruct_data (rows = decode rows, inputs = the first d
//                    present chunks), for thousands of parts per launch.  HBM-bound:
//                    algorithmic bytes per part = (d + n_out) * len.
//  sha256_kernel     FIPS 180-4 SHA-256, one lane per chunk (Sha256Hash::from_buf,
//                    src/file/hash/sha256.rs:20-26).  VALU-bound: a chunk is a serial chain of
//                    64-byte compressions, so parallelism = number of chunks.
//  fill_kernel       counter-based synthetic bytes for benchmarks/tests.
//
// GF multiply: no GF instruction exists, so a product c*x of four packed bytes is three
// v_perm_b32 byte-table lookups (x split into bits [2:0], [5:3], [7:6]; see gf256.hpp) combined
// with one v_bitop3_b32 (xor3).  The selectors of a data word are shared by every output row.
// Coefficient tables are wave-uniform and come in through scalar loads (s_load), so a row costs
// 3 v_perm + ~1.5 xor per data dword, with no LDS traffic and no bank conflicts.
#include "kernels.hpp"
#include "gf256.hpp"

namespace cec {
namespace {

constexpr int kApplyThreads = 256;
constexpr int kApplyIters = 4;  // 16-byte columns per thread per block
constexpr uint64_t kApplyTile = uint64_t(kApplyThreads) * 16u * kApplyIters;  // 16 KiB

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// v_perm_b32: byte lane i of the result = byte sel[i] (0..7) of the 8-byte value {hi:lo}.
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

struct Sel {
    uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel selectors(uint32_t x) {
    return {x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// c (x) x for 4 packed bytes, c given by its 5 packed table words.
__device__ __forceinline__ uint32_t gmul(const Sel& s, uint32_t t0, uint32_t t1, uint32_t t2,
                                         uint32_t t3, uint32_t t4) {
    return xor3(perm(t1, t0, s.s0), perm(t3, t2, s.s1), perm(0u, t4, s.s2));
}

__device__ __forceinline__ uint4 load_partial(const uint8_t* p, uint64_t n) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (uint64_t(k) < n) w[k >> 2] |= uint32_t(p[k]) << (8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_partial(uint8_t* p, const uint32_t w[4], uint64_t n) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (uint64_t(k) < n) p[k] = uint8_t(w[k >> 2] >> (8 * (k & 3)));
}

// Wave-uniform metadata (pattern records, part maps) is read through the constant address space
// so it lands in SGPRs via s_load instead of per-lane vector loads.
typedef __attribute__((address_space(4))) const uint32_t cu32;

__device__ __forceinline__ cu32* as_const(const uint32_t* p) {
    return (cu32*)(p);
}

// One 16-byte column (x .. x+16) of a part: acc[r] = XOR_j coef[r][j] (x) in_j[x..x+16).
// FULL: every lane of the block has 16 valid bytes and the layout is 16-byte aligned.
// tab points at row0's table of input 0; input j's RG tables start at tab + j*tab_stride.
template <int RG, bool FULL>
__device__ __forceinline__ void apply_column(uint8_t* pbase, uint64_t cs, uint64_t x,
                                             uint64_t rem, uint32_t d, uint32_t tab_stride,
                                             cu32* in_idx, cu32* out_idx, cu32* tab) {
    uint32_t acc[RG][4];
#pragma unroll
    for (int r = 0; r < RG; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    const uint64_t n = rem < 16 ? rem : 16;

#pragma unroll 1
    for (uint32_t j0 = 0; j0 < d; j0 += 4) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            v[u] = make_uint4(0u, 0u, 0u, 0u);
            if (j0 + u < d) {
                const uint8_t* src = pbase + uint64_t(in_idx[j0 + u]) * cs + x;
                if (FULL) v[u] = *reinterpret_cast<const uint4*>(src);
                else v[u] = load_partial(src, n);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (j0 + u < d) {
                const Sel s0 = selectors(v[u].x), s1 = selectors(v[u].y),
                          s2 = selectors(v[u].z), s3 = selectors(v[u].w);
cu32* tj = tab + size_t(j0 + u) * tab_stride;
#pragma unroll
                for (int r = 0; r < RG; ++r) {
                    cu32* t = tj + r * kTabWords;
                    const uint32_t t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3], t4 = t[4];
                    acc[r][0] ^= gmul(s0, t0, t1, t2, t3, t4);
                    acc[r][1] ^= gmul(s1, t0, t1, t2, t3, t4);
                    acc[r][2] ^= gmul(s2, t0, t1, t2, t3, t4);
                    acc[r][3] ^= gmul(s3, t0, t1, t2, t3, t4);
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RG; ++r) {
        uint8_t* dst = pbase + uint64_t(out_idx[r]) * cs + x;
        if (FULL)
            *reinterpret_cast<uint4*>(dst) = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
        else store_partial(dst, acc[r], n);
    }
}

// grid.x = n_parts * tiles_per_part (one 16 KiB column tile of one part per block),
// grid.y = row groups of exactly RG output rows starting at row_base.
template <int RG, bool VEC>
__global__ __launch_bounds__(kApplyThreads) void rs_apply_kernel(ApplyParams a,
                                                                 uint32_t tiles_per_part,
                                                                 uint32_t row_base) {
    const uint32_t lp = blockIdx.x / tiles_per_part;
    const uint32_t tile = blockIdx.x - lp * tiles_per_part;
    const uint32_t part = a.part_ids ? as_const(a.part_ids)[lp] : lp;
    cu32* pat = as_const(a.pat) + (a.part_pat ? as_const(a.part_pat)[lp] : 0u);
    const uint32_t d = a.d;
    const uint32_t n_out = a.n_rows;
    const uint32_t row0 = row_base + blockIdx.y * RG;
    cu32* in_idx = pat + 1;
    cu32* out_idx = pat + 1 + d + row0;
    cu32* tab = pat + 1 + d + n_out + size_t(row0) * kTabWords;
    const uint32_t tab_stride = n_out * kTabWords;
    uint8_t* pbase = a.base + uint64_t(part) * a.part_stride;
    const uint64_t len = a.len;
    const uint64_t cs = a.chunk_stride;
    constexpr uint64_t kStep = uint64_t(kApplyThreads) * 16u;

#pragma unroll 1
    for (int it = 0; it < kApplyIters; ++it) {
        const uint64_t xb = (uint64_t(tile) * kApplyIters + it) * kStep;  // block-uniform
        if (xb >= len) break;
        const uint64_t x = xb + uint64_t(threadIdx.x) * 16u;
        if (VEC && xb + kStep <= len) {
            apply_column<RG, true>(pbase, cs, x, len - x, d, tab_stride, in_idx, out_idx, tab);
        } else if (x < len) {
            apply_column<RG, false>(pbase, cs, x, len - x, d, tab_stride, in_idx, out_idx, tab);
        }
    }
}

// ------------------------------------------------------------------------------------------
// SHA-256
// ------------------------------------------------------------------------------------------

constexpr uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
    return __builtin_amdgcn_perm(x, x, 0x00010203u);
}

// One 64-byte compression; w[] holds the 16 big-endian message words (clobbered).
__device__ __forceinline__ void sha256_compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + kK[i] + wi;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = (a & b) | (c & (a | b));
        const uint32_t t2 = S0 + mj;
        h = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
    st[5] += f;
    st[6] += g;
    st[7] += h;
}

template <bool VEC>
__device__ __forceinline__ void load_block(const uint8_t* p, uint4 q[4]) {
    if (VEC) {
        const uint4* v = reinterpret_cast<const uint4*>(p);
        q[0] = v[0];
        q[1] = v[1];
        q[2] = v[2];
        q[3] = v[3];
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = load_partial(p + 16 * i, 16);
    }
}

__device__ __forceinline__ void block_words(const uint4 q[4], uint32_t w[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w[4 * i + 0] = bswap32(q[i].x);
        w[4 * i + 1] = bswap32(q[i].y);
        w[4 * i + 2] = bswap32(q[i].z);
        w[4 * i + 3] = bswap32(q[i].w);
    }
}

__device__ __forceinline__ void sha256_chunk(const uint8_t* p, uint64_t len, uint32_t st[8],
                                             bool vec) {
    st[0] = 0x6a09e667u;
    st[1] = 0xbb67ae85u;
    st[2] = 0x3c6ef372u;
    st[3] = 0xa54ff53au;
    st[4] = 0x510e527fu;
    st[5] = 0x9b05688cu;
    st[6] = 0x1f83d9abu;
    st[7] = 0x5be0cd19u;
    const uint64_t nfull = len >> 6;
    uint32_t w[16];
    if (nfull) {
        uint4 q[4];
        if (vec) load_block<true>(p, q);
        else load_block<false>(p, q);
#pragma unroll 1
        for (uint64_t b = 0; b < nfull; ++b) {
            block_words(q, w);
            if (b + 1 < nfull) {
                if (vec) load_block<true>(p + 64 * (b + 1), q);
                else load_block<false>(p + 64 * (b + 1), q);
            }
            sha256_compress(st, w);
        }
    }
    const uint8_t* tp = p + 64 * nfull;
    const uint32_t rem = uint32_t(len - 64 * nfull);
    const uint32_t tb = (rem + 9 <= 64) ? 1u : 2u;
    const uint64_t bits = len * 8;
#pragma unroll 1
    for (uint32_t blk = 0; blk < tb; ++blk) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t word = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t pos = blk * 64 + uint32_t(i * 4 + k);
                const uint32_t byte = pos < rem ? uint32_t(tp[pos]) : (pos == rem ? 0x80u : 0u);
                word = (word << 8) | byte;
            }
            w[i] = word;
        }
        if (blk == tb - 1) {
            w[14] = uint32_t(bits >> 32);
            w[15] = uint32_t(bits);
        }
        sha256_compress(st, w);
    }
}

template <bool VEC>
__global__ __launch_bounds__(64) void sha256_kernel(ShaParams a) {
    const uint32_t item = blockIdx.x * 64u + threadIdx.x;
    const uint32_t total = a.n_parts * a.n_chunks;
    if (item >= total) return;
    const uint8_t* p;
    uint64_t len;
    if (a.ptrs) {
        p = reinterpret_cast<const uint8_t*>(a.ptrs[item]);
        len = a.lens[item];
    } else {
        const uint32_t k = item / a.n_chunks;
        const uint32_t c = item - k * a.n_chunks;
        p = a.base + uint64_t(k) * a.part_stride + uint64_t(a.first_chunk + c) * a.chunk_stride;
        len = a.len;
    }
    uint32_t st[8];
    sha256_chunk(p, len, st, VEC);
    uint4* out = reinterpret_cast<uint4*>(a.digests + uint64_t(item) * 32u);
    out[0] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
    out[1] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
}

// ------------------------------------------------------------------------------------------
// Synthetic data
// ------------------------------------------------------------------------------------------

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

__host__ __device__ __forceinline__ uint64_t synth_key(uint64_t seed, uint64_t part,
                                                       uint64_t chunk) {
    return mix64(seed ^ mix64(part * 0x100000001B3ull + chunk + 0x9E3779B97F4A7C15ull));
}

__host__ __device__ __forceinline__ uint64_t synth_word(uint64_t key, uint64_t word) {
    return mix64(key + word * 0x9E3779B97F4A7C15ull);
}

__global__ __launch_bounds__(256) void fill_kernel(FillParams a, bool aligned8) {
    const uint64_t words = (a.len + 7) / 8;
    const uint64_t n_inst = uint64_t(a.n_parts) * a.n_chunks;
    for (uint64_t inst = blockIdx.y; inst < n_inst; inst += gridDim.y) {
        const uint64_t k = inst / a.n_chunks;
        const uint64_t c = inst - k * a.n_chunks;
        const uint64_t key = synth_key(a.seed, k, c);
        uint8_t* dst = a.base + k * a.part_stride + c * a.chunk_stride;
        for (uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w < words;
             w += uint64_t(gridDim.x) * blockDim.x) {
            const uint64_t v = synth_word(key, w);
            const uint64_t off = w * 8;
            if (aligned8 && off + 8 <= a.len) {
                *reinterpret_cast<uint64_t*>(dst + off) = v;
            } else {
                for (int b = 0; b < 8; ++b)
                    if (off + b < a.len) dst[off + b] = uint8_t(v >> (8 * b));
            }
        }
    }
}

template <int RG>
hipError_t launch_rg(const ApplyParams& a, uint32_t row_base, uint32_t groups, bool vec16,
                     hipStream_t s) {
    const uint32_t tiles = uint32_t((a.len + kApplyTile - 1) / kApplyTile);
    dim3 grid(a.n_parts * tiles, groups);
    if (vec16)
        hipLaunchKernelGGL((rs_apply_kernel<RG, true>), grid, dim3(kApplyThreads), 0, s, a, tiles,
                           row_base);
    else
        hipLaunchKernelGGL((rs_apply_kernel<RG, false>), grid, dim3(kApplyThreads), 0, s, a,
                           tiles, row_base);
    return hipGetLastError();
}

hipError_t launch_rows(const ApplyParams& a, uint32_t rg, uint32_t row_base, uint32_t groups,
                       bool vec16, hipStream_t s) {
    switch (rg) {
        case 1: return launch_rg<1>(a, row_base, groups, vec16, s);
        case 2: return launch_rg<2>(a, row_base, groups, vec16, s);
        case 3: return launch_rg<3>(a, row_base, groups, vec16, s);
        case 4: return launch_rg<4>(a, row_base, groups, vec16, s);
        case 5: return launch_rg<5>(a, row_base, groups, vec16, s);
        case 6: return launch_rg<6>(a, row_base, groups, vec16, s);
        case 7: return launch_rg<7>(a, row_base, groups, vec16, s);
        default: return launch_rg<8>(a, row_base, groups, vec16, s);
    }
}

}  // namespace

// Rows are processed in groups of kMaxRows (8) plus one remainder group, so every kernel
// instance handles exactly RG rows (no per-row predicate in the inner loop).
hipError_t launch_rs_apply(const ApplyParams& a, bool vec16, hipStream_t s) {
    if (a.n_parts == 0 || a.n_rows == 0 || a.len == 0) return hipSuccess;
    constexpr uint32_t kMaxRows = 8;
    const uint32_t full = a.n_rows / kMaxRows, rem = a.n_rows % kMaxRows;
    if (full) {
        hipError_t e = launch_rows(a, kMaxRows, 0, full, vec16, s);
        if (e != hipSuccess) return e;
    }
    if (rem) return launch_rows(a, rem, full * kMaxRows, 1, vec16, s);
    return hipSuccess;
}

hipError_t launch_sha256(const ShaParams& a, bool vec16, hipStream_t s) {
    const uint64_t total = uint64_t(a.n_parts) * a.n_chunks;
    if (total == 0) return hipSuccess;
    dim3 grid(uint32_t((total + 63) / 64));
    if (vec16) hipLaunchKernelGGL((sha256_kernel<true>), grid, dim3(64), 0, s, a);
    else hipLaunchKernelGGL((sha256_kernel<false>), grid, dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_fill(const FillParams& a, hipStream_t s) {
    const uint64_t n_inst = uint64_t(a.n_parts) * a.n_chunks;
    if (n_inst == 0 || a.len == 0) return hipSuccess;
    const uint64_t words = (a.len + 7) / 8;
    uint32_t gx = uint32_t(std::min<uint64_t>((words + 255) / 256, 64));
    uint32_t gy = uint32_t(std::min<uint64_t>(n_inst, 65535));
    const bool aligned8 = (reinterpret_cast<uintptr_t>(a.base) % 8 == 0) &&
                          (a.part_stride % 8 == 0) && (a.chunk_stride % 8 == 0);
    hipLaunchKernelGGL(fill_kernel, dim3(gx, gy), dim3(256), 0, s, a, aligned8);
    return hipGetLastError();
}

uint8_t synth_byte(uint64_t seed, uint64_t part, uint64_t chunk, uint64_t offset) {
    const uint64_t v = synth_word(synth_key(seed, part, chunk), offset / 8);
    return uint8_t(v >> (8 * (offset % 8)));
}

}  // namespace cec
