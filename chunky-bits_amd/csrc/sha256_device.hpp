// sha256_device.hpp — SHA-256 (FIPS 180-4) device building blocks for gfx950, shared by the
// SHA-256 kernels and the fused encode+hash kernel.  Costs: see device_common.hpp.
#pragma once

#include "device_common.hpp"

namespace cec {
namespace sha {

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

constexpr uint32_t kH0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                             0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
    return __builtin_amdgcn_perm(x, x, 0x00010203u);
}

// Full-rate single-instruction Ch / Maj (v_bitop3_b32 truth tables over S0=0xF0, S1=0xCC,
// S2=0xAA).
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

__device__ __forceinline__ uint32_t big_s0(uint32_t a) {
    return xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
}
__device__ __forceinline__ uint32_t big_s1(uint32_t e) {
    return xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
}
__device__ __forceinline__ uint32_t small_s0(uint32_t w) {
    return xor3(rotr(w, 7), rotr(w, 18), w >> 3);
}
__device__ __forceinline__ uint32_t small_s1(uint32_t w) {
    return xor3(rotr(w, 17), rotr(w, 19), w >> 10);
}

// W[t] for t in [16, 64) in place over a 16-word ring.
__device__ __forceinline__ uint32_t schedule_next(uint32_t w[16], int i) {
    const uint32_t v = small_s1(w[(i - 2) & 15]) + w[(i - 7) & 15] + small_s0(w[(i - 15) & 15]) +
                       w[i & 15];
    w[i & 15] = v;
    return v;
}

__device__ __forceinline__ void round_step(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                           uint32_t& e, uint32_t& f, uint32_t& g, uint32_t& h,
                                           uint32_t kw) {
    const uint32_t t1 = h + kw + ch(e, f, g) + big_s1(e);
    const uint32_t t2 = big_s0(a) + maj(a, b, c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
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

// Words of padded tail block `blk` (0 or 1) of a message whose last rem (< 64) bytes start at
// tp (FIPS 180-4 §5.1.1: 0x80, zeros, 64-bit big-endian bit length).
__device__ __forceinline__ void tail_words(const uint8_t* tp, uint32_t rem, uint32_t blk,
                                           uint32_t tb, uint64_t bits, uint32_t w[16]) {
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
}

__device__ __forceinline__ uint32_t tail_blocks(uint32_t rem) { return (rem + 9 <= 64) ? 1u : 2u; }

__device__ __forceinline__ void store_digest(uint8_t* out, const uint32_t st[8]) {
    uint4* o = reinterpret_cast<uint4*>(out);
    o[0] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
    o[1] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
}

__device__ __forceinline__ void compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const uint32_t wi = i < 16 ? w[i] : schedule_next(w, i);
        round_step(a, b, c, d, e, f, g, h, wi + kK[i]);
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


}  // namespace sha
}  // namespace cec
