// gf_device.hpp — GF(2^8) multiply-by-constant for gfx950 via v_perm_b32 byte tables (layout
// of the 5 packed table words: gf256.hpp pack_coef).  Shared by rs_kernels.hip and the fused
// encode+hash kernel.
#pragma once

#include "device_common.hpp"

namespace cec {
namespace gf {

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

}  // namespace gf
}  // namespace cec
