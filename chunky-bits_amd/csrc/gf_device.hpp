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

// Product tables (the fused encoder and rs_apply's LDS path): for one input and byte value x, an
// entry of E bytes packs c[r]*x for every output row r (row r in byte r).  A data byte then costs
// one ds_read plus half an xor3 for all rows, instead of three half-rate v_perm per row.

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

}  // namespace gf
}  // namespace cec
