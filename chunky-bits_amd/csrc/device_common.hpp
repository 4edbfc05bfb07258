// device_common.hpp — small gfx950 device helpers shared by the kernel sources.
//
// Instruction costs measured on MI355X (tools/ubench_valu.hip): with two
// waves per SIMD, v_add/v_xor/v_and/shifts and v_bitop3_b32 issue at full rate (~2.4 SIMD
// cycles per wave64 instruction) while v_alignbit_b32, v_add3_u32, v_perm_b32 and v_bfi_b32 are
// half rate (~4.5); a lone wave issues at best every ~5 cycles and a dependent chain costs
// ~10-11 cycles per step.  The helpers below pick the full-rate form where one exists.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace cec {

// Drop a status an earlier, non-fatal HIP call left on this host thread (an event query that
// was not ready, a pointer query on pageable memory), so the hipGetLastError() after the next
// launch reports that launch only.
inline void clear_stale_error() { (void)hipGetLastError(); }

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// v_perm_b32: byte lane i of the result = byte sel[i] (0..7) of the 8-byte value {hi:lo}.
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
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

// Wave-uniform metadata (pattern records, part maps) is read through the constant address
// space so it lands in SGPRs via s_load instead of per-lane vector loads.
typedef __attribute__((address_space(4))) const uint32_t cu32;

__device__ __forceinline__ cu32* as_const(const uint32_t* p) { return (cu32*)(p); }

// 16-byte load through the global address space: global_load_dwordx4 counts in vmcnt only (a
// flat load also counts in lgkmcnt, so an LDS-only wait would drain it too).
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u32 gv4u32;
__device__ __forceinline__ uint4 gload16(const uint8_t* p) {
    const v4u32 t = *(gv4u32*)(reinterpret_cast<uintptr_t>(p));
    return make_uint4(t.x, t.y, t.z, t.w);
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS ops (lgkmcnt) but leaves
// global loads in flight across it (__syncthreads() would also wait for vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

}  // namespace cec
