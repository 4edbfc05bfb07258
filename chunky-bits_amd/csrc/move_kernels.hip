// move_kernels.hip — moves chunks between a packed device buffer and a part batch's strided
// positions (device memory on both sides).
//
// The host-staged read pipeline takes the loaded chunks of a batch back to back (the order a
// reader produces them: part by part, chunk index ascending), so the upload is ONE copy-engine
// command per batch instead of one per run of consecutive loaded chunks (~900 per 256-part
// RS(10,4) batch at ~11 us each: 47 vs 57 GB/s, tools/h2d_bench.hip).  This kernel then places
// chunk j of the packed buffer at its batch position ids[j] = k*t + i: an HBM-to-HBM copy of the
// loaded bytes (~1 ms per 2.5 GiB batch), far below the PCIe time it saves.  With packed_ids the
// packed side is itself indexed (chunk j at packed_ids[j]): a retry takes its kept chunks back
// out of the read pipeline's carry pool with one launch (CEC_READ_CARRY), and the carry stash
// kernels below put them in, on the device, with no host round trip.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device_common.hpp"
#include "kernels.hpp"

namespace cec {
namespace {

constexpr uint32_t kMoveThreads = 256;
constexpr uint64_t kMoveSlice = uint64_t(256) << 10;  // bytes of a chunk per work item
constexpr uint32_t kMoveGrid = 2048;

typedef unsigned int mv4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(kMoveThreads) move_chunks_kernel(MoveParams a, bool vec16) {
    const uint64_t slices = (a.len + kMoveSlice - 1) / kMoveSlice;
    const uint64_t items = uint64_t(a.n) * slices;
    for (uint64_t w = blockIdx.x; w < items; w += gridDim.x) {
        const uint64_t j = w / slices;
        const uint64_t off = (w % slices) * kMoveSlice;
        const uint64_t n = (a.len - off < kMoveSlice) ? a.len - off : kMoveSlice;
        const uint32_t id = a.ids[j];
        uint8_t* b = a.batch + uint64_t(id / a.t) * a.part_stride + uint64_t(id % a.t) * a.chunk_stride + off;
        const uint64_t pj = a.packed_ids ? a.packed_ids[j] : j;
        uint8_t* p = a.packed + pj * a.len + off;
        const uint8_t* src = a.to_batch ? p : b;
        uint8_t* dst = a.to_batch ? b : p;
        if (vec16) {
            const mv4* __restrict__ s4 = reinterpret_cast<const mv4*>(src);
            mv4* __restrict__ d4 = reinterpret_cast<mv4*>(dst);
            const uint64_t n16 = n >> 4;
            for (uint64_t x = threadIdx.x; x < n16; x += 2 * kMoveThreads) {
                const mv4 v0 = __builtin_nontemporal_load(&s4[x]);
                mv4 v1 = {0u, 0u, 0u, 0u};
                if (x + kMoveThreads < n16) v1 = __builtin_nontemporal_load(&s4[x + kMoveThreads]);
                __builtin_nontemporal_store(v0, &d4[x]);
                if (x + kMoveThreads < n16) __builtin_nontemporal_store(v1, &d4[x + kMoveThreads]);
            }
        } else {
            for (uint64_t x = threadIdx.x; x < n; x += kMoveThreads) dst[x] = src[x];
        }
    }
}

// A chunk that verified: checked by an earlier pass (CEC_PRESENT_VERIFIED) or loaded and ok.
__device__ inline bool carry_verified(const CarryStashParams& a, uint64_t x) {
    const uint8_t f = a.present[x];
    return f == 0x80 || (f != 0 && a.ok[x] != 0);
}

// One workgroup: each thread takes a contiguous range of parts, counts the ones to keep, and a
// workgroup-wide scan of the counts gives every kept part its rank among them (part order).
constexpr uint32_t kStashAssignThreads = 1024;
__global__ void __launch_bounds__(kStashAssignThreads) carry_assign_kernel(CarryStashParams a) {
    __shared__ uint32_t scan[kStashAssignThreads];
    const uint32_t tid = threadIdx.x;
    const uint32_t per = (a.n_parts + kStashAssignThreads - 1) / kStashAssignThreads;
    const uint32_t k0 = min(a.n_parts, tid * per), k1 = min(a.n_parts, k0 + per);
    auto keep = [&](uint32_t k) {
        uint32_t good = 0;
        for (uint32_t i = 0; i < a.t; ++i) good += carry_verified(a, uint64_t(k) * a.t + i) ? 1u : 0u;
        return good > 0 && good < a.d;
    };
    uint32_t cnt = 0;
    for (uint32_t k = k0; k < k1; ++k) cnt += keep(k) ? 1u : 0u;
    scan[tid] = cnt;
    __syncthreads();
    for (uint32_t off = 1; off < kStashAssignThreads; off <<= 1) {
        const uint32_t v = tid >= off ? scan[tid - off] : 0u;
        __syncthreads();
        scan[tid] += v;
        __syncthreads();
    }
    uint32_t rank = scan[tid] - cnt;
    for (uint32_t k = k0; k < k1; ++k) {
        int32_t e = -1;
        if (keep(k)) {
            if (rank < a.n_reserved) e = int32_t(a.reserved[rank]);
            ++rank;
        }
        a.map[k] = e;
    }
}

// Grid-stride over (part, chunk, slice): a slice of a kept part's verified chunk goes to its entry.
__global__ void __launch_bounds__(kMoveThreads) carry_copy_kernel(CarryStashParams a, bool vec16) {
    const uint64_t slices = (a.len + kMoveSlice - 1) / kMoveSlice;
    const uint64_t items = uint64_t(a.n_parts) * a.t * slices;
    for (uint64_t w = blockIdx.x; w < items; w += gridDim.x) {
        const uint64_t x = w / slices;  // k * t + i
        const uint64_t k = x / a.t, i = x % a.t;
        const int32_t e = a.map[k];
        if (e < 0 || !carry_verified(a, x)) continue;
        const uint64_t off = (w % slices) * kMoveSlice;
        const uint64_t n = (a.len - off < kMoveSlice) ? a.len - off : kMoveSlice;
        const uint8_t* src = a.batch + k * a.part_stride + i * a.chunk_stride + off;
        uint8_t* dst = a.pool + (uint64_t(e) * a.t + i) * a.len + off;
        if (vec16) {
            const mv4* __restrict__ s4 = reinterpret_cast<const mv4*>(src);
            mv4* __restrict__ d4 = reinterpret_cast<mv4*>(dst);
            for (uint64_t y = threadIdx.x; y < (n >> 4); y += kMoveThreads)
                __builtin_nontemporal_store(__builtin_nontemporal_load(&s4[y]), &d4[y]);
        } else {
            for (uint64_t y = threadIdx.x; y < n; y += kMoveThreads) dst[y] = src[y];
        }
    }
}

}  // namespace

hipError_t launch_carry_stash(const CarryStashParams& a, hipStream_t s) {
    if (a.n_parts == 0) return hipSuccess;
    if (!a.batch || !a.pool || !a.present || !a.ok || !a.map || a.t == 0 || a.len == 0 ||
        (a.n_reserved && !a.reserved))
        return hipErrorInvalidValue;
    clear_stale_error();
    hipLaunchKernelGGL(carry_assign_kernel, dim3(1), dim3(kStashAssignThreads), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || a.n_reserved == 0) return e;
    const uint64_t bits = reinterpret_cast<uintptr_t>(a.batch) | reinterpret_cast<uintptr_t>(a.pool) |
                          a.part_stride | a.chunk_stride | a.len;
    const uint64_t items = uint64_t(a.n_parts) * a.t * ((a.len + kMoveSlice - 1) / kMoveSlice);
    const uint32_t grid = uint32_t(std::min<uint64_t>(items, kMoveGrid));
    hipLaunchKernelGGL(carry_copy_kernel, dim3(grid), dim3(kMoveThreads), 0, s, a, (bits & 15) == 0);
    return hipGetLastError();
}

hipError_t launch_move_chunks(const MoveParams& a, hipStream_t s) {
    if (a.n == 0 || a.len == 0) return hipSuccess;
    if (!a.batch || !a.packed || !a.ids || a.t == 0) return hipErrorInvalidValue;
    const uint64_t bits = reinterpret_cast<uintptr_t>(a.batch) |
                          reinterpret_cast<uintptr_t>(a.packed) | a.part_stride | a.chunk_stride |
                          a.len;
    const uint64_t items = uint64_t(a.n) * ((a.len + kMoveSlice - 1) / kMoveSlice);
    const uint32_t grid = uint32_t(std::min<uint64_t>(items, kMoveGrid));
    clear_stale_error();
    hipLaunchKernelGGL(move_chunks_kernel, dim3(grid), dim3(kMoveThreads), 0, s, a,
                       (bits & 15) == 0);
    return hipGetLastError();
}

}  // namespace cec
