// move_kernels.hip — moves chunks between a packed device buffer and a part batch's strided
// positions (device memory on both sides).
//
// The host-staged read pipeline takes the loaded chunks of a batch back to back (the order a
// reader produces them: part by part, chunk index ascending), so the upload is ONE copy-engine
// command per batch instead of one per run of consecutive loaded chunks (~900 per 256-part
// RS(10,4) batch at ~11 us each: 47 vs 57 GB/s, tools/h2d_bench.hip).  This kernel then places
// chunk j of the packed buffer at its batch position ids[j] = k*t + i: an HBM-to-HBM copy of the
// loaded bytes (~1 ms per 2.5 GiB batch), far below the PCIe time it saves.  With packed_ids the
// packed side is itself indexed (chunk j at packed_ids[j]): the read pipeline's carry pool moves
// a batch's kept chunks in and out with one launch each (CEC_READ_CARRY).
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

}  // namespace

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
