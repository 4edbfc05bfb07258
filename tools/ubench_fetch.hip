// Calibration (dev tool): FETCH_SIZE vs known bytes for the read patterns of the engine.
//   coalesced: lane i reads 16 B at base + 16*i + k*1024 (rs_apply_kernel's pattern)
//   per_lane : lane = one 1 MiB stream, reads 64 B blocks in order (sha256_lane_kernel's pattern)
// Each kernel reads exactly BYTES bytes once; run under rocprofv3 --pmc FETCH_SIZE and compare.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t kStream = 1 << 20;

__global__ void coalesced(const uint4* __restrict__ p, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16;
         i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void per_lane(const uint8_t* __restrict__ p, size_t n_streams,
                                                uint32_t* out) {
    const size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (s >= n_streams) return;
    const uint4* q = reinterpret_cast<const uint4*>(p + s * kStream);
    uint32_t acc = 0;
    for (size_t b = 0; b < kStream / 64; ++b) {
        uint4 v0 = q[4 * b], v1 = q[4 * b + 1], v2 = q[4 * b + 2], v3 = q[4 * b + 3];
        acc ^= v0.x ^ v1.y ^ v2.z ^ v3.w ^ v0.w ^ v1.x ^ v2.y ^ v3.z;
        acc = (acc << 1) | (acc >> 31);
    }
    out[s] = acc;
}

// RS(20,p) fused build's encoder pattern (fused_kernels.hip, C4 shape): 16 parts per
// workgroup, 8 lanes per part; per 64-byte step lane c of part g reads 8 B at
// chunk_j + s*64 + 8*c for the 20 data chunks j, so a 128-byte line's two halves are read one
// step apart.  The real kernel spends ~5 us per step on the SHA waves beside it; `delay`
// reproduces that gap (s_sleep) so L2 can evict a line between its halves, as it would there.
constexpr size_t kC4Chunk = 256 * 1024;
constexpr int kC4D = 20, kC4T = 28;
__global__ __launch_bounds__(128) void wide8_steps(const uint8_t* __restrict__ p, size_t n_parts,
                                                   int delay, uint32_t* out) {
    const uint32_t g = threadIdx.x / 8, c = threadIdx.x % 8;
    const size_t part = blockIdx.x * (size_t)16 + g;
    if (part >= n_parts) return;
    const uint8_t* base = p + part * kC4T * kC4Chunk + 8 * c;
    uint32_t acc = 0;
    for (size_t s = 0; s < kC4Chunk / 64; ++s) {
#pragma unroll
        for (int j = 0; j < kC4D; ++j) {
            const uint2 v = *reinterpret_cast<const uint2*>(base + j * kC4Chunk + s * 64);
            acc ^= v.x + v.y;
        }
        for (int k = 0; k < delay; ++k) __builtin_amdgcn_s_sleep(127);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    const size_t n_streams = 57344;
    const size_t bytes = n_streams * kStream;  // 56 GiB: the C2 hashed bytes
    uint8_t* p;
    uint32_t* out;
    if (hipMalloc(&p, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    if (hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
    (void)hipMemset(p, 1, bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float ms;
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(coalesced, dim3(8192), dim3(256), 0, 0, (const uint4*)p, bytes / 16, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    printf("coalesced: %zu bytes, %.2f ms, %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(per_lane, dim3((n_streams + 255) / 256), dim3(256), 0, 0, p, n_streams, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    printf("per_lane : %zu bytes, %.2f ms, %.1f GB/s\n", bytes, ms, bytes / ms / 1e6);
    // C4 layout: 4096 parts x 28 chunks x 256 KiB (fits in the same allocation); the kernel
    // reads the 20 data chunks of every part once: 4096 * 20 * 256 KiB bytes.
    const size_t c4_parts = 4096, c4_read = c4_parts * kC4D * kC4Chunk;
    for (int delay : {0, 2}) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(wide8_steps, dim3(c4_parts / 16), dim3(128), 0, 0, p, c4_parts, delay,
                           out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        printf("wide8_steps delay=%d: %zu bytes, %.2f ms, %.1f GB/s\n", delay, c4_read, ms,
               c4_read / ms / 1e6);
    }
    return 0;
}
