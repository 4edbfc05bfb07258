// Streaming ceiling for the RS(10,4) access pattern (dev tool): part-major batch
// [part][14][1 MiB]; each thread reads its column of the 10 data chunks and writes 4 outputs
// (trivial xor "parity"), no GF work.  Sweeps bytes per lane, columns per thread and threads per
// block so rs_apply_kernel can be compared with the best achievable rate for its pattern.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_stream.hip -o tools/ubench_stream
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr int D = 10, P = 4, T = D + P;
constexpr size_t L = 1 << 20;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4u ld(const uint8_t* p) {
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return *reinterpret_cast<const v4u*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(uint8_t* p, v4u v) {
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
    else *reinterpret_cast<v4u*>(p) = v;
}

// V = 16-byte vectors per lane per input (1, 2, 4); ITERS column steps per thread (grid-tile).
template <int V, int ITERS, bool NT>
__global__ void stream_kernel(uint8_t* base, uint32_t tiles_per_part) {
    const uint32_t part = blockIdx.x / tiles_per_part;
    const uint32_t tile = blockIdx.x - part * tiles_per_part;
    uint8_t* pb = base + size_t(part) * T * L;
    const size_t step = size_t(blockDim.x) * 16 * V;
#pragma unroll 1
    for (int it = 0; it < ITERS; ++it) {
        const size_t x = (size_t(tile) * ITERS + it) * step + size_t(threadIdx.x) * 16;
        v4u acc[V];
        for (int u = 0; u < V; ++u) acc[u] = v4u{0, 0, 0, 0};
        v4u in[D][V];
#pragma unroll
        for (int j = 0; j < D; ++j)
#pragma unroll
            for (int u = 0; u < V; ++u) in[j][u] = ld<NT>(pb + j * L + x + size_t(u) * blockDim.x * 16);
#pragma unroll
        for (int j = 0; j < D; ++j)
#pragma unroll
            for (int u = 0; u < V; ++u) acc[u] ^= in[j][u];
#pragma unroll
        for (int r = 0; r < P; ++r)
#pragma unroll
            for (int u = 0; u < V; ++u)
                st<NT>(pb + (D + r) * L + x + size_t(u) * blockDim.x * 16, acc[u] + v4u{unsigned(r), unsigned(r), unsigned(r), unsigned(r)});
    }
}

template <int V, int ITERS, bool NT>
void run(uint8_t* base, uint32_t parts, int threads, const char* name) {
    const size_t per_block = size_t(threads) * 16 * V * ITERS;
    const uint32_t tiles = uint32_t(L / per_block);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((stream_kernel<V, ITERS, NT>), dim3(parts * tiles), dim3(threads), 0, 0,
                           base, tiles);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r && ms < best) best = ms;
    }
    const double bytes = double(parts) * T * L;
    printf("%-28s threads %4d  V %d ITERS %d NT %d : %8.3f ms  %7.0f GB/s\n", name, threads, V,
           ITERS, int(NT), best, bytes / best / 1e6);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const uint32_t parts = argc > 1 ? uint32_t(atoi(argv[1])) : 4096;
    uint8_t* base;
    CK(hipMalloc(&base, size_t(parts) * T * L));
    CK(hipMemset(base, 1, size_t(parts) * T * L));
    run<1, 4, false>(base, parts, 256, "v1 it4 (rs_apply shape)");
    run<1, 4, true>(base, parts, 256, "v1 it4 nt");
    run<1, 1, false>(base, parts, 256, "v1 it1");
    run<1, 16, false>(base, parts, 256, "v1 it16");
    run<2, 2, false>(base, parts, 256, "v2 it2");
    run<2, 4, false>(base, parts, 256, "v2 it4");
    run<4, 1, false>(base, parts, 256, "v4 it1");
    run<4, 2, false>(base, parts, 256, "v4 it2");
    run<1, 4, false>(base, parts, 512, "v1 it4 t512");
    run<2, 2, false>(base, parts, 512, "v2 it2 t512");
    run<1, 4, false>(base, parts, 1024, "v1 it4 t1024");
    run<2, 2, true>(base, parts, 256, "v2 it2 nt");
    CK(hipFree(base));
    return 0;
}
