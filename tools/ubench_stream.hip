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
// cs = chunk stride (L, or L + a pad that staggers the 14 streams of a part across channels).
template <int V, int ITERS, bool NT>
__global__ void stream_kernel(uint8_t* base, uint32_t tiles_per_part, size_t cs) {
    const uint32_t part = blockIdx.x / tiles_per_part;
    const uint32_t tile = blockIdx.x - part * tiles_per_part;
    uint8_t* pb = base + size_t(part) * T * cs;
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
            for (int u = 0; u < V; ++u) in[j][u] = ld<NT>(pb + j * cs + x + size_t(u) * blockDim.x * 16);
#pragma unroll
        for (int j = 0; j < D; ++j)
#pragma unroll
            for (int u = 0; u < V; ++u) acc[u] ^= in[j][u];
#pragma unroll
        for (int r = 0; r < P; ++r)
#pragma unroll
            for (int u = 0; u < V; ++u)
                st<NT>(pb + (D + r) * cs + x + size_t(u) * blockDim.x * 16, acc[u] + v4u{unsigned(r), unsigned(r), unsigned(r), unsigned(r)});
    }
}

// Loads and stores with separate cache policies (round 3): NTL non-temporal loads, NTS
// non-temporal stores; XCD=true maps blocks so that each of the 8 XCDs (blocks are dealt to them
// round-robin) walks its own contiguous run of parts.
template <int V, bool NTL, bool NTS, bool XCD>
__global__ void stream_mix_kernel(uint8_t* base, uint32_t tiles_per_part, uint32_t n_blocks) {
    uint32_t b = blockIdx.x;
    if (XCD) {  // block b runs on XCD b % 8: give XCD x the blocks [x*n/8, (x+1)*n/8)
        const uint32_t per = n_blocks / 8;
        b = (b % 8) * per + b / 8;
    }
    const uint32_t part = b / tiles_per_part;
    const uint32_t tile = b - part * tiles_per_part;
    uint8_t* pb = base + size_t(part) * T * L;
    const size_t x = size_t(tile) * blockDim.x * 16 * V + size_t(threadIdx.x) * 16;
    v4u acc[V];
    for (int u = 0; u < V; ++u) acc[u] = v4u{0, 0, 0, 0};
    v4u in[D][V];
#pragma unroll
    for (int j = 0; j < D; ++j)
#pragma unroll
        for (int u = 0; u < V; ++u) in[j][u] = ld<NTL>(pb + j * L + x + size_t(u) * blockDim.x * 16);
#pragma unroll
    for (int j = 0; j < D; ++j)
#pragma unroll
        for (int u = 0; u < V; ++u) acc[u] ^= in[j][u];
#pragma unroll
    for (int r = 0; r < P; ++r)
#pragma unroll
        for (int u = 0; u < V; ++u)
            st<NTS>(pb + (D + r) * L + x + size_t(u) * blockDim.x * 16,
                    acc[u] + v4u{unsigned(r), unsigned(r), unsigned(r), unsigned(r)});
}

template <int V, bool NTL, bool NTS, bool XCD>
void run_mix(uint8_t* base, uint32_t parts, int cap = 0) {
    // cap > 0: at most `cap` 256-thread blocks per CU (an unused LDS reservation, 160 KiB per CU)
    const uint32_t lds = cap > 0 ? 163840u / uint32_t(cap + 1) + 2048u : 0u;
    if (lds > 65536)
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&stream_mix_kernel<V, NTL, NTS, XCD>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    const uint32_t tiles = uint32_t(L / (size_t(256) * 16 * V));
    const uint32_t n = parts * tiles;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f, sum = 0;
    for (int r = 0; r < 8; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((stream_mix_kernel<V, NTL, NTS, XCD>), dim3(n), dim3(256), lds, 0, base,
                           tiles, n);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r) {
            sum += ms;
            if (ms < best) best = ms;
        }
    }
    const double bytes = double(parts) * T * L;
    printf("mix V %d nt-load %d nt-store %d xcd-map %d cap %d : best %8.3f ms %7.0f GB/s, mean %7.0f GB/s\n",
           V, int(NTL), int(NTS), int(XCD), cap, best, bytes / best / 1e6, bytes / (sum / 7) / 1e6);
    fflush(stdout);
}

// Reconstruct-shaped pattern: the D inputs read, W (< P) outputs written (a 2-erasure
// reconstruct_data writes 1-2 data chunks per part).
template <int V, bool NT, int W, bool XCD = false>
__global__ void stream_w_kernel(uint8_t* base, uint32_t tiles_per_part, size_t cs) {
    uint32_t b = blockIdx.x;
    if (XCD) {  // as stream_mix_kernel: XCD x walks the blocks [x*n/8, (x+1)*n/8)
        const uint32_t per = gridDim.x / 8;
        b = (b % 8) * per + b / 8;
    }
    const uint32_t part = b / tiles_per_part;
    const uint32_t tile = b - part * tiles_per_part;
    uint8_t* pb = base + size_t(part) * T * cs;
    const size_t x = size_t(tile) * blockDim.x * 16 * V + size_t(threadIdx.x) * 16;
    v4u acc[V];
    for (int u = 0; u < V; ++u) acc[u] = v4u{0, 0, 0, 0};
    v4u in[D][V];
#pragma unroll
    for (int j = 0; j < D; ++j)
#pragma unroll
        for (int u = 0; u < V; ++u) in[j][u] = ld<NT>(pb + j * cs + x + size_t(u) * blockDim.x * 16);
#pragma unroll
    for (int j = 0; j < D; ++j)
#pragma unroll
        for (int u = 0; u < V; ++u) acc[u] ^= in[j][u];
#pragma unroll
    for (int r = 0; r < W; ++r)
#pragma unroll
        for (int u = 0; u < V; ++u)
            st<NT>(pb + (D + r) * cs + x + size_t(u) * blockDim.x * 16, acc[u] + v4u{unsigned(r), 0u, 0u, 0u});
}

template <int V, bool NT, int W, bool XCD = false>
void run_w(uint8_t* base, uint32_t parts, int threads, int cap = 0) {
    const uint32_t lds = cap > 0 ? 163840u / uint32_t(cap + 1) + 2048u : 0u;
    if (lds > 65536)
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&stream_w_kernel<V, NT, W, XCD>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    const uint32_t tiles = uint32_t(L / (size_t(threads) * 16 * V));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((stream_w_kernel<V, NT, W, XCD>), dim3(parts * tiles), dim3(threads), lds, 0,
                           base, tiles, L);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r && ms < best) best = ms;
    }
    const double bytes = double(parts) * (D + W) * L;
    printf("reads %d + writes %d  V %d NT %d threads %4d xcd-map %d cap %d : %8.3f ms  %7.0f GB/s\n",
           D, W, V, int(NT), threads, int(XCD), cap, best, bytes / best / 1e6);
    fflush(stdout);
}

// Read-only (14 streams) / write-only (14 streams) ceilings of the same layout.
template <bool NT>
__global__ void read_kernel(const uint8_t* base, uint32_t tiles_per_part, uint32_t* sink) {
    const uint32_t part = blockIdx.x / tiles_per_part;
    const uint32_t tile = blockIdx.x - part * tiles_per_part;
    const uint8_t* pb = base + size_t(part) * T * L;
    const size_t x = size_t(tile) * blockDim.x * 32 + size_t(threadIdx.x) * 16;
    v4u acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < T; ++j) {
        acc ^= ld<NT>(pb + j * L + x);
        acc ^= ld<NT>(pb + j * L + x + blockDim.x * 16);
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <bool NT>
__global__ void write_kernel(uint8_t* base, uint32_t tiles_per_part) {
    const uint32_t part = blockIdx.x / tiles_per_part;
    const uint32_t tile = blockIdx.x - part * tiles_per_part;
    uint8_t* pb = base + size_t(part) * T * L;
    const size_t x = size_t(tile) * blockDim.x * 32 + size_t(threadIdx.x) * 16;
    const v4u v = {part, tile, threadIdx.x, 7u};
#pragma unroll
    for (int j = 0; j < T; ++j) {
        st<NT>(pb + j * L + x, v);
        st<NT>(pb + j * L + x + blockDim.x * 16, v);
    }
}

// Persistent: one workgroup per CU slot walks whole parts (grid-stride over 8 KiB steps).
template <bool NT>
__global__ void persistent_kernel(uint8_t* base, uint32_t parts) {
    const size_t steps_per_part = L / (size_t(blockDim.x) * 32);
    const size_t total = size_t(parts) * steps_per_part;
    for (size_t s = blockIdx.x; s < total; s += gridDim.x) {
        const size_t part = s / steps_per_part, step = s - part * steps_per_part;
        uint8_t* pb = base + part * T * L;
        const size_t x = step * blockDim.x * 32 + size_t(threadIdx.x) * 16;
        v4u acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
        v4u in0[D], in1[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            in0[j] = ld<NT>(pb + j * L + x);
            in1[j] = ld<NT>(pb + j * L + x + blockDim.x * 16);
        }
#pragma unroll
        for (int j = 0; j < D; ++j) {
            acc0 ^= in0[j];
            acc1 ^= in1[j];
        }
#pragma unroll
        for (int r = 0; r < P; ++r) {
            st<NT>(pb + (D + r) * L + x, acc0);
            st<NT>(pb + (D + r) * L + x + blockDim.x * 16, acc1);
        }
    }
}

template <typename K>
void run_simple(const char* name, K launch, double bytes) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r && ms < best) best = ms;
    }
    printf("%-40s : %8.3f ms  %7.0f GB/s\n", name, best, bytes / best / 1e6);
    fflush(stdout);
}

template <int V, int ITERS, bool NT>
void run(uint8_t* base, uint32_t parts, int threads, const char* name, size_t pad = 0) {
    const size_t per_block = size_t(threads) * 16 * V * ITERS;
    const uint32_t tiles = uint32_t(L / per_block);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((stream_kernel<V, ITERS, NT>), dim3(parts * tiles), dim3(threads), 0, 0,
                           base, tiles, L + pad);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r && ms < best) best = ms;
    }
    const double bytes = double(parts) * T * L;
    printf("%-28s threads %4d  V %d ITERS %d NT %d pad %6zu : %8.3f ms  %7.0f GB/s\n", name,
           threads, V, ITERS, int(NT), pad, best, bytes / best / 1e6);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const uint32_t parts = argc > 1 ? uint32_t(atoi(argv[1])) : 4096;
    const size_t max_pad = 64 * 1024 + 256;
    uint8_t* base;
    CK(hipMalloc(&base, size_t(parts) * T * (L + max_pad)));
    CK(hipMemset(base, 1, size_t(parts) * T * (L + max_pad)));
    if (argc > 2 && argv[2][0] == 'w') {  // reconstruct-shaped ceilings: 10 reads + W writes
        run_w<2, true, 1>(base, parts, 256);
        run_w<2, true, 2>(base, parts, 256);
        run_w<2, true, 3>(base, parts, 256);
        run_w<2, true, 4>(base, parts, 256);
        run_w<4, true, 2>(base, parts, 256);
        run_w<1, true, 2>(base, parts, 256);
        run_w<2, false, 2>(base, parts, 256);
        run_w<2, true, 2>(base, parts, 512);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'x') {  // reconstruct-shaped ceilings with the XCD-aware order
        for (int rep = 0; rep < 2; ++rep) {
            run_w<2, true, 1, false>(base, parts, 256);
            run_w<2, true, 1, true>(base, parts, 256);
            run_w<2, true, 2, false>(base, parts, 256);
            run_w<2, true, 2, true>(base, parts, 256);
            run_w<2, true, 4, false>(base, parts, 256);
            run_w<2, true, 4, true>(base, parts, 256);
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'v') {  // bytes per lane x residency cap
        for (int rep = 0; rep < 2; ++rep)
            for (int cap : {1, 2, 3, 4}) {
                run_mix<1, true, true, true>(base, parts, cap);
                run_mix<2, true, true, true>(base, parts, cap);
                run_mix<4, true, true, true>(base, parts, cap);
            }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'c') {  // residency caps (blocks per CU) on the best mix shape
        for (int rep = 0; rep < 2; ++rep) {
            for (int cap : {0, 1, 2, 3, 4, 6}) run_mix<2, true, true, true>(base, parts, cap);
            for (int cap : {0, 2, 3}) {
                run_w<2, true, 1, true>(base, parts, 256, cap);
                run_w<2, true, 2, true>(base, parts, 256, cap);
            }
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'm') {  // load / store policies and XCD-aware block mapping
        for (int rep = 0; rep < 2; ++rep) {
            run_mix<2, true, true, false>(base, parts);
            run_mix<2, true, false, false>(base, parts);
            run_mix<2, false, true, false>(base, parts);
            run_mix<2, false, false, false>(base, parts);
            run_mix<2, true, true, true>(base, parts);
            run_mix<2, true, false, true>(base, parts);
            run_mix<4, true, true, false>(base, parts);
            run_mix<4, true, false, false>(base, parts);
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'p') {  // chunk-stride pad sweep of the best shapes
        for (size_t pad : {size_t(0), size_t(256), size_t(1024), size_t(4096), size_t(8192 + 256),
                           size_t(65536), max_pad}) {
            run<2, 1, true>(base, parts, 256, "v2 it1 nt", pad);
            run<4, 1, true>(base, parts, 256, "v4 it1 nt", pad);
        }
        return 0;
    }
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
    run<2, 1, true>(base, parts, 256, "v2 it1 nt");
    run<4, 1, true>(base, parts, 256, "v4 it1 nt");
    run<2, 2, true>(base, parts, 512, "v2 it2 nt t512");
    const double all = double(parts) * T * L;
    const uint32_t tiles = uint32_t(L / (256 * 32));
    uint32_t* sink;
    CK(hipMalloc(&sink, 64));
    run_simple("read-only 14 streams", [&] {
        hipLaunchKernelGGL((read_kernel<false>), dim3(parts * tiles), dim3(256), 0, 0, base, tiles, sink); }, all);
    run_simple("read-only 14 streams nt", [&] {
        hipLaunchKernelGGL((read_kernel<true>), dim3(parts * tiles), dim3(256), 0, 0, base, tiles, sink); }, all);
    run_simple("write-only 14 streams", [&] {
        hipLaunchKernelGGL((write_kernel<false>), dim3(parts * tiles), dim3(256), 0, 0, base, tiles); }, all);
    run_simple("write-only 14 streams nt", [&] {
        hipLaunchKernelGGL((write_kernel<true>), dim3(parts * tiles), dim3(256), 0, 0, base, tiles); }, all);
    for (int wg : {1024, 2048, 4096, 8192}) {
        char name[64];
        snprintf(name, sizeof name, "persistent nt grid %d", wg);
        run_simple(name, [&] {
            hipLaunchKernelGGL((persistent_kernel<true>), dim3(wg), dim3(256), 0, 0, base, parts); }, all);
    }
    CK(hipFree(base));
    return 0;
}
