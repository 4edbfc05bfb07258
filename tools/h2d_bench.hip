// H2D forms for the read stream's loaded chunks (dev tool): a batch of P parts x d loaded chunks
// of L bytes, scattered in a pinned [P][t][L] slot (random d of t per part), copied into a
// device [P][t][L] batch.  Compares
//   contig  : one copy of the same number of bytes (the link's ceiling)
//   runs    : one hipMemcpyAsync per run of consecutive loaded chunks (the pipeline today)
//   batch   : the same runs through hipMemcpyBatchAsync
//   kernel  : one gather kernel reading the pinned slot over PCIe (16 B per lane, non-temporal
//             device stores), the run table in device memory
// Each form is timed over `reps` batches on one stream; GB/s = loaded bytes / time.
//   hipcc --offload-arch=gfx950 -O3 -o tools/h2d_bench tools/h2d_bench.hip
//   tools/h2d_bench [parts=256] [L=1048576] [reps=8]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,                 \
                         hipGetErrorString(e_));                                           \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Run {
    unsigned long long off;  // byte offset in both slot and batch
    unsigned long long len;
};

// One workgroup per run slice of 1 MiB: 256 lanes x 16 B x 256 iterations.
__global__ void __launch_bounds__(256) gather_kernel(const u32x4* __restrict__ host,
                                                     u32x4* __restrict__ dev,
                                                     const Run* __restrict__ runs,
                                                     const unsigned* __restrict__ slice_run,
                                                     unsigned n_slices) {
    const unsigned s = blockIdx.x;
    if (s >= n_slices) return;
    const unsigned r = slice_run[s];
    const unsigned long long first = runs[r].off >> 4;
    const unsigned long long len16 = runs[r].len >> 4;
    // slice index within its run
    unsigned k = 0;
    while (s - k > 0 && slice_run[s - k - 1] == r) ++k;
    const unsigned long long lo = (unsigned long long)k << 16;  // 1 MiB / 16 B
    const unsigned long long hi = lo + (1ull << 16) < len16 ? lo + (1ull << 16) : len16;
    for (unsigned long long i = lo + threadIdx.x; i < hi; i += 256 * 4) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < hi) v[u] = host[first + i + u * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < hi) __builtin_nontemporal_store(v[u], &dev[first + i + u * 256]);
    }
}

struct Piece {
    const u32x4* src;
    u32x4* dst;
    unsigned long long len16;  // <= 64 Ki (1 MiB)
};

// Persistent form: grid-stride over a host-built list of <= 1 MiB pieces.
__global__ void __launch_bounds__(256) piece_kernel(const Piece* __restrict__ pieces, unsigned n) {
    for (unsigned q = blockIdx.x; q < n; q += gridDim.x) {
        const u32x4* __restrict__ src = pieces[q].src;
        u32x4* __restrict__ dst = pieces[q].dst;
        const unsigned len = unsigned(pieces[q].len16);
        for (unsigned i = threadIdx.x; i < len; i += 256 * 4) {
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * 256 < len) v[u] = src[i + u * 256];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * 256 < len) __builtin_nontemporal_store(v[u], &dst[i + u * 256]);
        }
    }
}

int main(int argc, char** argv) {
    const size_t P = argc > 1 ? std::atol(argv[1]) : 256;
    const size_t L = argc > 2 ? std::atol(argv[2]) : (1 << 20);
    const int reps = argc > 3 ? std::atoi(argv[3]) : 8;
    const size_t d = 10, t = 14;
    const size_t bytes = P * t * L, loaded = P * d * L;
    uint8_t *h = nullptr, *dv = nullptr, *dc = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&h), bytes, hipHostMallocPortable));
    CK(hipMalloc(&dv, bytes));
    CK(hipMalloc(&dc, loaded));
    for (size_t i = 0; i < bytes; i += 4096) h[i] = uint8_t(i >> 12);
    std::mt19937 rng(1);
    std::vector<Run> runs;
    for (size_t k = 0; k < P; ++k) {
        std::vector<int> idx(t);
        for (size_t i = 0; i < t; ++i) idx[i] = int(i);
        std::shuffle(idx.begin(), idx.end(), rng);
        std::vector<bool> m(t, false);
        for (size_t i = 0; i < d; ++i) m[idx[i]] = true;
        for (size_t i = 0; i < t;) {
            if (!m[i]) {
                ++i;
                continue;
            }
            size_t j = i;
            while (j < t && m[j]) ++j;
            runs.push_back({(k * t + i) * L, (j - i) * L});
            i = j;
        }
    }
    std::vector<unsigned> slice_run;
    for (size_t r = 0; r < runs.size(); ++r)
        for (unsigned long long o = 0; o < runs[r].len; o += (1u << 20)) slice_run.push_back(unsigned(r));
    Run* d_runs = nullptr;
    unsigned* d_sr = nullptr;
    CK(hipMalloc(&d_runs, runs.size() * sizeof(Run)));
    CK(hipMalloc(&d_sr, slice_run.size() * sizeof(unsigned)));
    CK(hipMemcpy(d_runs, runs.data(), runs.size() * sizeof(Run), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sr, slice_run.data(), slice_run.size() * sizeof(unsigned), hipMemcpyHostToDevice));
    std::vector<void*> dsts, srcs;
    std::vector<size_t> sizes;
    for (const auto& r : runs) {
        dsts.push_back(dv + r.off);
        srcs.push_back(h + r.off);
        sizes.push_back(r.len);
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    {
        hipPointerAttribute_t attr{};
        CK(hipPointerGetAttributes(&attr, h + 12345));
        std::printf("pointer attributes of an interior pinned address: type %d, devicePointer - p = "
                    "%lld, hostPointer - p = %lld\n", int(attr.type),
                    (long long)(reinterpret_cast<uint8_t*>(attr.devicePointer) - (h + 12345)),
                    (long long)(reinterpret_cast<uint8_t*>(attr.hostPointer) - (h + 12345)));
    }
    std::printf("P=%zu L=%zu: %zu runs, %zu slices, %.2f GiB loaded per batch\n", P, L, runs.size(),
                slice_run.size(), double(loaded) / double(1 << 30));
    auto time_it = [&](const char* name, auto fn) {
        fn();
        CK(hipStreamSynchronize(s));
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) fn();
        CK(hipStreamSynchronize(s));
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("%-8s %7.2f GB/s  (%.2f ms per batch)\n", name, double(loaded) * reps / sec / 1e9,
                    sec * 1e3 / reps);
        std::fflush(stdout);
    };
    time_it("contig", [&] { CK(hipMemcpyAsync(dc, h, loaded, hipMemcpyHostToDevice, s)); });
    time_it("runs", [&] {
        for (const auto& r : runs) CK(hipMemcpyAsync(dv + r.off, h + r.off, r.len, hipMemcpyHostToDevice, s));
    });
    time_it("batch", [&] {
        size_t fail = 0;
        CK(hipMemcpyBatchAsync(dsts.data(), srcs.data(), sizes.data(), dsts.size(), nullptr, nullptr,
                               0, &fail, s));
    });
    time_it("kernel", [&] {
        hipLaunchKernelGGL(gather_kernel, dim3(unsigned(slice_run.size())), dim3(256), 0, s,
                           reinterpret_cast<const u32x4*>(h), reinterpret_cast<u32x4*>(dv), d_runs,
                           d_sr, unsigned(slice_run.size()));
        CK(hipGetLastError());
    });
    // correctness of the kernel form on one run
    std::vector<uint8_t> back(runs[0].len);
    CK(hipMemcpy(back.data(), dv + runs[0].off, runs[0].len, hipMemcpyDeviceToHost));
    bool ok = true;
    for (size_t i = 0; i < runs[0].len; i += 4096) ok = ok && back[i] == h[runs[0].off + i];
    std::printf("kernel copy check: %s\n", ok ? "ok" : "MISMATCH");
    std::vector<Piece> h2d, d2h;
    for (const auto& r : runs)
        for (unsigned long long o = 0; o < r.len; o += (1u << 20)) {
            const unsigned long long n = std::min<unsigned long long>(1u << 20, r.len - o);
            h2d.push_back({reinterpret_cast<const u32x4*>(h + r.off + o),
                           reinterpret_cast<u32x4*>(dv + r.off + o), n >> 4});
            d2h.push_back({reinterpret_cast<const u32x4*>(dv + r.off + o),
                           reinterpret_cast<u32x4*>(h + r.off + o), n >> 4});
        }
    Piece *d_h2d = nullptr, *d_d2h = nullptr;
    CK(hipMalloc(&d_h2d, h2d.size() * sizeof(Piece)));
    CK(hipMalloc(&d_d2h, d2h.size() * sizeof(Piece)));
    CK(hipMemcpy(d_h2d, h2d.data(), h2d.size() * sizeof(Piece), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_d2h, d2h.data(), d2h.size() * sizeof(Piece), hipMemcpyHostToDevice));
    for (unsigned grid : {32u, 64u, 128u, 256u, 512u, 1024u, unsigned(h2d.size())}) {
        char name[32];
        std::snprintf(name, sizeof(name), "pc%u", grid);
        time_it(name, [&] {
            hipLaunchKernelGGL(piece_kernel, dim3(grid), dim3(256), 0, s, d_h2d, unsigned(h2d.size()));
            CK(hipGetLastError());
        });
    }
    time_it("d2h-runs", [&] {
        for (const auto& r : runs) CK(hipMemcpyAsync(h + r.off, dv + r.off, r.len, hipMemcpyDeviceToHost, s));
    });
    time_it("d2h-cont", [&] { CK(hipMemcpyAsync(h, dc, loaded, hipMemcpyDeviceToHost, s)); });
    for (unsigned grid : {64u, 256u, unsigned(d2h.size())}) {
        char name[32];
        std::snprintf(name, sizeof(name), "d2h-pc%u", grid);
        time_it(name, [&] {
            hipLaunchKernelGGL(piece_kernel, dim3(grid), dim3(256), 0, s, d_d2h, unsigned(d2h.size()));
            CK(hipGetLastError());
        });
    }
    // both directions at once on two streams: runs vs kernels
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto both = [&](const char* name, auto up, auto down) {
        up();
        down();
        CK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            up();
            down();
        }
        CK(hipDeviceSynchronize());
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("%-8s %7.2f GB/s of up-volume\n", name, double(loaded) * reps / sec / 1e9);
        std::fflush(stdout);
    };
    both("bi-copy", [&] { CK(hipMemcpyAsync(dc, h, loaded, hipMemcpyHostToDevice, s)); },
         [&] { CK(hipMemcpyAsync(h + (bytes - loaded), dv, loaded, hipMemcpyDeviceToHost, s2)); });
    both("bi-kern", [&] { hipLaunchKernelGGL(piece_kernel, dim3(256), dim3(256), 0, s, d_h2d, unsigned(h2d.size())); },
         [&] { CK(hipMemcpyAsync(h, dc, loaded, hipMemcpyDeviceToHost, s2)); });
    both("bi-kk", [&] { hipLaunchKernelGGL(piece_kernel, dim3(128), dim3(256), 0, s, d_h2d, unsigned(h2d.size())); },
         [&] { hipLaunchKernelGGL(piece_kernel, dim3(128), dim3(256), 0, s2, d_d2h, unsigned(d2h.size())); });
    both("bi-ck", [&] { CK(hipMemcpyAsync(dc, h, loaded, hipMemcpyHostToDevice, s)); },
         [&] { hipLaunchKernelGGL(piece_kernel, dim3(128), dim3(256), 0, s2, d_d2h, unsigned(d2h.size())); });
    // the read stream's mix: all loaded chunks up, ~29% of that volume (rebuilt chunks) down
    const size_t nd = d2h.size() * 2 / 7;
    const size_t nr = runs.size() * 2 / 7;
    both("mix-cc", [&] { for (const auto& r : runs) CK(hipMemcpyAsync(dv + r.off, h + r.off, r.len, hipMemcpyHostToDevice, s)); },
         [&] { for (size_t i = 0; i < nr; ++i) CK(hipMemcpyAsync(h + runs[i].off, dv + runs[i].off, runs[i].len, hipMemcpyDeviceToHost, s2)); });
    both("mix-kc", [&] { hipLaunchKernelGGL(piece_kernel, dim3(128), dim3(256), 0, s, d_h2d, unsigned(h2d.size())); },
         [&] { for (size_t i = 0; i < nr; ++i) CK(hipMemcpyAsync(h + runs[i].off, dv + runs[i].off, runs[i].len, hipMemcpyDeviceToHost, s2)); });
    both("mix-kk", [&] { hipLaunchKernelGGL(piece_kernel, dim3(128), dim3(256), 0, s, d_h2d, unsigned(h2d.size())); },
         [&] { hipLaunchKernelGGL(piece_kernel, dim3(64), dim3(256), 0, s2, d_d2h, unsigned(nd)); });
    both("mix-ck", [&] { for (const auto& r : runs) CK(hipMemcpyAsync(dv + r.off, h + r.off, r.len, hipMemcpyHostToDevice, s)); },
         [&] { hipLaunchKernelGGL(piece_kernel, dim3(64), dim3(256), 0, s2, d_d2h, unsigned(nd)); });
    CK(hipStreamDestroy(s2));
    CK(hipFree(d_runs));
    CK(hipFree(d_sr));
    CK(hipFree(dv));
    CK(hipFree(dc));
    CK(hipHostFree(h));
    return ok ? 0 : 1;
}
