// Minimal test of stream-ordered allocation reuse (dev tool; round 3, VERDICT r2 "weak" #7).
//
// Round 2 replaced hipMallocAsync / hipFreeAsync for per-launch metadata with an event-recycled
// pool after reads returned chunks the decode had not yet rewritten, and attributed that to the
// runtime reusing freed memory before work still reading it had finished.  This program asks
// the runtime that question directly, with no engine code:
//
//   stream A: P = hipMallocAsync; fill P with 0xA5A5A5A5; reader kernel re-reads P for ~20 ms and
//             counts words that are not 0xA5A5A5A5; hipFreeAsync(P)
//   stream B: Q = hipMallocAsync (same size); fill Q with 0x5A5A5A5A; hipFreeAsync(Q)
//
// Modes: "independent" (B has no ordering with A: the pool may reuse P for Q only once A's free
// has completed), "event" (B waits on an event recorded after A's free: reuse is legal and the
// reader is finished by then), "same" (Q allocated on A: stream order).  Per trial it prints
// whether Q == P and how many words the reader saw change.  Any nonzero count means freed memory
// was handed out and written while a kernel queued before the free was still reading it.
//
// Mode "join" is round 2's read-path shape itself: a side stream B waits on a fork event of A,
// allocates its metadata words with hipMallocAsync, uploads them, queues a host function that
// releases the host copy, runs a slow writer kernel (reading the words, writing an output
// buffer), frees the words with hipFreeAsync and records a join event; A waits on the join and
// copies the output to the host.  Any output word missing means A's copy ran before B's kernel
// finished although A waited on B's join.
//   hipcc --offload-arch=gfx950 -O3 tools/repro_free_async.hip -o tools/repro_free_async
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

constexpr int kThreads = 256, kBlocks = 1024;

// Every thread re-reads its words of p `reps` times and stores its own mismatch count and the
// last wrong value it saw, and the count over its FIRST pass alone (plain per-thread vector
// stores: no atomics).
__global__ void reader(const uint32_t* p, size_t n, uint32_t expect, int reps, uint32_t* bad) {
    const size_t tid = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    const size_t nt = stride;
    uint32_t miss = 0, first = 0, seen = expect;
    for (int r = 0; r < reps; ++r)
        for (size_t i = tid; i < n; i += stride) {
            const uint32_t v = __builtin_nontemporal_load(p + i);
            if (v != expect) {
                ++miss;
                first += r == 0;
                seen = v;
            }
        }
    bad[tid] = miss;
    bad[nt + tid] = first;
    bad[2 * nt + tid] = seen;
}

// The fill as a kernel on the stream (REPRO_FILL=kernel) instead of hipMemsetD32Async.
__global__ void fill(uint32_t* p, size_t n, uint32_t v) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

bool g_fill_kernel = false;
// REPRO_FREE=late: free only after the streams are synchronized (control); default: the free is
// queued right behind the work that uses the memory, as stream-ordered allocation allows.
bool g_free_late = false;

void fill_async(uint32_t* p, uint32_t v, size_t n, hipStream_t s) {
    if (g_fill_kernel) {
        hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, s, p, n, v);
        CK(hipGetLastError());
    } else {
        CK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(p), int(v), n, s));
    }
}

// Host buffers: pageable std::vector (default) or page-locked (REPRO_PINNED=1).
template <typename T>
T* host_buf(size_t n) {
    if (getenv("REPRO_PINNED") && getenv("REPRO_PINNED")[0] == '1') {
        void* p = nullptr;
        CK(hipHostMalloc(&p, n * sizeof(T), hipHostMallocDefault));
        return static_cast<T*>(p);
    }
    return new T[n];
}

// Writes out[i] = words[i % nw] + r for r = 0..reps-1 (the last pass leaves words[i % nw] +
// reps - 1): slow on purpose, reading the metadata words throughout.
__global__ void writer(const uint32_t* words, size_t nw, uint32_t* out, size_t n, int reps) {
    const size_t tid = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (int r = 0; r < reps; ++r)
        for (size_t i = tid; i < n; i += stride)
            __builtin_nontemporal_store(__builtin_nontemporal_load(words + i % nw) + uint32_t(r),
                                        out + i);
}

void release_host(void* p) { delete static_cast<std::vector<uint32_t>*>(p); }

int run_join(int trials, int reps) {
    const size_t n = size_t(1) << 22, nw = 4096;
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    uint32_t* out = nullptr;
    CK(hipMalloc(&out, n * sizeof(uint32_t)));
    uint32_t* host = host_buf<uint32_t>(n);
    int bad_trials = 0;
    for (int k = 0; k < trials; ++k) {
        fill_async(out, 0u, n, A);
        CK(hipEventRecord(fork, A));
        CK(hipStreamWaitEvent(B, fork, 0));
        auto* words = new std::vector<uint32_t>(nw);
        for (size_t i = 0; i < nw; ++i) (*words)[i] = uint32_t(k * 7919 + i) | 1u;
        uint32_t* dw = nullptr;
        CK(hipMallocAsync(reinterpret_cast<void**>(&dw), nw * sizeof(uint32_t), B));
        CK(hipMemcpyAsync(dw, words->data(), nw * sizeof(uint32_t), hipMemcpyHostToDevice, B));
        std::vector<uint32_t> expect(*words);
        CK(hipLaunchHostFunc(B, release_host, words));
        hipLaunchKernelGGL(writer, dim3(kBlocks), dim3(kThreads), 0, B, dw, nw, out, n, reps);
        CK(hipGetLastError());
        if (!g_free_late) CK(hipFreeAsync(dw, B));
        CK(hipEventRecord(join, B));
        CK(hipStreamWaitEvent(A, join, 0));
        CK(hipMemcpyAsync(host, out, n * sizeof(uint32_t), hipMemcpyDeviceToHost, A));
        CK(hipStreamSynchronize(A));
        size_t wrong = 0, at = 0;
        for (size_t i = 0; i < n; ++i)
            if (host[i] != expect[i % nw] + uint32_t(reps - 1) && !wrong++) at = i;
        bad_trials += wrong != 0;
        if (g_free_late) {
            CK(hipStreamSynchronize(B));
            CK(hipFreeAsync(dw, B));
        }
        printf("mode join        trial %2d: output words not yet written when A copied: %zu "
               "(first at %zu: %08x, expected %08x)\n", k, wrong, at, host[at],
               expect[at % nw] + uint32_t(reps - 1));
        fflush(stdout);
        CK(hipStreamSynchronize(B));
    }
    printf("mode join: %d trials, output incomplete in %d\n", trials, bad_trials);
    CK(hipFree(out));
    return bad_trials ? 3 : 0;
}

// Mode "fresh": every trial gets newly mapped device memory -- hipMalloc (REPRO_ALLOC=sync) or
// hipMallocAsync after trimming the default pool to 0 (REPRO_ALLOC=async, the default) -- fills
// it with a kernel right away and runs the reader.  Wrong words in a later pass of the reader
// (the first pass right) mean the memory changed under a kernel that was the only user of it:
// e.g. the driver's clear of a fresh allocation landing after the user's first writes.
int run_fresh(int trials, int reps) {
    const size_t n = size_t(1) << 22, bytes = n * sizeof(uint32_t);
    const bool sync_alloc = getenv("REPRO_ALLOC") && !strcmp(getenv("REPRO_ALLOC"), "sync");
    hipStream_t A;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    hipMemPool_t pool;
    CK(hipDeviceGetDefaultMemPool(&pool, 0));
    uint32_t* bad = nullptr;
    const size_t nt = size_t(kThreads) * kBlocks;
    CK(hipMalloc(&bad, 3 * nt * sizeof(uint32_t)));
    uint32_t* host = host_buf<uint32_t>(3 * nt);
    int corrupted = 0;
    for (int k = 0; k < trials; ++k) {
        uint32_t* P = nullptr;
        CK(hipMemsetAsync(bad, 0, 3 * nt * sizeof(uint32_t), A));
        if (sync_alloc) {
            CK(hipMalloc(reinterpret_cast<void**>(&P), bytes));
        } else {
            CK(hipMemPoolTrimTo(pool, 0));
            CK(hipMallocAsync(reinterpret_cast<void**>(&P), bytes, A));
        }
        fill_async(P, 0xA5A5A5A5u, n, A);
        hipLaunchKernelGGL(reader, dim3(kBlocks), dim3(kThreads), 0, A, P, n, 0xA5A5A5A5u, reps,
                           bad);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(A));
        CK(hipMemcpy(host, bad, 3 * nt * sizeof(uint32_t), hipMemcpyDeviceToHost));
        unsigned long long miss = 0, first = 0;
        uint32_t seen = 0xA5A5A5A5u;
        for (size_t i = 0; i < nt; ++i) {
            miss += host[i];
            first += host[nt + i];
            if (host[2 * nt + i] != 0xA5A5A5A5u) seen = host[2 * nt + i];
        }
        corrupted += miss != 0;
        printf("mode fresh (%s) trial %2d: P %p, wrong words seen: %llu (first pass %llu, a wrong "
               "value: %08x)\n", sync_alloc ? "hipMalloc" : "hipMallocAsync after trim", k,
               static_cast<void*>(P), miss, first, seen);
        fflush(stdout);
        if (sync_alloc) CK(hipFree(P));
        else CK(hipFreeAsync(P, A));
        CK(hipStreamSynchronize(A));
    }
    printf("mode fresh (%s): %d trials, reader saw changed words in %d\n",
           sync_alloc ? "hipMalloc" : "hipMallocAsync after trim", trials, corrupted);
    CK(hipFree(bad));
    return corrupted ? 3 : 0;
}

int main(int argc, char** argv) {
    const char* mode = argc > 1 ? argv[1] : "independent";
    const int trials = argc > 2 ? atoi(argv[2]) : 20;
    const int reps = argc > 3 ? atoi(argv[3]) : 64;
    g_fill_kernel = getenv("REPRO_FILL") && !strcmp(getenv("REPRO_FILL"), "kernel");
    g_free_late = getenv("REPRO_FREE") && !strcmp(getenv("REPRO_FREE"), "late");
    // REPRO_THRESHOLD=max: the default pool keeps freed memory (never trims it at sync points)
    if (getenv("REPRO_THRESHOLD") && !strcmp(getenv("REPRO_THRESHOLD"), "max")) {
        hipMemPool_t pool;
        CK(hipDeviceGetDefaultMemPool(&pool, 0));
        uint64_t thr = ~uint64_t(0);
        CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
    }
    printf("free: %s, pool release threshold: %s\n", g_free_late ? "after sync" : "stream-ordered",
           getenv("REPRO_THRESHOLD") ? getenv("REPRO_THRESHOLD") : "default");
    printf("fill: %s, host buffers: %s\n", g_fill_kernel ? "kernel" : "hipMemsetD32Async",
           getenv("REPRO_PINNED") && getenv("REPRO_PINNED")[0] == '1' ? "page-locked" : "pageable");
    if (!strcmp(mode, "join")) return run_join(trials, reps);
    if (!strcmp(mode, "fresh")) return run_fresh(trials, reps);
    const size_t n = size_t(1) << 22;  // 16 MiB of words
    const size_t bytes = n * sizeof(uint32_t);
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    hipEvent_t freed, t0, t1;
    CK(hipEventCreateWithFlags(&freed, hipEventDisableTiming));
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    uint32_t* bad = nullptr;
    const size_t nt = size_t(kThreads) * kBlocks;
    CK(hipMalloc(&bad, 3 * nt * sizeof(uint32_t)));
    uint32_t* host = host_buf<uint32_t>(3 * nt);
    int reused = 0, corrupted = 0;
    for (int k = 0; k < trials; ++k) {
        uint32_t *P = nullptr, *Q = nullptr;
        CK(hipMemsetAsync(bad, 0, 3 * nt * sizeof(uint32_t), A));
        CK(hipMallocAsync(reinterpret_cast<void**>(&P), bytes, A));
        fill_async(P, 0xA5A5A5A5u, n, A);
        CK(hipEventRecord(t0, A));
        hipLaunchKernelGGL(reader, dim3(kBlocks), dim3(kThreads), 0, A, P, n, 0xA5A5A5A5u, reps,
                           bad);
        CK(hipGetLastError());
        CK(hipEventRecord(t1, A));
        if (!g_free_late) CK(hipFreeAsync(P, A));
        hipStream_t qs = B;
        if (!strcmp(mode, "event")) {
            CK(hipEventRecord(freed, A));
            CK(hipStreamWaitEvent(B, freed, 0));
        } else if (!strcmp(mode, "same")) {
            qs = A;
        }
        CK(hipMallocAsync(reinterpret_cast<void**>(&Q), bytes, qs));
        fill_async(Q, 0x5A5A5A5Au, n, qs);
        if (!g_free_late) CK(hipFreeAsync(Q, qs));
        CK(hipStreamSynchronize(A));
        CK(hipStreamSynchronize(B));
        if (g_free_late) {
            CK(hipFreeAsync(P, A));
            CK(hipFreeAsync(Q, qs));
        }
        CK(hipMemcpy(host, bad, 3 * nt * sizeof(uint32_t), hipMemcpyDeviceToHost));
        unsigned long long miss = 0, first = 0;
        uint32_t seen = 0xA5A5A5A5u;
        for (size_t i = 0; i < nt; ++i) {
            miss += host[i];
            first += host[nt + i];
            if (host[2 * nt + i] != 0xA5A5A5A5u) seen = host[2 * nt + i];
        }
        float ms = 0;
        CK(hipEventElapsedTime(&ms, t0, t1));
        reused += P == Q;
        corrupted += miss != 0;
        printf("mode %-11s trial %2d: P %p Q %p, reader %.1f ms, wrong words seen: %llu (first "
               "pass %llu, a wrong value: %08x)\n", mode, k, static_cast<void*>(P),
               static_cast<void*>(Q), ms, miss, first, seen);
        fflush(stdout);
    }
    printf("mode %s: %d trials, Q reused P's address %d times, reader saw changed words in %d\n",
           mode, trials, reused, corrupted);
    CK(hipFree(bad));
    return corrupted ? 3 : 0;
}
