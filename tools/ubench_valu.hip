// Microbenchmark (dev tool, not product): per-wave VALU issue cost of the integer ops the
// SHA-256 and GF(2^8) kernels use, on gfx950.  One block; waves_per_simd = blockDim/256.
// Reports cycles per instruction per wave (s_memtime) for 8 independent chains (ILP 8) and
// a single dependent chain (ILP 1).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP, int ILP>
__global__ void kern(uint32_t* out, uint64_t* cyc, int iters) {
    uint32_t a[8], b = threadIdx.x * 7 + 1, c = threadIdx.x ^ 0x55;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x + i * 13;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#define STEP(i) if (i < ILP || ILP == 8) { \
            if (OP == 0) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(b)); \
            if (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c)); \
            if (OP == 2) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)); \
            if (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)); \
            if (OP == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b)); \
            if (OP == 5) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(b), "v"(c)); \
            if (OP == 6) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)); \
            if (OP == 7) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[i])); \
            if (OP == 8) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b)); \
            if (OP == 9) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b)); \
            }
            if (ILP == 8) { REP8(STEP) } else { STEP(0) }
#undef STEP
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP, int ILP>
double run(int threads, int blocks, int iters) {
    uint32_t* out; uint64_t* cyc;
    hipMalloc(&out, blocks * threads * 4);
    hipMalloc(&cyc, blocks * (threads / 64) * 8);
    hipLaunchKernelGGL((kern<OP, ILP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    hipLaunchKernelGGL((kern<OP, ILP>), dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    int nw = blocks * (threads / 64);
    uint64_t* h = new uint64_t[nw];
    hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
    delete[] h; hipFree(out); hipFree(cyc);
    const double n_inst = double(iters) * 8 * (ILP == 8 ? 8 : 1);
    return mx / n_inst;  // s_memtime ticks per instruction per wave
}

static const char* names[] = {"v_alignbit_b32", "v_bitop3_b32", "v_add3_u32", "v_add_u32",
                              "v_xor_b32", "v_perm_b32", "v_bfi_b32", "v_lshrrev_b32",
                              "v_and_b32", "v_add_f32"};

template <int OP>
void row(int iters) {
    printf("%-16s  ilp8: 1w/simd %.2f  2w/simd %.2f  4w/simd %.2f | ilp1: 1w %.2f  2w %.2f\n",
           names[OP], run<OP, 8>(256, 1, iters), run<OP, 8>(512, 1, iters),
           run<OP, 8>(1024, 1, iters), run<OP, 1>(256, 1, iters * 4),
           run<OP, 1>(512, 1, iters * 4));
}

int main() {
    int iters = 4096;
    // s_memtime tick rate vs shader clock: report both via a timed kernel
    row<0>(iters); row<1>(iters); row<2>(iters); row<3>(iters); row<4>(iters);
    row<5>(iters); row<6>(iters); row<7>(iters); row<8>(iters); row<9>(iters);
    return 0;
}
