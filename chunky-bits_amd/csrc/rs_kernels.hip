// rs_kernels.hip — gfx950 (MI355X, CDNA4) GF(2^8) Reed-Solomon kernels + synthetic fill.
//
//  rs_apply_kernel      GF(2^8) matrix x chunk-set multiply.  One kernel serves
//                       ReedSolomon::encode_sep (rows = parity rows of M, inputs = the d data
//                       chunks) and reconstruct / reconstruct_data (rows = decode rows, inputs =
//                       the first d present chunks), for thousands of parts per launch.
//                       HBM-bound: algorithmic bytes per part = (d + n_out) * len.
//  rs_apply_var_kernel  the same for a reconstruct batch whose parts miss different numbers of
//                       chunks: one launch, each block dispatched on its pattern's row count.
//  fill_kernel          counter-based synthetic bytes for benchmarks/tests.
//
// GF multiply: no GF instruction exists, so a product c*x of four packed bytes is three
// v_perm_b32 byte-table lookups (x split into bits [2:0], [5:3], [7:6]; see gf256.hpp) combined
// with one v_bitop3_b32 (xor3).  The selectors of a data word are shared by every output row.
// Coefficient tables are wave-uniform and come in through scalar loads (s_load), so a row costs
// 3 v_perm + ~1.5 xor per data dword, with no LDS traffic and no bank conflicts.
//
// Memory shape: a block owns a 16 KiB (rs_apply_kernel) or 8 KiB (bit-sliced encoder, mixed-
// pattern reconstruct) column range of one part; each lane moves V 16-byte columns per input per
// step (V = 2: two 1 KiB-per-wave loads per input in flight) with non-temporal loads and stores
// (every byte is touched once), blocks in an XCD-aware order, and on large grids a residency cap
// of 2-3 blocks per CU (apply_lds).  RS(10,4) encode streams 6.40 TB/s and 2-erasure
// reconstruct_data 5.96 TB/s.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "device_common.hpp"
#include "gf256.hpp"
#include "gf_const.hpp"
#include "gf_device.hpp"
#include "kernels.hpp"
#include "knobs.hpp"

namespace cec {
namespace {

using namespace gf;

constexpr int kApplyThreads = 256;
constexpr uint64_t kApplyTile = 16384;  // default bytes of one part's column range per block
constexpr uint64_t kSpan = uint64_t(kApplyThreads) * 16u;  // bytes per block per column step
constexpr uint32_t kMaxApplyRows = 8;

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    if (NT) {
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *reinterpret_cast<const uint4*>(p);
}

template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) {
    if (NT) {
        v4u w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(p));
    } else {
        *reinterpret_cast<uint4*>(p) = v;
    }
}

// V 16-byte columns (x + c*kSpan, c < V) of a part: acc[r] = XOR_j coef[r][j] (x) in_j[...].
// FULL: every lane of the block has V*16 valid bytes and the layout is 16-byte aligned
// (otherwise V == 1 with a byte-granular load/store of a rem < 16 tail).
// tab points at row0's table of input 0; input j's RG tables start at tab + j*tab_stride.
// GROUP inputs (x V columns) are loaded before any is multiplied; NT selects non-temporal
// loads/stores (streamed once, never re-read).
template <int RG, bool FULL, int GROUP, int V, bool NT>
__device__ __forceinline__ void apply_column(uint8_t* pbase, uint64_t cs, uint64_t x,
                                             uint64_t rem, uint32_t d, uint32_t tab_stride,
                                             cu32* in_idx, cu32* out_idx, cu32* tab) {
    static_assert(FULL || V == 1, "ragged columns are single");
    uint32_t acc[RG][V][4];
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int c = 0; c < V; ++c) acc[r][c][0] = acc[r][c][1] = acc[r][c][2] = acc[r][c][3] = 0u;
    const uint64_t n = rem < 16 ? rem : 16;

#pragma unroll 1
    for (uint32_t j0 = 0; j0 < d; j0 += GROUP) {
        uint4 v[GROUP][V];
#pragma unroll
        for (int u = 0; u < GROUP; ++u) {
#pragma unroll
            for (int c = 0; c < V; ++c) v[u][c] = make_uint4(0u, 0u, 0u, 0u);
            if (j0 + u < d) {
                const uint8_t* src = pbase + uint64_t(in_idx[j0 + u]) * cs + x;
#pragma unroll
                for (int c = 0; c < V; ++c) {
                    if (FULL) v[u][c] = ld16<NT>(src + c * kSpan);
                    else v[u][c] = load_partial(src, n);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < GROUP; ++u) {
            if (j0 + u < d) {
                cu32* tj = tab + size_t(j0 + u) * tab_stride;
#pragma unroll
                for (int c = 0; c < V; ++c) {
                    const Sel s0 = selectors(v[u][c].x), s1 = selectors(v[u][c].y),
                              s2 = selectors(v[u][c].z), s3 = selectors(v[u][c].w);
#pragma unroll
                    for (int r = 0; r < RG; ++r) {
                        cu32* t = tj + r * kTabWords;
                        const uint32_t t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3], t4 = t[4];
                        acc[r][c][0] ^= gmul(s0, t0, t1, t2, t3, t4);
                        acc[r][c][1] ^= gmul(s1, t0, t1, t2, t3, t4);
                        acc[r][c][2] ^= gmul(s2, t0, t1, t2, t3, t4);
                        acc[r][c][3] ^= gmul(s3, t0, t1, t2, t3, t4);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RG; ++r) {
        uint8_t* dst = pbase + uint64_t(out_idx[r]) * cs + x;
#pragma unroll
        for (int c = 0; c < V; ++c) {
            if (FULL)
                st16<NT>(dst + c * kSpan,
                         make_uint4(acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]));
            else
                store_partial(dst, acc[r][c], n);
        }
    }
}

// One 16 KiB column tile of one part, rows [row0, row0 + RG) of its pattern record (n_out rows
// in all).  Full column steps (kSpan*V bytes, aligned layout) take the V-wide path; the rest
// (ragged end, unaligned layouts) the byte-granular single-column path.
template <int RG, bool VEC, int GROUP, int V, bool NT>
__device__ __forceinline__ void apply_tile(const ApplyParams& a, cu32* pat, uint32_t part,
                                           uint32_t tile, uint32_t n_out, uint32_t row0,
                                           uint32_t tile_bytes) {
    const uint32_t d = a.d;
    cu32* in_idx = pat + 1;
    cu32* out_idx = pat + 1 + d + row0;
    cu32* tab = pat + 1 + d + n_out + size_t(row0) * kTabWords;
    const uint32_t tab_stride = n_out * kTabWords;
    uint8_t* pbase = a.base + uint64_t(part) * a.part_stride;
    const uint64_t len = a.len;
    const uint64_t cs = a.chunk_stride;
    const uint64_t t0 = uint64_t(tile) * tile_bytes;
    const uint64_t t1 = t0 + tile_bytes < len ? t0 + tile_bytes : len;
#pragma unroll 1
    for (uint64_t xb = t0; xb < t1; xb += kSpan * V) {  // block-uniform
        const uint64_t x = xb + uint64_t(threadIdx.x) * 16u;
        if (VEC && xb + kSpan * V <= len) {
            apply_column<RG, true, GROUP, V, NT>(pbase, cs, x, len - x, d, tab_stride, in_idx,
                                                 out_idx, tab);
        } else {
#pragma unroll 1
            for (uint64_t xc = x; xc < t1 && xc < xb + kSpan * V; xc += kSpan)
                apply_column<RG, false, 4, 1, false>(pbase, cs, xc, len - xc, d, tab_stride,
                                                     in_idx, out_idx, tab);
        }
    }
}

// ---- compile-time d: the same multiply with every input's loads issued one group ahead ----
// With d a run-time value the column loop above waits for each group's loads before it multiplies
// (`unroll 1`, no prefetch across groups).  For the compiled input counts (rs_apply_var_kernel's
// CDG instantiations) the loop unrolls at compile time and group J0 + G's loads go out before
// group J0's multiplies, as in the bit-sliced encoder.
template <int D, int G, int J0, int V>
__device__ __forceinline__ void vp_load(uint4 (&v)[G][V], const uint8_t* pbase, uint64_t cs,
                                        uint64_t x, cu32* in_idx) {
#pragma unroll
    for (int u = 0; u < G; ++u)
        if (J0 + u < D) {
            const uint8_t* src = pbase + uint64_t(in_idx[J0 + u]) * cs + x;
#pragma unroll
            for (int c = 0; c < V; ++c) v[u][c] = ld16<true>(src + c * kSpan);
        }
}

template <int D, int RG, int G, int J0, int V>
__device__ __forceinline__ void vp_mul(uint32_t (&acc)[RG][V][4], uint4 (&v)[G][V], cu32* tab,
                                       uint32_t tab_stride) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
        if (J0 + u < D) {
            cu32* tj = tab + size_t(J0 + u) * tab_stride;
#pragma unroll
            for (int c = 0; c < V; ++c) {
                const Sel s0 = selectors(v[u][c].x), s1 = selectors(v[u][c].y),
                          s2 = selectors(v[u][c].z), s3 = selectors(v[u][c].w);
#pragma unroll
                for (int r = 0; r < RG; ++r) {
                    cu32* t = tj + r * kTabWords;
                    const uint32_t t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3], t4 = t[4];
                    acc[r][c][0] ^= gmul(s0, t0, t1, t2, t3, t4);
                    acc[r][c][1] ^= gmul(s1, t0, t1, t2, t3, t4);
                    acc[r][c][2] ^= gmul(s2, t0, t1, t2, t3, t4);
                    acc[r][c][3] ^= gmul(s3, t0, t1, t2, t3, t4);
                }
            }
        }
    }
}

template <int D, int RG, int G, int J0, int V>
struct VpSteps {
    __device__ static __forceinline__ void run(uint32_t (&acc)[RG][V][4], uint4 (&v)[2][G][V],
                                               const uint8_t* pbase, uint64_t cs, uint64_t x,
                                               cu32* in_idx, cu32* tab, uint32_t tab_stride) {
        constexpr int buf = (J0 / G) & 1;
        if constexpr (J0 + G < D) vp_load<D, G, J0 + G, V>(v[buf ^ 1], pbase, cs, x, in_idx);
        vp_mul<D, RG, G, J0, V>(acc, v[buf], tab, tab_stride);
        if constexpr (J0 + G < D)
            VpSteps<D, RG, G, J0 + G, V>::run(acc, v, pbase, cs, x, in_idx, tab, tab_stride);
    }
};

// apply_column<RG, true, ., V, true> for d == D.
template <int D, int RG, int G, int V>
__device__ __forceinline__ void vp_column(uint8_t* pbase, uint64_t cs, uint64_t x,
                                          uint32_t tab_stride, cu32* in_idx, cu32* out_idx,
                                          cu32* tab) {
    uint32_t acc[RG][V][4];
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int c = 0; c < V; ++c) acc[r][c][0] = acc[r][c][1] = acc[r][c][2] = acc[r][c][3] = 0u;
    uint4 v[2][G][V];
    vp_load<D, G, 0, V>(v[0], pbase, cs, x, in_idx);
    VpSteps<D, RG, G, 0, V>::run(acc, v, pbase, cs, x, in_idx, tab, tab_stride);
#pragma unroll
    for (int r = 0; r < RG; ++r) {
        uint8_t* dst = pbase + uint64_t(out_idx[r]) * cs + x;
#pragma unroll
        for (int c = 0; c < V; ++c)
            st16<true>(dst + c * kSpan,
                       make_uint4(acc[r][c][0], acc[r][c][1], acc[r][c][2], acc[r][c][3]));
    }
}

// apply_tile with d == D (aligned layout, non-temporal, two columns per lane): full steps take
// vp_column, the ragged end the byte path.
template <int D, int RG, int G>
__device__ __forceinline__ void apply_tile_cd(const ApplyParams& a, cu32* pat, uint32_t part,
                                              uint32_t tile, uint32_t n_out, uint32_t tile_bytes) {
    constexpr int V = 2;
    cu32* in_idx = pat + 1;
    cu32* out_idx = pat + 1 + D;
    cu32* tab = pat + 1 + D + n_out;
    const uint32_t tab_stride = n_out * kTabWords;
    uint8_t* pbase = a.base + uint64_t(part) * a.part_stride;
    const uint64_t len = a.len;
    const uint64_t cs = a.chunk_stride;
    const uint64_t t0 = uint64_t(tile) * tile_bytes;
    const uint64_t t1 = t0 + tile_bytes < len ? t0 + tile_bytes : len;
#pragma unroll 1
    for (uint64_t xb = t0; xb < t1; xb += kSpan * V) {  // block-uniform
        const uint64_t x = xb + uint64_t(threadIdx.x) * 16u;
        if (xb + kSpan * V <= len) {
            vp_column<D, RG, G, V>(pbase, cs, x, tab_stride, in_idx, out_idx, tab);
        } else {
#pragma unroll 1
            for (uint64_t xc = x; xc < t1 && xc < xb + kSpan * V; xc += kSpan)
                apply_column<RG, false, 4, 1, false>(pbase, cs, xc, len - xc, D, tab_stride,
                                                     in_idx, out_idx, tab);
        }
    }
}

// XCD-aware block order.  The dispatcher deals a grid's blocks to the 8 XCDs round-robin (block
// b to XCD b % 8), so in launch order neighbouring tiles of a part land on different XCDs and
// every XCD streams a slice of every part at once.  Renumbering so that XCD x runs the contiguous
// range [x*q + min(x, r), ...) of the n blocks (q = n / 8, r = n % 8: a bijection for any n)
// gives each XCD whole runs of parts instead.  For the 10-read / 4-write stream of an RS(10,4)
// encode with no GF work this lifts the chip from 5.72-5.74 to 6.26-6.27 TB/s
// (tools/ubench_stream.hip mode m, profiles/r3_full/ubench_mix.log).
constexpr uint32_t kXcds = 8;

__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
    const uint32_t x = b % kXcds, i = b / kXcds, q = n / kXcds, r = n % kXcds;
    return x * q + (x < r ? x : r) + i;
}

// grid.x = n_parts * tiles_per_part (one 16 KiB column tile of one part per block),
// grid.y = row groups of exactly RG output rows starting at row_base.  xcd: block order of
// xcd_block (else launch order).
template <int RG, bool VEC, int GROUP, int V, bool NT>
__global__ __launch_bounds__(kApplyThreads) void rs_apply_kernel(ApplyParams a,
                                                                 uint32_t tiles_per_part,
                                                                 uint32_t row_base, bool xcd,
                                                                 uint32_t tile_bytes) {
    const uint32_t bx = xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t lp = bx / tiles_per_part;
    const uint32_t tile = bx - lp * tiles_per_part;
    const uint32_t part = a.part_ids ? as_const(a.part_ids)[lp] : lp;
    cu32* pat = as_const(a.pat) + (a.part_pat ? as_const(a.part_pat)[lp] : 0u);
    apply_tile<RG, VEC, GROUP, V, NT>(a, pat, part, tile, a.n_rows, row_base + blockIdx.y * RG,
                                      tile_bytes);
}

// Reconstruct with mixed erasure counts in ONE launch: every listed part's pattern carries its
// own row count n_out (1..MAXRG, the record's first word); each block branches (block-uniformly)
// to the exact-RG body, so no row is predicated inside the inner loop.  MAXRG is the batch's
// largest row count rounded up to 2, 4 or 8 (host side): the kernel's register allocation is the
// widest body's, so a 2-erasure batch compiled for 8 rows would run at half the occupancy.
// CD > 0 (aligned non-temporal builds only): the batch's d equals CD (host-checked), every tile
// takes apply_tile_cd with loads CDG inputs ahead.
template <int RG, int MAXRG, typename F>
__device__ __forceinline__ void rg_dispatch(uint32_t n, F&& f) {
    if (n == RG) f(std::integral_constant<int, RG>{});
    else if constexpr (RG < MAXRG) rg_dispatch<RG + 1, MAXRG>(n, f);
    // n > MAXRG or 0: never listed -- the host routes n_out > 8 to row-group launches and checks
    // every listed record against the launch's row class (capi.cpp reconstruct_batch)
}

template <bool VEC, int GROUP, int V, bool NT, int MAXRG, int CD = 0, int CDG = 0>
__global__ __launch_bounds__(kApplyThreads) void rs_apply_var_kernel(ApplyParams a,
                                                                     uint32_t tiles_per_part,
                                                                     bool xcd, uint32_t tile_bytes) {
    const uint32_t bx = xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t lp = bx / tiles_per_part;
    const uint32_t tile = bx - lp * tiles_per_part;
    const uint32_t part = as_const(a.part_ids)[lp];
    cu32* pat = as_const(a.pat) + as_const(a.part_pat)[lp];
    rg_dispatch<1, MAXRG>(pat[0], [&](auto rg) {
        constexpr int RG = decltype(rg)::value;
        if constexpr (CD > 0) {
            static_assert(VEC && V == 2 && NT, "compile-time d: aligned non-temporal build");
            apply_tile_cd<CD, RG, CDG>(a, pat, part, tile, RG, tile_bytes);
        } else {
            apply_tile<RG, VEC, GROUP, V, NT>(a, pat, part, tile, RG, 0, tile_bytes);
        }
    });
}

// ------------------------------------------------------------------------------------------
// Bit-sliced encode for the common shapes: RS(d, p) with the parity rows compile-time constants.
//
// The v_perm multiply above costs, per data dword, 3 selector ops plus 3 half-rate v_perm and
// 2 xors per parity row: for RS(10,4) about 84 SIMD cycles per 64 data dwords, against ~39 for
// the HBM stream (the encode was co-bound).  Bit-sliced, the same multiply is a
// fixed XOR network: a lane's 32 bytes of one input (its two 16-byte columns) are transposed
// into 8 bit planes (plane i = bit i of all 32 bytes; 12 two-word bit swaps, 48 full-rate ops),
// output plane o of row r is the XOR of the input planes i with bit o of c[r][j]*2^i set
// (gf_const.hpp kBits, about half of them), and the 8 planes of each row are transposed back.
// With the matrix known at compile time the network is straight-line v_bitop3 xor3s: RS(10,4)
// ≈ 17 full-rate ops per data dword (6 transpose in, 9 xor, 2.4 transpose out), about half the
// v_perm form.  Loads and stores are the rs_apply ones (non-temporal, two 16-byte columns 4 KiB
// apart per lane, XCD-aware block order); ragged tails take the v_perm byte path.
// ------------------------------------------------------------------------------------------

// bitop3 select: m ? x : y per bit.
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t x, uint32_t y) {
    return __builtin_amdgcn_bitop3_b32(m, x, y, 0xCA);
}

// Swap bit k (k & S set) of a with bit k - S of b, in every byte.
template <int S>
__device__ __forceinline__ void swap_bits(uint32_t& a, uint32_t& b) {
    constexpr uint32_t lo = S == 1 ? 0x55555555u : S == 2 ? 0x33333333u : 0x0F0F0F0Fu;
    constexpr uint32_t hi = lo << S;
    const uint32_t na = bsel(hi, b << S, a);
    const uint32_t nb = bsel(lo, a >> S, b);
    a = na;
    b = nb;
}

// 8x8 bit transpose in each byte lane of 8 words: bit k of byte m of w[j] <-> bit j of byte m of
// w[k].  Each stage swaps one bit of the word index with the same bit of the bit index, so the
// three commute and the whole is an involution (the same network maps planes back to bytes).
__device__ __forceinline__ void transpose8(uint32_t (&w)[8]) {
    swap_bits<1>(w[0], w[1]);
    swap_bits<1>(w[2], w[3]);
    swap_bits<1>(w[4], w[5]);
    swap_bits<1>(w[6], w[7]);
    swap_bits<2>(w[0], w[2]);
    swap_bits<2>(w[1], w[3]);
    swap_bits<2>(w[4], w[6]);
    swap_bits<2>(w[5], w[7]);
    swap_bits<4>(w[0], w[4]);
    swap_bits<4>(w[1], w[5]);
    swap_bits<4>(w[2], w[6]);
    swap_bits<4>(w[3], w[7]);
}

constexpr int kBsGroup = 2;  // inputs per network step (terms pair across both into xor3s)

// Input words of inputs J0 .. J0 + kBsGroup: a lane's two 16-byte columns (x, x + kSpan).
template <int D, int J0>
__device__ __forceinline__ void bs_load(uint32_t (&w)[kBsGroup][8], const uint8_t* pbase,
                                        uint64_t cs, uint64_t x, cu32* in_idx) {
#pragma unroll
    for (int u = 0; u < kBsGroup; ++u) {
        if (J0 + u < D) {
            const uint8_t* src = pbase + uint64_t(in_idx[J0 + u]) * cs + x;
            const uint4 c0 = ld16<true>(src), c1 = ld16<true>(src + kSpan);
            w[u][0] = c0.x, w[u][1] = c0.y, w[u][2] = c0.z, w[u][3] = c0.w;
            w[u][4] = c1.x, w[u][5] = c1.y, w[u][6] = c1.z, w[u][7] = c1.w;
        }
    }
}

// acc[r][o] ^= the planes of inputs J0 .. J0 + kBsGroup that feed bit o of row r, two per xor3.
template <int D, int P, int J0>
__device__ __forceinline__ void bs_group(uint32_t (&acc)[P][8], uint32_t (&w)[kBsGroup][8]) {
    using S = gfc::Shape<D, P>;
#pragma unroll
    for (int u = 0; u < kBsGroup; ++u)
        if (J0 + u < D) transpose8(w[u]);
#pragma unroll
    for (int r = 0; r < P; ++r) {
#pragma unroll
        for (int o = 0; o < 8; ++o) {
            uint32_t pend = 0;
            bool has = false;
#pragma unroll
            for (int u = 0; u < kBsGroup; ++u) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if (J0 + u < D && ((S::kBits.m[r][J0 + u < D ? J0 + u : 0][o] >> i) & 1)) {
                        if (has) {
                            acc[r][o] = xor3(acc[r][o], pend, w[u][i]);
                            has = false;
                        } else {
                            pend = w[u][i];
                            has = true;
                        }
                    }
                }
            }
            if (has) acc[r][o] ^= pend;
        }
    }
}

// Groups J0, J0 + kBsGroup, ... with the next group's loads issued before this group's network.
template <int D, int P, int J0>
struct BsSteps {
    __device__ static __forceinline__ void run(uint32_t (&acc)[P][8],
                                               uint32_t (&w)[2][kBsGroup][8],
                                               const uint8_t* pbase, uint64_t cs, uint64_t x,
                                               cu32* in_idx) {
        constexpr int buf = (J0 / kBsGroup) & 1;
        if constexpr (J0 + kBsGroup < D) bs_load<D, J0 + kBsGroup>(w[buf ^ 1], pbase, cs, x, in_idx);
        bs_group<D, P, J0>(acc, w[buf]);
        if constexpr (J0 + kBsGroup < D)
            BsSteps<D, P, J0 + kBsGroup>::run(acc, w, pbase, cs, x, in_idx);
    }
};

// Two full 16-byte columns (x, x + kSpan) of every parity row of one part.
template <int D, int P>
__device__ __forceinline__ void bs_column(uint8_t* pbase, uint64_t cs, uint64_t x, cu32* in_idx,
                                          cu32* out_idx) {
    uint32_t acc[P][8];
#pragma unroll
    for (int r = 0; r < P; ++r)
#pragma unroll
        for (int o = 0; o < 8; ++o) acc[r][o] = 0u;
    uint32_t w[2][kBsGroup][8];
    bs_load<D, 0>(w[0], pbase, cs, x, in_idx);
    BsSteps<D, P, 0>::run(acc, w, pbase, cs, x, in_idx);
#pragma unroll
    for (int r = 0; r < P; ++r) {
        transpose8(acc[r]);
        uint8_t* dst = pbase + uint64_t(out_idx[r]) * cs + x;
        st16<true>(dst, make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]));
        st16<true>(dst + kSpan, make_uint4(acc[r][4], acc[r][5], acc[r][6], acc[r][7]));
    }
}

// grid.x = n_parts * tiles_per_part, as rs_apply_kernel; the pattern record is the codec's
// encode record (its indices; its v_perm tables serve the ragged tail).  The host launches this
// only for 16-byte aligned layouts whose run-time matrix equals gfc::Shape<D, P> (checked once
// per codec, bs_encode_matches).
template <int D, int P>
__global__ __launch_bounds__(kApplyThreads) void rs_encode_bs_kernel(ApplyParams a,
                                                                     uint32_t tiles_per_part,
                                                                     bool xcd, uint32_t tile_bytes) {
    const uint32_t bx = xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t lp = bx / tiles_per_part;
    const uint32_t tile = bx - lp * tiles_per_part;
    const uint32_t part = a.part_ids ? as_const(a.part_ids)[lp] : lp;
    cu32* pat = as_const(a.pat);
    cu32* in_idx = pat + 1;
    cu32* out_idx = pat + 1 + D;
    cu32* tab = pat + 1 + D + P;
    uint8_t* pbase = a.base + uint64_t(part) * a.part_stride;
    const uint64_t len = a.len;
    const uint64_t cs = a.chunk_stride;
    const uint64_t t0 = uint64_t(tile) * tile_bytes;
    const uint64_t t1 = t0 + tile_bytes < len ? t0 + tile_bytes : len;
#pragma unroll 1
    for (uint64_t xb = t0; xb < t1; xb += 2 * kSpan) {  // block-uniform
        const uint64_t x = xb + uint64_t(threadIdx.x) * 16u;
        if (xb + 2 * kSpan <= len) {
            bs_column<D, P>(pbase, cs, x, in_idx, out_idx);
        } else {
#pragma unroll 1
            for (uint64_t xc = x; xc < t1 && xc < xb + 2 * kSpan; xc += kSpan)
                apply_column<P, false, 4, 1, false>(pbase, cs, xc, len - xc, D, P * kTabWords,
                                                    in_idx, out_idx, tab);
        }
    }
}

// ------------------------------------------------------------------------------------------
// Synthetic data
// ------------------------------------------------------------------------------------------

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

__host__ __device__ __forceinline__ uint64_t synth_key(uint64_t seed, uint64_t part,
                                                       uint64_t chunk) {
    return mix64(seed ^ mix64(part * 0x100000001B3ull + chunk + 0x9E3779B97F4A7C15ull));
}

__host__ __device__ __forceinline__ uint64_t synth_word(uint64_t key, uint64_t word) {
    return mix64(key + word * 0x9E3779B97F4A7C15ull);
}

__global__ __launch_bounds__(256) void fill_kernel(FillParams a, bool aligned8) {
    const uint64_t words = (a.len + 7) / 8;
    const uint64_t n_inst = uint64_t(a.n_parts) * a.n_chunks;
    for (uint64_t inst = blockIdx.y; inst < n_inst; inst += gridDim.y) {
        const uint64_t k = inst / a.n_chunks;
        const uint64_t c = inst - k * a.n_chunks;
        const uint64_t key = synth_key(a.seed, k, c);
        uint8_t* dst = a.base + k * a.part_stride + c * a.chunk_stride;
        for (uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w < words;
             w += uint64_t(gridDim.x) * blockDim.x) {
            const uint64_t v = synth_word(key, w);
            const uint64_t off = w * 8;
            if (aligned8 && off + 8 <= a.len) {
                *reinterpret_cast<uint64_t*>(dst + off) = v;
            } else {
                for (int b = 0; b < 8; ++b)
                    if (off + b < a.len) dst[off + b] = uint8_t(v >> (8 * b));
            }
        }
    }
}

// CEC_APPLY_TUNE (tuning knob, latched once: knobs.hpp; unset = "nt"): "nt" = non-temporal loads and
// stores, "v1" = one 16-byte column per lane per step instead of two, "g8" = 8 inputs in
// flight per lane instead of 4; any other string = plain loads, two columns, groups of 4.
// Measured on C2 encode (tools/apply_ab.py, MI355X): nt 10.79 ms, plain 11.20, v1 11.25,
// v1+nt 11.15, g8 11.26, nt+g8 10.85.
int apply_tune() { return knobs().apply_tune; }

// CEC_APPLY_XCD (A/B knob; unset = 1): 0 launches the apply kernels' blocks in
// plain launch order instead of the XCD-aware order (xcd_block).
bool apply_xcd() { return knobs().apply_xcd; }

// LDS of one CU on the current device, cached per device: 160 KiB on gfx950 (MI355X), else
// what the runtime reports (hipDeviceAttributeMaxSharedMemoryPerMultiprocessor); 0 when
// unknown, which turns the residency caps below off rather than mis-sizing them.
uint32_t lds_per_cu() {
    static std::atomic<uint32_t> cache[64];  // 0 = not read yet, 1 = unknown
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return 0;
    }
    uint32_t v = cache[dev].load(std::memory_order_relaxed);
    if (!v) {
        hipDeviceProp_t prop;
        int attr = 0;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess &&
            std::strncmp(prop.gcnArchName, "gfx950", 6) == 0)
            v = 160u * 1024u;
        else if (hipDeviceGetAttribute(&attr, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor,
                                       dev) == hipSuccess && attr > 0)
            v = uint32_t(attr);
        else
            v = 1;
        (void)hipGetLastError();
        cache[dev].store(v, std::memory_order_relaxed);
    }
    return v == 1 ? 0 : v;
}

// Residency cap.  The GF kernels stream 10-28 chunks per part 1 MiB (chunk stride) apart, and on
// MI355X they run faster with FEWER blocks in flight than their registers allow: interleaved on
// one box (profiles/r3_occ_ab/), RS(10,4) bit-sliced encode 9.53 ms at 2 blocks (= waves per
// SIMD) per CU vs 9.88 at its register-bound 6; 2-erasure reconstruct_data 8.11 at 2 vs 8.26 at
// 3 (the 8-row build) and 8.57 at 6 (the 2-row build); C3 (1-4 rows) 9.58 at 3 vs 10.15 at 2;
// RS(20,8) encode no different (3 by registers).  The cap is an unused LDS reservation (160 KiB
// per CU), on top of any the caller asked for, and only for grids of at least kCapMinBlocks
// blocks (the device-resident batches it was measured on; the host pipelines' 256-part batches
// share the chip with SHA-256 kernels and keep the register-bound occupancy).
// CEC_APPLY_BLOCKS_PER_CU (A/B knob): n > 0 caps every apply launch at n blocks
// per CU, 0 turns the cap off; unset = the per-kernel default `def_cap` (0 = none).
constexpr uint64_t kCapMinBlocks = 65536;
uint32_t apply_lds(uint32_t reserve, int def_cap, uint64_t n_blocks) {
    const int knob = knobs().apply_blocks_per_cu;
    const int n = knob >= 0 ? knob : (n_blocks >= kCapMinBlocks ? def_cap : 0);
    const uint32_t cu_lds = lds_per_cu();
    if (n <= 0 || n > 16 || cu_lds == 0) return reserve;
    // floor(cu_lds / lds) == n; a cap the part's LDS cannot express (lds above the per-launch
    // maximum, 64 KiB parts at n = 1) is dropped rather than failing the launch
    const uint32_t lds = cu_lds / uint32_t(n + 1) + 2048u;
    if (lds > cu_lds) return reserve;
    return std::max(reserve, lds);
}

// CEC_APPLY_RGCLS (A/B knob; unset = 1): 0 runs every reconstruct batch on the
// var kernel compiled for 8 rows instead of the batch's row class (2, 4 or 8).
bool apply_rg_classes() { return knobs().apply_rg_classes; }

// CEC_APPLY_CD (A/B knob; unset = 1): for d == 10 reconstruct batches, the
// compile-time-d var kernel (apply_tile_cd, loads 5 inputs ahead); 0 = the run-time-d kernel.
// Interleaved on one box with the residency caps (profiles/r3_cap_ab/): c3e2 8.07-8.09 vs
// 8.12-8.14 ms, C3 9.64-9.68 vs 9.71-9.75 (groups of 2 and 10 measured the same as 5 without
// the caps, profiles/r3_cd_ab/).
bool apply_cd() { return knobs().apply_cd; }

// CEC_APPLY_TILE (A/B knob): bytes of one part's column range per block, a
// multiple of 8 KiB (one full two-column step of a block) up to 256 KiB; default `def`:
// kApplyTile for rs_apply_kernel, kBsTile for the bit-sliced encoder and the mixed-pattern
// reconstruct.  Measured interleaved on one box with the residency caps
// (profiles/r3_tilecap_ab/, 8 / 16 / 32 KiB): RS(10,4) bit-sliced encode 9.46 / 9.72 / 9.86 ms,
// c3e2 7.89 / 7.96 / 8.39, C3 9.20 / 9.35 / 9.61.  (Without the caps C3 had preferred 16 KiB,
// profiles/r3_tile2_ab/.)
constexpr uint64_t kBsTile = 8192;
uint64_t apply_tile_bytes(uint64_t def = kApplyTile) {
    const uint64_t v = knobs().apply_tile;
    return v && v % 8192 == 0 && v <= (256u << 10) ? v : def;
}

// Launch KERNEL<PRE... VEC, GROUP, V, NT> as picked by the tuning knob; layouts that are not
// 16-byte aligned take the byte-granular instantiation.
template <typename Launch>
hipError_t dispatch_apply(bool vec16, Launch&& go) {
    if (!vec16) return go(std::integral_constant<int, -1>{});
    switch (apply_tune()) {
        case 1: return go(std::integral_constant<int, 1>{});
        case 2: return go(std::integral_constant<int, 2>{});
        case 3: return go(std::integral_constant<int, 3>{});
        case 4: return go(std::integral_constant<int, 4>{});
        case 5: return go(std::integral_constant<int, 5>{});
        default: return go(std::integral_constant<int, 0>{});
    }
}

// tune code -> template arguments
template <int K> struct Tune {
    static constexpr bool kVec = K >= 0;
    static constexpr int kGroup = K >= 0 && (K & 2) ? 8 : 4;
    static constexpr int kV = K < 0 || (K & 4) ? 1 : 2;
    static constexpr bool kNt = K >= 0 && (K & 1);
};

// Lets `kernel` reserve `bytes` of dynamic LDS (a host-side attribute; set on every such launch,
// since the instantiations share one function-pointer type).
template <typename K>
bool allow_lds(K kernel, uint32_t bytes) {
    return bytes <= 64 * 1024 ||
           hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes)) == hipSuccess;
}

// A dispatch's grid is at most 2^32 - 1 work-items (the AQL packet's 32-bit grid size): with
// kApplyThreads per block, at most this many blocks.  Larger batches (many parts of long chunks,
// e.g. 4096 x 64 MiB) are split over several launches of whole parts.
constexpr uint64_t kMaxApplyBlocks = 0xFFFFFFFFull / kApplyThreads;
// CEC_APPLY_MAX_BLOCKS (test knob) lowers the limit so the split is exercised
// at test sizes; results are identical either way.
uint64_t max_apply_blocks() {
    const uint64_t v = knobs().apply_max_blocks;
    return v ? std::min<uint64_t>(v, kMaxApplyBlocks) : kMaxApplyBlocks;
}

// fn(sub) for launches of at most max_parts parts each: part ranges [p0, p0 + n) as a base
// offset (parts addressed directly) or as offsets into the listed part_ids / part_pat.
template <typename Fn>
hipError_t for_part_ranges(const ApplyParams& a, uint64_t max_parts, Fn fn) {
    for (uint64_t p0 = 0; p0 < a.n_parts; p0 += max_parts) {
        ApplyParams b = a;
        b.n_parts = uint32_t(std::min<uint64_t>(max_parts, a.n_parts - p0));
        if (a.part_ids) {
            b.part_ids = a.part_ids + p0;
            if (a.part_pat) b.part_pat = a.part_pat + p0;
        } else {
            b.base = a.base + p0 * a.part_stride;
        }
        const hipError_t e = fn(b);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int RG>
hipError_t launch_rg(const ApplyParams& a, uint32_t row_base, uint32_t groups, bool vec16,
                     hipStream_t s) {
    const uint64_t tb = apply_tile_bytes();
    const uint64_t tiles = (a.len + tb - 1) / tb;
    const uint64_t max_blocks = max_apply_blocks();
    if (tiles > max_blocks) return hipErrorInvalidValue;
    return for_part_ranges(a, max_blocks / tiles, [&](const ApplyParams& b) {
        const dim3 grid(uint32_t(b.n_parts * tiles), groups);
        return dispatch_apply(vec16, [&](auto k) {
            using T = Tune<decltype(k)::value>;
            auto* kern = &rs_apply_kernel<RG, T::kVec, T::kGroup, T::kV, T::kNt>;
            // 1-3 rows: 3 blocks per CU (RS(2,1) / RS(4,2) / RS(8,2) / RS(6,3) encode 1-2 %
            // faster than by registers, profiles/r3_vperm_shapes_ab/); 4+ rows: no gain
            const uint32_t lds =
                apply_lds(b.lds_reserve, RG <= 3 ? 3 : 0, uint64_t(grid.x) * groups);
            if (!allow_lds(kern, lds)) return hipErrorInvalidValue;
            clear_stale_error();
            hipLaunchKernelGGL(kern, grid, dim3(kApplyThreads), lds, s, b,
                               uint32_t(tiles), row_base, apply_xcd(), uint32_t(tb));
            return hipGetLastError();
        });
    });
}

hipError_t launch_rows(const ApplyParams& a, uint32_t rg, uint32_t row_base, uint32_t groups,
                       bool vec16, hipStream_t s) {
    switch (rg) {
        case 1: return launch_rg<1>(a, row_base, groups, vec16, s);
        case 2: return launch_rg<2>(a, row_base, groups, vec16, s);
        case 3: return launch_rg<3>(a, row_base, groups, vec16, s);
        case 4: return launch_rg<4>(a, row_base, groups, vec16, s);
        case 5: return launch_rg<5>(a, row_base, groups, vec16, s);
        case 6: return launch_rg<6>(a, row_base, groups, vec16, s);
        case 7: return launch_rg<7>(a, row_base, groups, vec16, s);
        default: return launch_rg<8>(a, row_base, groups, vec16, s);
    }
}

// CEC_APPLY_BS (A/B knob; unset = 1): 0 sends the compiled shapes' encodes to
// the v_perm kernel too.
bool apply_bs() { return knobs().apply_bs; }

template <int D, int P>
hipError_t launch_bs(const ApplyParams& a, hipStream_t s) {
    const uint64_t tb = apply_tile_bytes(kBsTile);
    const uint64_t tiles = (a.len + tb - 1) / tb;
    const uint64_t max_blocks = max_apply_blocks();
    if (tiles > max_blocks) return hipErrorInvalidValue;
    return for_part_ranges(a, max_blocks / tiles, [&](const ApplyParams& b) {
        auto* kern = &rs_encode_bs_kernel<D, P>;
        const uint64_t n_blocks = b.n_parts * tiles;
        // measured per shape: RS(10,4) 2 blocks per CU, RS(3,2) 3 (6.71 vs 6.92-7.23 ms for 8 192
        // parts x 1 MiB, profiles/r3_c1enc_ab/), RS(20,8) its register-bound 3
        const int cap = D == 10 && P == 4 ? 2 : D == 3 && P == 2 ? 3 : 0;
        const uint32_t lds = apply_lds(b.lds_reserve, cap, n_blocks);
        if (!allow_lds(kern, lds)) return hipErrorInvalidValue;
        clear_stale_error();
        hipLaunchKernelGGL(kern, dim3(uint32_t(n_blocks)), dim3(kApplyThreads), lds, s, b,
                           uint32_t(tiles), apply_xcd(), uint32_t(tb));
        return hipGetLastError();
    });
}

// The compiled bit-sliced shapes: the reference's example clusters (RS(3,2), examples/*.yaml)
// and the bench configurations (RS(10,4), RS(20,8)).
template <typename Fn>
bool with_bs_shape(uint32_t d, uint32_t p, Fn&& fn) {
    if (d == 3 && p == 2) return fn(gfc::Shape<3, 2>{}, std::integral_constant<int, 3>{},
                                    std::integral_constant<int, 2>{});
    if (d == 10 && p == 4) return fn(gfc::Shape<10, 4>{}, std::integral_constant<int, 10>{},
                                     std::integral_constant<int, 4>{});
    if (d == 20 && p == 8) return fn(gfc::Shape<20, 8>{}, std::integral_constant<int, 20>{},
                                     std::integral_constant<int, 8>{});
    return false;
}

}  // namespace

bool bs_encode_matches(uint32_t d, uint32_t p, const uint8_t* parity_rows) {
    return with_bs_shape(d, p, [&](auto shape, auto, auto) {
        using S = decltype(shape);
        for (uint32_t r = 0; r < p; ++r)
            for (uint32_t j = 0; j < d; ++j)
                if (S::kMat.c[r][j] != parity_rows[r * d + j]) return false;
        return true;
    });
}

hipError_t launch_rs_encode(const ApplyParams& a, bool vec16, hipStream_t s) {
    if (a.n_parts == 0 || a.n_rows == 0 || a.len == 0) return hipSuccess;
    if (a.std_encode && vec16 && !a.part_pat && apply_bs()) {
        hipError_t e = hipErrorInvalidValue;
        const bool shaped = with_bs_shape(a.d, a.n_rows, [&](auto, auto dd, auto pp) {
            e = launch_bs<decltype(dd)::value, decltype(pp)::value>(a, s);
            return true;
        });
        if (shaped) return e;
    }
    return launch_rs_apply(a, vec16, s);
}

// Rows are processed in groups of kMaxApplyRows (8) plus one remainder group, so every kernel
// instance handles exactly RG rows (no per-row predicate in the inner loop).
hipError_t launch_rs_apply(const ApplyParams& a, bool vec16, hipStream_t s) {
    if (a.n_parts == 0 || a.n_rows == 0 || a.len == 0) return hipSuccess;
    const uint32_t full = a.n_rows / kMaxApplyRows, rem = a.n_rows % kMaxApplyRows;
    if (full) {
        hipError_t e = launch_rows(a, kMaxApplyRows, 0, full, vec16, s);
        if (e != hipSuccess) return e;
    }
    if (rem) return launch_rows(a, rem, full * kMaxApplyRows, 1, vec16, s);
    return hipSuccess;
}

// Listed parts (part_ids / part_pat) whose patterns have 1..kMaxApplyRows rows each: one launch.
// a.n_rows = the largest row count in the batch (0: unknown, up to kMaxApplyRows).
hipError_t launch_rs_apply_var(const ApplyParams& a, bool vec16, hipStream_t s) {
    if (a.n_parts == 0 || a.len == 0) return hipSuccess;
    if (!a.part_ids || !a.part_pat) return hipErrorInvalidValue;
    if (a.n_rows > kMaxApplyRows) return hipErrorInvalidValue;
    const uint64_t tb = apply_tile_bytes(kBsTile);  // 8 KiB with the caps (see kBsTile)
    const uint64_t tiles = (a.len + tb - 1) / tb;
    const uint64_t max_blocks = max_apply_blocks();
    if (tiles > max_blocks) return hipErrorInvalidValue;
    // not under a caller's LDS reservation: the read path's decode beside the SHA-256
    // verification (capi.cpp decode_lds) loses with it (c3r 44.0-44.5 vs 42.6-42.8 ms,
    // profiles/r3_c3r_ab/): its loads run ahead into the SHA chains' bandwidth
    const bool cd = apply_cd() && a.lds_reserve == 0;
    const uint32_t rows = a.n_rows ? a.n_rows : kMaxApplyRows;
    const int cls = !apply_rg_classes() ? 8 : rows <= 2 ? 2 : rows <= 4 ? 4 : 8;  // MAXRG
    return for_part_ranges(a, max_blocks / tiles, [&](const ApplyParams& b) {
        const dim3 grid(uint32_t(b.n_parts * tiles));
        // 2-row class: 2 blocks per CU, 4-row class: 3, 8-row: by registers (3)
        const uint32_t lds = apply_lds(b.lds_reserve, cls == 2 ? 2 : cls == 4 ? 3 : 0, grid.x);
        auto go = [&](auto* kern) {
            if (!allow_lds(kern, lds)) return hipErrorInvalidValue;
            clear_stale_error();
            hipLaunchKernelGGL(kern, grid, dim3(kApplyThreads), lds, s, b,
                               uint32_t(tiles), apply_xcd(), uint32_t(tb));
            return hipGetLastError();
        };
        auto by_class = [&](auto k2, auto k4, auto k8) {
            return cls == 2 ? go(k2) : cls == 4 ? go(k4) : go(k8);
        };
        if (vec16 && apply_tune() == 1 && b.d == 10 && cd)
            return by_class(&rs_apply_var_kernel<true, 4, 2, true, 2, 10, 5>,
                            &rs_apply_var_kernel<true, 4, 2, true, 4, 10, 5>,
                            &rs_apply_var_kernel<true, 4, 2, true, 8, 10, 5>);
        return dispatch_apply(vec16, [&](auto k) {
            using T = Tune<decltype(k)::value>;
            // the default build (nt) and the byte-granular one get the row classes; the other
            // tuning codes are A/B builds at the full 8 rows
            constexpr bool classes = decltype(k)::value == 1 || decltype(k)::value == -1;
            if constexpr (classes)
                return by_class(&rs_apply_var_kernel<T::kVec, T::kGroup, T::kV, T::kNt, 2>,
                                &rs_apply_var_kernel<T::kVec, T::kGroup, T::kV, T::kNt, 4>,
                                &rs_apply_var_kernel<T::kVec, T::kGroup, T::kV, T::kNt, 8>);
            else
                return go(&rs_apply_var_kernel<T::kVec, T::kGroup, T::kV, T::kNt, 8>);
        });
    });
}

uint32_t max_var_rows() { return kMaxApplyRows; }


hipError_t launch_fill(const FillParams& a, hipStream_t s) {
    const uint64_t n_inst = uint64_t(a.n_parts) * a.n_chunks;
    if (n_inst == 0 || a.len == 0) return hipSuccess;
    const uint64_t words = (a.len + 7) / 8;
    uint32_t gx = uint32_t(std::min<uint64_t>((words + 255) / 256, 64));
    uint32_t gy = uint32_t(std::min<uint64_t>(n_inst, 65535));
    const bool aligned8 = (reinterpret_cast<uintptr_t>(a.base) % 8 == 0) &&
                          (a.part_stride % 8 == 0) && (a.chunk_stride % 8 == 0);
    clear_stale_error();
    hipLaunchKernelGGL(fill_kernel, dim3(gx, gy), dim3(256), 0, s, a, aligned8);
    return hipGetLastError();
}

uint8_t synth_byte(uint64_t seed, uint64_t part, uint64_t chunk, uint64_t offset) {
    const uint64_t v = synth_word(synth_key(seed, part, chunk), offset / 8);
    return uint8_t(v >> (8 * (offset % 8)));
}

}  // namespace cec
