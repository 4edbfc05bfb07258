// Host check of the bit-sliced encoder's design (rs_encode_bs_kernel, rs_kernels.hip), no GPU:
//  1. gf_const.hpp's compile-time parity rows equal the run-time builder's (gf256.cpp) for every
//     compiled shape, and its bit matrices reproduce the field multiply for all 256 x values;
//  2. the kernel's data path restated on the host with plain integer ops (the 8x8 bit transpose
//     by three swap stages, the XOR network over kBits, the transpose back) gives byte for byte
//     the direct GF(2^8) encode of random 32-byte lane slices.
// The GPU tests compare the kernel itself with the oracle; this pins the construction it rests on.
// Build: g++ -std=c++17 -O2 -I<csrc> bitslice_check.cpp <csrc>/gf256.cpp
#include <cstdint>
#include <cstdio>
#include <random>

#include "gf256.hpp"
#include "gf_const.hpp"

namespace {

int failures = 0;

void fail(const char* what, int d, int p, int a, int b) {
    if (failures++ < 20) std::printf("FAIL %s RS(%d,%d) at %d,%d\n", what, d, p, a, b);
}

template <int S>
void swap_bits(uint32_t& a, uint32_t& b) {
    constexpr uint32_t lo = S == 1 ? 0x55555555u : S == 2 ? 0x33333333u : 0x0F0F0F0Fu;
    constexpr uint32_t hi = lo << S;
    const uint32_t na = (hi & (b << S)) | (~hi & a);
    const uint32_t nb = (lo & (a >> S)) | (~lo & b);
    a = na;
    b = nb;
}

void transpose8(uint32_t (&w)[8]) {
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

template <int D, int P>
void check_shape(std::mt19937_64& rng) {
    using S = cec::gfc::Shape<D, P>;
    const cec::Gf256& g = cec::Gf256::get();
    const cec::ByteMatrix m = cec::build_coding_matrix(D, P);
    for (int r = 0; r < P; ++r)
        for (int j = 0; j < D; ++j)
            if (S::kMat.c[r][j] != m.at(D + r, j)) fail("matrix", D, P, r, j);
    for (int r = 0; r < P; ++r)
        for (int j = 0; j < D; ++j)
            for (int x = 0; x < 256; ++x) {
                uint8_t y = 0;
                for (int o = 0; o < 8; ++o) {
                    int bit = 0;
                    for (int i = 0; i < 8; ++i)
                        if ((S::kBits.m[r][j][o] >> i) & 1) bit ^= (x >> i) & 1;
                    y = uint8_t(y | (bit << o));
                }
                if (y != g.mul(S::kMat.c[r][j], uint8_t(x))) fail("bit matrix", D, P, r * D + j, x);
            }
    // a lane's slice: 32 bytes (two 16-byte columns) of each of D inputs
    for (int trial = 0; trial < 200; ++trial) {
        uint32_t in[D][8];
        for (int j = 0; j < D; ++j)
            for (int k = 0; k < 8; ++k) in[j][k] = uint32_t(rng());
        if (trial == 0)
            for (int j = 0; j < D; ++j)
                for (int k = 0; k < 8; ++k) in[j][k] = 0xFFFFFFFFu;
        uint32_t acc[P][8] = {};
        for (int j = 0; j < D; ++j) {
            uint32_t w[8];
            for (int k = 0; k < 8; ++k) w[k] = in[j][k];
            transpose8(w);
            for (int r = 0; r < P; ++r)
                for (int o = 0; o < 8; ++o)
                    for (int i = 0; i < 8; ++i)
                        if ((S::kBits.m[r][j][o] >> i) & 1) acc[r][o] ^= w[i];
        }
        for (int r = 0; r < P; ++r) {
            transpose8(acc[r]);
            for (int k = 0; k < 32; ++k) {
                uint8_t want = 0;
                for (int j = 0; j < D; ++j)
                    want ^= g.mul(S::kMat.c[r][j], uint8_t(in[j][k / 4] >> (8 * (k % 4))));
                const uint8_t got = uint8_t(acc[r][k / 4] >> (8 * (k % 4)));
                if (got != want) fail("network", D, P, r, k);
            }
        }
    }
}

}  // namespace

template <int D, int P>
void print_shape() {
    using S = cec::gfc::Shape<D, P>;
    std::printf("%d %d", D, P);
    for (int r = 0; r < P; ++r)
        for (int j = 0; j < D; ++j) std::printf(" %d", S::kMat.c[r][j]);
    std::printf("\n");
}

int main(int argc, char** argv) {
    if (argc > 1) {  // --print: the compiled shapes' parity rows, one shape per line
        print_shape<3, 2>();
        print_shape<10, 4>();
        print_shape<20, 8>();
        return 0;
    }
    std::mt19937_64 rng(20261017);
    check_shape<3, 2>(rng);
    check_shape<10, 4>(rng);
    check_shape<20, 8>(rng);
    check_shape<1, 1>(rng);
    check_shape<5, 5>(rng);
    if (failures) {
        std::printf("%d failures\n", failures);
        return 1;
    }
    std::printf("ok\n");
    return 0;
}
