// gf_const.hpp — compile-time GF(2^8) and encode matrices for the bit-sliced encoder.
//
// The same field and construction as gf256.cpp (reed_solomon_erasure 4.0.2 / galois_8:
// polynomial 0x11D, generator 2, M = V * inv(V[0..d]) with V[r][c] = galois_8::exp(r, c)), but
// evaluated by the compiler, so the parity rows of a given RS(d, p) are constants of the kernel
// that encodes it.  Used on the host too: the launcher only takes the bit-sliced kernel when the
// codec's run-time matrix equals this one byte for byte (bs_encode_matches in rs_kernels.hip).
//
// Bit matrices.  Multiplication by a constant c is GF(2)-linear in the bits of x:
//     bit o of c*x = XOR over i of  x_i & (bit o of c*2^i)
// so for a coefficient c, kBits[o] is the 8-bit mask of the input bits i that feed output bit o.
#pragma once

#include <cstdint>

namespace cec {
namespace gfc {

struct Tables {
    uint8_t exp[512];
    uint8_t log[256];
};

constexpr Tables make_tables() {
    Tables t{};
    unsigned x = 1;
    for (unsigned i = 0; i < 255; ++i) {
        t.exp[i] = uint8_t(x);
        t.exp[i + 255] = uint8_t(x);
        t.log[x] = uint8_t(i);
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    return t;
}

inline constexpr Tables kTables = make_tables();

constexpr uint8_t mul(uint8_t a, uint8_t b) {
    return (a == 0 || b == 0) ? 0 : kTables.exp[kTables.log[a] + kTables.log[b]];
}

constexpr uint8_t inv(uint8_t a) {  // a != 0
    return kTables.exp[(255 - kTables.log[a]) % 255];
}

// galois_8::exp(a, n): 1 for n == 0, 0 for a == 0, else a^n.
constexpr uint8_t pow(uint8_t a, unsigned n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return kTables.exp[(unsigned(kTables.log[a]) * n) % 255];
}

template <int D, int P>
struct EncodeMatrix {
    uint8_t c[P][D];  // parity row r, data input j
};

// Parity rows of the systematic coding matrix M = V * inv(V_top).
template <int D, int P>
constexpr EncodeMatrix<D, P> encode_matrix() {
    uint8_t w[D][2 * D] = {};  // [V_top | I], Gauss-Jordan to [I | inv(V_top)]
    for (int r = 0; r < D; ++r) {
        for (int c = 0; c < D; ++c) w[r][c] = pow(uint8_t(r), unsigned(c));
        w[r][D + r] = 1;
    }
    for (int col = 0; col < D; ++col) {
        int piv = col;
        while (w[piv][col] == 0) ++piv;  // V_top is invertible (distinct points 0..d-1)
        if (piv != col)
            for (int c = 0; c < 2 * D; ++c) {
                const uint8_t t = w[piv][c];
                w[piv][c] = w[col][c];
                w[col][c] = t;
            }
        const uint8_t s = inv(w[col][col]);
        for (int c = 0; c < 2 * D; ++c) w[col][c] = mul(s, w[col][c]);
        for (int r = 0; r < D; ++r) {
            if (r == col || w[r][col] == 0) continue;
            const uint8_t f = w[r][col];
            for (int c = 0; c < 2 * D; ++c) w[r][c] ^= mul(f, w[col][c]);
        }
    }
    EncodeMatrix<D, P> m{};
    for (int r = 0; r < P; ++r)
        for (int j = 0; j < D; ++j) {
            uint8_t acc = 0;
            for (int k = 0; k < D; ++k) acc ^= mul(pow(uint8_t(D + r), unsigned(k)), w[k][D + j]);
            m.c[r][j] = acc;
        }
    return m;
}

template <int D, int P>
struct BitMatrices {
    uint8_t m[P][D][8];  // [row][input][output bit] = mask of the input bits feeding it
};

template <int D, int P>
constexpr BitMatrices<D, P> bit_matrices() {
    const EncodeMatrix<D, P> e = encode_matrix<D, P>();
    BitMatrices<D, P> b{};
    for (int r = 0; r < P; ++r)
        for (int j = 0; j < D; ++j)
            for (int i = 0; i < 8; ++i) {
                const uint8_t col = mul(e.c[r][j], uint8_t(1u << i));
                for (int o = 0; o < 8; ++o)
                    if ((col >> o) & 1) b.m[r][j][o] = uint8_t(b.m[r][j][o] | (1u << i));
            }
    return b;
}

template <int D, int P>
struct Shape {
    static constexpr EncodeMatrix<D, P> kMat = encode_matrix<D, P>();
    static constexpr BitMatrices<D, P> kBits = bit_matrices<D, P>();
};

}  // namespace gfc
}  // namespace cec
