// gf256.hpp — host-side GF(2^8) arithmetic and coding-matrix construction for the engine.
//
// Field and matrix are those of reed_solomon_erasure 4.0.2 / galois_8 (the crate
// the reference builds at src/file/file_part.rs:77 and src/file/writer.rs:131): generating
// polynomial 0x11D, generator 2, coding matrix M = V * inv(V[0..d]) with V[r][c] = r^c.
// Only tiny d x d matrices are handled here (construction, decode-submatrix inversion, and the
// packing of coefficients into the v_perm_b32 lookup tables the gfx950 kernels consume); every
// byte of shard data is processed on the GPU.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace cec {

struct Gf256 {
    uint8_t log[256];
    uint8_t exp[512];

    Gf256();
    uint8_t mul(uint8_t a, uint8_t b) const {
        return (a == 0 || b == 0) ? 0 : exp[log[a] + log[b]];
    }
    uint8_t div(uint8_t a, uint8_t b) const;  // b != 0
    uint8_t pow(uint8_t a, size_t n) const;   // crate galois_8::exp semantics
    static const Gf256& get();
};

// Row-major byte matrix.
struct ByteMatrix {
    size_t rows = 0, cols = 0;
    std::vector<uint8_t> v;
    ByteMatrix() = default;
    ByteMatrix(size_t r, size_t c) : rows(r), cols(c), v(r * c, 0) {}
    uint8_t& at(size_t r, size_t c) { return v[r * cols + c]; }
    uint8_t at(size_t r, size_t c) const { return v[r * cols + c]; }
};

// (d+p) x d systematic coding matrix.
ByteMatrix build_coding_matrix(size_t d, size_t p);
// Gauss-Jordan inverse; returns false if singular.
bool invert(const ByteMatrix& m, ByteMatrix& out);
ByteMatrix multiply(const ByteMatrix& a, const ByteMatrix& b);

// ---------------------------------------------------------------------------------------------
// v_perm_b32 product tables.
//
// Multiplication by a constant c is GF(2)-linear in the bits of x, so with x split as
// x = x[2:0] ^ x[5:3]<<3 ^ x[7:6]<<6:
//     c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[(x >> 6) & 3]
// T0/T1 have 8 one-byte entries (two dwords: lo = entries 0..3, hi = entries 4..7) and T2 has 4
// (one dword).  v_perm_b32(hi, lo, sel) returns, per byte lane, entry sel (0..7) of the 8-byte
// table {hi:lo}, so one instruction performs 4 byte lookups.  A coefficient therefore packs into
// 5 dwords: {T0.lo, T0.hi, T1.lo, T1.hi, T2}.
// ---------------------------------------------------------------------------------------------
constexpr int kTabWords = 5;
void pack_coef(uint8_t c, uint32_t out[kTabWords]);

// ---------------------------------------------------------------------------------------------
// Pattern record (u32 words), consumed by rs_apply_kernel:
//   [0]                 n_out
//   [1 .. 1+d)          input chunk indices (the d source chunks of the part)
//   [1+d .. 1+d+n_out)  output chunk indices
//   then d*n_out*5      packed coefficient tables, input j, row r at ((j*n_out)+r)*5
//                       (input-major: one input's tables for a row group are contiguous)
// ---------------------------------------------------------------------------------------------
inline size_t pattern_words(size_t d, size_t n_out) { return 1 + d + n_out + n_out * d * kTabWords; }
void write_pattern(uint32_t* dst, size_t d, const std::vector<uint32_t>& in_idx,
                   const std::vector<uint32_t>& out_idx, const ByteMatrix& rows);

}  // namespace cec
