// gf256.cpp — see gf256.hpp.
#include "gf256.hpp"

#include <cstring>

namespace cec {

Gf256::Gf256() {
    std::memset(log, 0, sizeof log);
    std::memset(exp, 0, sizeof exp);
    unsigned x = 1;
    for (unsigned i = 0; i < 255; ++i) {
        exp[i] = static_cast<uint8_t>(x);
        exp[i + 255] = static_cast<uint8_t>(x);
        log[x] = static_cast<uint8_t>(i);
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
}

const Gf256& Gf256::get() {
    static const Gf256 g;
    return g;
}

uint8_t Gf256::div(uint8_t a, uint8_t b) const {
    if (a == 0) return 0;
    int l = int(log[a]) - int(log[b]);
    if (l < 0) l += 255;
    return exp[l];
}

uint8_t Gf256::pow(uint8_t a, size_t n) const {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return exp[(size_t(log[a]) * n) % 255];
}

ByteMatrix multiply(const ByteMatrix& a, const ByteMatrix& b) {
    const Gf256& g = Gf256::get();
    ByteMatrix out(a.rows, b.cols);
    for (size_t r = 0; r < a.rows; ++r)
        for (size_t c = 0; c < b.cols; ++c) {
            uint8_t acc = 0;
            for (size_t k = 0; k < a.cols; ++k) acc ^= g.mul(a.at(r, k), b.at(k, c));
            out.at(r, c) = acc;
        }
    return out;
}

bool invert(const ByteMatrix& m, ByteMatrix& out) {
    const Gf256& g = Gf256::get();
    const size_t n = m.rows;
    ByteMatrix w(n, 2 * n);
    for (size_t r = 0; r < n; ++r) {
        for (size_t c = 0; c < n; ++c) w.at(r, c) = m.at(r, c);
        w.at(r, n + r) = 1;
    }
    for (size_t col = 0; col < n; ++col) {
        size_t piv = col;
        while (piv < n && w.at(piv, col) == 0) ++piv;
        if (piv == n) return false;
        if (piv != col)
            for (size_t c = 0; c < 2 * n; ++c) std::swap(w.at(piv, c), w.at(col, c));
        const uint8_t inv = g.div(1, w.at(col, col));
        for (size_t c = 0; c < 2 * n; ++c) w.at(col, c) = g.mul(inv, w.at(col, c));
        for (size_t r = 0; r < n; ++r) {
            if (r == col) continue;
            const uint8_t f = w.at(r, col);
            if (!f) continue;
            for (size_t c = 0; c < 2 * n; ++c) w.at(r, c) ^= g.mul(f, w.at(col, c));
        }
    }
    out = ByteMatrix(n, n);
    for (size_t r = 0; r < n; ++r)
        for (size_t c = 0; c < n; ++c) out.at(r, c) = w.at(r, n + c);
    return true;
}

ByteMatrix build_coding_matrix(size_t d, size_t p) {
    const Gf256& g = Gf256::get();
    const size_t t = d + p;
    ByteMatrix vand(t, d);
    for (size_t r = 0; r < t; ++r)
        for (size_t c = 0; c < d; ++c) vand.at(r, c) = g.pow(static_cast<uint8_t>(r), c);
    ByteMatrix top(d, d), top_inv;
    for (size_t r = 0; r < d; ++r)
        for (size_t c = 0; c < d; ++c) top.at(r, c) = vand.at(r, c);
    invert(top, top_inv);  // distinct evaluation points 0..d-1: always invertible
    return multiply(vand, top_inv);
}

void pack_coef(uint8_t c, uint32_t out[kTabWords]) {
    const Gf256& g = Gf256::get();
    auto word = [&](unsigned e0, unsigned e1, unsigned e2, unsigned e3) {
        return uint32_t(g.mul(c, uint8_t(e0))) | (uint32_t(g.mul(c, uint8_t(e1))) << 8) |
               (uint32_t(g.mul(c, uint8_t(e2))) << 16) | (uint32_t(g.mul(c, uint8_t(e3))) << 24);
    };
    out[0] = word(0, 1, 2, 3);
    out[1] = word(4, 5, 6, 7);
    out[2] = word(0, 8, 16, 24);
    out[3] = word(32, 40, 48, 56);
    out[4] = word(0, 64, 128, 192);
}

void write_pattern(uint32_t* dst, size_t d, const std::vector<uint32_t>& in_idx,
                   const std::vector<uint32_t>& out_idx, const ByteMatrix& rows) {
    const size_t n_out = out_idx.size();
    dst[0] = uint32_t(n_out);
    for (size_t j = 0; j < d; ++j) dst[1 + j] = in_idx[j];
    for (size_t r = 0; r < n_out; ++r) dst[1 + d + r] = out_idx[r];
    uint32_t* tab = dst + 1 + d + n_out;
    for (size_t r = 0; r < n_out; ++r)
        for (size_t j = 0; j < d; ++j) pack_coef(rows.at(r, j), tab + (j * n_out + r) * kTabWords);
}

}  // namespace cec
