/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product
 * library (chunky-bits_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker / the CPU baseline.
 *
 * CPU restatement of the two third-party crates the reference's hot path calls (neither is
 * vendored in /root/reference):
 *
 *   reed-solomon-erasure 4.0.2 (Cargo.lock:1031-1037, pure-Rust galois_8 path; `simd-accel` off,
 *   Cargo.toml:21) — restated from its published algorithm:
 *     * GF(2^8) with generating polynomial 29 (x^8+x^4+x^3+x^2+1 = 0x11D), generator 2:
 *       LOG/EXP tables built by repeated doubling (crate build.rs), mul via LOG/EXP,
 *       exp(a,n) = EXP[LOG[a]*n mod 255], exp(.,0)=1, exp(0,n>0)=0.
 *     * Coding matrix M = V * inv(V[0..d]), V[r][c] = exp(r, c), r < d+p, c < d
 *       (so the top d x d of M is the identity; parity rows are M[d..d+p]).
 *     * encode_sep: parity[i] = XOR_j M[d+i][j] (x) data[j]    (code_some_slices loop order:
 *       for j in inputs { for i in outputs { mul_slice (j==0) / mul_slice_xor (j>0) } }).
 *     * reconstruct / reconstruct_data: take the FIRST d present shards (index order), invert
 *       those d rows of M, rebuild the missing data shards; `reconstruct` then recomputes the
 *       missing parity from the full data with the parity rows.
 *     * argument checks and their order (check_piece_count!/check_slices! macros and the
 *       reconstruct_internal prologue), returning the crate's Error variants with the codes of
 *       include/chunky_ec.h.
 *   Call sites in the reference: src/file/file_part.rs:77,128,161-165,302-304,
 *   src/file/writer.rs:131, src/bin/chunky-bits/main.rs:263,289,557.
 *
 *   sha2 0.9.9 (Cargo.lock:1221-1231) — SHA-256 per FIPS 180-4; called via Sha256::digest at
 *   src/file/hash/sha256.rs:20-26.  A scalar restatement plus an x86 SHA-NI variant (sha2 0.9.9
 *   dispatches to SHA-NI through `cpufeatures` when present), used only for the CPU baseline.
 *
 * Pinning (tests/test_oracle.py): the reference's own KAT sha256("Hello World")
 * (tests/hash.rs:3-4), hashlib (OpenSSL FIPS 180-4) on many lengths, and the crate's /
 * JavaReedSolomon's published known-answer tests (galois mul/exp values and the RS(5,5)
 * "one encode" vector) — those come from the crate's test-suite, which is not in this
 * container, and are recorded in tests/golden/crate_kats.json.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <cpuid.h>
#endif

/* Error codes: identical numbering to include/chunky_ec.h (reed_solomon_erasure::Error order). */
enum {
    OR_OK = 0,
    OR_TOO_FEW_SHARDS = 1,
    OR_TOO_MANY_SHARDS = 2,
    OR_TOO_FEW_DATA_SHARDS = 3,
    OR_TOO_MANY_DATA_SHARDS = 4,
    OR_TOO_FEW_PARITY_SHARDS = 5,
    OR_TOO_MANY_PARITY_SHARDS = 6,
    OR_TOO_FEW_BUFFER_SHARDS = 7,
    OR_TOO_MANY_BUFFER_SHARDS = 8,
    OR_INCORRECT_SHARD_SIZE = 9,
    OR_TOO_FEW_SHARDS_PRESENT = 10,
    OR_EMPTY_SHARD = 11,
    OR_INVALID_SHARD_FLAGS = 12,
    OR_INVALID_INDEX = 13,
    OR_SINGULAR_MATRIX = 50, /* matrix-internal; unreachable through ReedSolomon for d+p<=256 */
    OR_INVALID_ARGUMENT = 101,
};

/* ------------------------------------------------------------------------------------------ */
/* GF(2^8)                                                                                    */
/* ------------------------------------------------------------------------------------------ */

static uint8_t LOG_T[256];
static uint8_t EXP_T[512];
static uint8_t MUL_T[256][256];
static pthread_once_t gf_once = PTHREAD_ONCE_INIT;

static void gf_init(void) {
    /* crate build.rs gen_log_table(GENERATING_POLYNOMIAL = 29): walk b = 2^log. */
    unsigned b = 1;
    for (unsigned log = 0; log < 255; log++) {
        LOG_T[b] = (uint8_t)log;
        b <<= 1;
        if (b >= 256) b = (b - 256) ^ 29u;
    }
    /* gen_exp_table: EXP[LOG[i]] = i, duplicated at +255 so LOG[a]+LOG[b] never wraps. */
    for (unsigned i = 1; i < 256; i++) {
        EXP_T[LOG_T[i]] = (uint8_t)i;
        EXP_T[LOG_T[i] + 255] = (uint8_t)i;
    }
    for (unsigned a = 0; a < 256; a++)
        for (unsigned c = 0; c < 256; c++)
            MUL_T[a][c] = (a == 0 || c == 0) ? 0 : EXP_T[LOG_T[a] + LOG_T[c]];
}

static inline void gf_ready(void) { pthread_once(&gf_once, gf_init); }

uint8_t or_gf_mul(uint8_t a, uint8_t b) {
    gf_ready();
    return MUL_T[a][b];
}

uint8_t or_gf_div(uint8_t a, uint8_t b) {
    gf_ready();
    if (a == 0) return 0;
    if (b == 0) return 0; /* crate panics; callers never pass 0 */
    int l = (int)LOG_T[a] - (int)LOG_T[b];
    if (l < 0) l += 255;
    return EXP_T[l];
}

uint8_t or_gf_exp(uint8_t a, size_t n) {
    gf_ready();
    if (n == 0) return 1;
    if (a == 0) return 0;
    size_t l = (size_t)LOG_T[a] * n;
    while (l >= 255) l -= 255;
    return EXP_T[l];
}

/* ------------------------------------------------------------------------------------------ */
/* Matrices over GF(2^8) (crate matrix.rs semantics)                                          */
/* ------------------------------------------------------------------------------------------ */

/* Gauss-Jordan inversion of an n x n matrix `m` (row major) into `out`. */
static int gf_invert(const uint8_t* m, size_t n, uint8_t* out) {
    size_t w = 2 * n;
    uint8_t* a = (uint8_t*)calloc(n * w, 1);
    if (!a) return OR_INVALID_ARGUMENT;
    for (size_t r = 0; r < n; r++) {
        memcpy(a + r * w, m + r * n, n);
        a[r * w + n + r] = 1;
    }
    for (size_t r = 0; r < n; r++) {
        if (a[r * w + r] == 0) {
            for (size_t rb = r + 1; rb < n; rb++) {
                if (a[rb * w + r] != 0) {
                    for (size_t c = 0; c < w; c++) {
                        uint8_t t = a[r * w + c];
                        a[r * w + c] = a[rb * w + c];
                        a[rb * w + c] = t;
                    }
                    break;
                }
            }
        }
        if (a[r * w + r] == 0) {
            free(a);
            return OR_SINGULAR_MATRIX;
        }
        if (a[r * w + r] != 1) {
            uint8_t scale = or_gf_div(1, a[r * w + r]);
            for (size_t c = 0; c < w; c++) a[r * w + c] = MUL_T[scale][a[r * w + c]];
        }
        for (size_t rb = r + 1; rb < n; rb++) {
            uint8_t s = a[rb * w + r];
            if (s) for (size_t c = 0; c < w; c++) a[rb * w + c] ^= MUL_T[s][a[r * w + c]];
        }
    }
    for (size_t d = 0; d < n; d++) {
        for (size_t ra = 0; ra < d; ra++) {
            uint8_t s = a[ra * w + d];
            if (s) for (size_t c = 0; c < w; c++) a[ra * w + c] ^= MUL_T[s][a[d * w + c]];
        }
    }
    for (size_t r = 0; r < n; r++) memcpy(out + r * n, a + r * w + n, n);
    free(a);
    return OR_OK;
}

/* ReedSolomon::new(d, p) checks + build_matrix.  `out` is (d+p) x d, row major. */
int or_rs_matrix(size_t d, size_t p, uint8_t* out) {
    gf_ready();
    if (d == 0) return OR_TOO_FEW_DATA_SHARDS;
    if (p == 0) return OR_TOO_FEW_PARITY_SHARDS;
    if (d + p > 256) return OR_TOO_MANY_SHARDS;
    size_t t = d + p;
    uint8_t* v = (uint8_t*)malloc(t * d);
    uint8_t* top_inv = (uint8_t*)malloc(d * d);
    if (!v || !top_inv) return OR_INVALID_ARGUMENT;
    for (size_t r = 0; r < t; r++)
        for (size_t c = 0; c < d; c++) v[r * d + c] = or_gf_exp((uint8_t)r, c);
    int st = gf_invert(v, d, top_inv); /* top d x d of V */
    if (st == OR_OK) {
        for (size_t r = 0; r < t; r++)
            for (size_t c = 0; c < d; c++) {
                uint8_t acc = 0;
                for (size_t k = 0; k < d; k++) acc ^= MUL_T[v[r * d + k]][top_inv[k * d + c]];
                out[r * d + c] = acc;
            }
    }
    free(v);
    free(top_inv);
    return st;
}

int or_gf_invert(const uint8_t* m, size_t n, uint8_t* out) {
    gf_ready();
    return gf_invert(m, n, out);
}

/* crate galois_8::mul_slice / mul_slice_xor, pure-Rust path: MUL_TABLE row, unrolled by 4. */
static void mul_slice(uint8_t c, const uint8_t* in, uint8_t* out, size_t len) {
    const uint8_t* mt = MUL_T[c];
    size_t n = 0;
    if (len > 4) {
        size_t lim = len - 4;
        while (n < lim) {
            out[n] = mt[in[n]];
            out[n + 1] = mt[in[n + 1]];
            out[n + 2] = mt[in[n + 2]];
            out[n + 3] = mt[in[n + 3]];
            n += 4;
        }
    }
    for (; n < len; n++) out[n] = mt[in[n]];
}

static void mul_slice_xor(uint8_t c, const uint8_t* in, uint8_t* out, size_t len) {
    const uint8_t* mt = MUL_T[c];
    size_t n = 0;
    if (len > 4) {
        size_t lim = len - 4;
        while (n < lim) {
            out[n] ^= mt[in[n]];
            out[n + 1] ^= mt[in[n + 1]];
            out[n + 2] ^= mt[in[n + 2]];
            out[n + 3] ^= mt[in[n + 3]];
            n += 4;
        }
    }
    for (; n < len; n++) out[n] ^= mt[in[n]];
}

/* code_some_slices(matrix_rows, inputs, outputs) */
static void code_some_slices(const uint8_t* const* rows, size_t n_in, const uint8_t* const* in,
                             size_t n_out, uint8_t* const* out, size_t len) {
    for (size_t j = 0; j < n_in; j++)
        for (size_t i = 0; i < n_out; i++) {
            if (j == 0) mul_slice(rows[i][j], in[j], out[i], len);
            else mul_slice_xor(rows[i][j], in[j], out[i], len);
        }
}

/* check_slices!(multi => s) */
static int check_multi(const size_t* lens, size_t n) {
    size_t size = lens[0];
    if (size == 0) return OR_EMPTY_SHARD;
    for (size_t i = 0; i < n; i++)
        if (lens[i] != size) return OR_INCORRECT_SHARD_SIZE;
    return OR_OK;
}

/* ReedSolomon::encode_sep(&data, &mut parity) */
int or_rs_encode_sep(size_t d, size_t p, const uint8_t* const* data, const size_t* data_lens,
                     size_t n_data, uint8_t* const* parity, const size_t* parity_lens,
                     size_t n_parity) {
    gf_ready();
    uint8_t* m = (uint8_t*)malloc((d + p) * d);
    if (!m) return OR_INVALID_ARGUMENT;
    int st = or_rs_matrix(d, p, m);
    if (st) { free(m); return st; }
    if (n_data < d) st = OR_TOO_FEW_DATA_SHARDS;
    else if (n_data > d) st = OR_TOO_MANY_DATA_SHARDS;
    else if (n_parity < p) st = OR_TOO_FEW_PARITY_SHARDS;
    else if (n_parity > p) st = OR_TOO_MANY_PARITY_SHARDS;
    if (!st) st = check_multi(data_lens, n_data);
    if (!st) st = check_multi(parity_lens, n_parity);
    if (!st && data_lens[0] != parity_lens[0]) st = OR_INCORRECT_SHARD_SIZE;
    if (!st) {
        const uint8_t** rows = (const uint8_t**)malloc(p * sizeof(*rows));
        for (size_t i = 0; i < p; i++) rows[i] = m + (d + i) * d;
        code_some_slices(rows, d, data, p, parity, data_lens[0]);
        free(rows);
    }
    free(m);
    return st;
}

/*
 * ReedSolomon::reconstruct / reconstruct_data on Option<Vec<u8>> shards.
 * present[i] != 0 <=> Some(shard) with lens[i] bytes.  For a missing slot that the crate would
 * initialise (every missing slot, or only missing DATA slots when data_only), the caller passes
 * a buffer in shards[i] of at least the present shard length; on success present[i] is set to 1
 * for every slot filled (data_only leaves missing parity slots as None, like the crate).
 */
int or_rs_reconstruct(size_t d, size_t p, uint8_t* const* shards, const size_t* lens,
                      uint8_t* present, size_t n_shards, int data_only) {
    gf_ready();
    uint8_t* m = (uint8_t*)malloc((d + p) * d);
    if (!m) return OR_INVALID_ARGUMENT;
    int st = or_rs_matrix(d, p, m);
    if (st) { free(m); return st; }
    size_t t = d + p;
    if (n_shards < t) { free(m); return OR_TOO_FEW_SHARDS; }
    if (n_shards > t) { free(m); return OR_TOO_MANY_SHARDS; }
    size_t n_present = 0, len = 0;
    int have_len = 0;
    for (size_t i = 0; i < t; i++) {
        if (!present[i]) continue;
        if (lens[i] == 0) { free(m); return OR_EMPTY_SHARD; }
        n_present++;
        if (have_len && lens[i] != len) { free(m); return OR_INCORRECT_SHARD_SIZE; }
        len = lens[i];
        have_len = 1;
    }
    if (n_present == t) { free(m); return OR_OK; }
    if (n_present < d) { free(m); return OR_TOO_FEW_SHARDS_PRESENT; }

    size_t valid[256], n_valid = 0, miss_data[256], n_md = 0, miss_par[256], n_mp = 0;
    for (size_t i = 0; i < t; i++) {
        if (present[i]) {
            if (n_valid < d) valid[n_valid++] = i;
        } else if (i < d) {
            miss_data[n_md++] = i;
        } else if (!data_only) {
            miss_par[n_mp++] = i;
        }
    }
    uint8_t* sub = (uint8_t*)malloc(d * d);
    uint8_t* dec = (uint8_t*)malloc(d * d);
    for (size_t r = 0; r < d; r++) memcpy(sub + r * d, m + valid[r] * d, d);
    st = gf_invert(sub, d, dec);
    if (!st && n_md) {
        const uint8_t* rows[256];
        const uint8_t* in[256];
        uint8_t* out[256];
        for (size_t k = 0; k < n_md; k++) { rows[k] = dec + miss_data[k] * d; out[k] = shards[miss_data[k]]; }
        for (size_t j = 0; j < d; j++) in[j] = shards[valid[j]];
        code_some_slices(rows, d, in, n_md, out, len);
        for (size_t k = 0; k < n_md; k++) present[miss_data[k]] = 1;
    }
    if (!st && n_mp) {
        const uint8_t* rows[256];
        const uint8_t* in[256];
        uint8_t* out[256];
        for (size_t k = 0; k < n_mp; k++) { rows[k] = m + miss_par[k] * d; out[k] = shards[miss_par[k]]; }
        for (size_t j = 0; j < d; j++) in[j] = shards[j];
        code_some_slices(rows, d, in, n_mp, out, len);
        for (size_t k = 0; k < n_mp; k++) present[miss_par[k]] = 1;
    }
    free(sub);
    free(dec);
    free(m);
    return st;
}

/* ------------------------------------------------------------------------------------------ */
/* SHA-256 (FIPS 180-4)                                                                       */
/* ------------------------------------------------------------------------------------------ */

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static const uint32_t H0_256[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_blocks_scalar(uint32_t st[8], const uint8_t* p, size_t nblocks) {
    for (; nblocks; nblocks--, p += 64) {
        uint32_t w[64];
        for (int i = 0; i < 16; i++)
            w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
                   ((uint32_t)p[4 * i + 2] << 8) | (uint32_t)p[4 * i + 3];
        for (int i = 16; i < 64; i++) {
            uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
                 h = st[7];
        for (int i = 0; i < 64; i++) {
            uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
            uint32_t ch = (e & f) ^ (~e & g);
            uint32_t t1 = h + S1 + ch + K256[i] + w[i];
            uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
            uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
            uint32_t t2 = S0 + mj;
            h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        st[0] += a; st[1] += b; st[2] += c; st[3] += d;
        st[4] += e; st[5] += f; st[6] += g; st[7] += h;
    }
}

#if defined(__x86_64__)
__attribute__((target("sha,sse4.1,ssse3"))) static void sha256_blocks_shani(uint32_t st[8],
                                                                            const uint8_t* p,
                                                                            size_t nblocks) {
    const __m128i BSWAP = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i tmp = _mm_loadu_si128((const __m128i*)&st[0]);
    __m128i s1 = _mm_loadu_si128((const __m128i*)&st[4]);
    tmp = _mm_shuffle_epi32(tmp, 0xB1);           /* CDAB */
    s1 = _mm_shuffle_epi32(s1, 0x1B);             /* EFGH */
    __m128i s0 = _mm_alignr_epi8(tmp, s1, 8);     /* ABEF */
    s1 = _mm_blend_epi16(s1, tmp, 0xF0);          /* CDGH */
    for (; nblocks; nblocks--, p += 64) {
        __m128i abef = s0, cdgh = s1;
        __m128i w[4];
#pragma GCC unroll 16
        for (int g = 0; g < 16; g++) {
            __m128i m;
            if (g < 4) {
                m = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * g)), BSWAP);
            } else {
                __m128i m0 = w[g & 3], m1 = w[(g + 1) & 3], m2 = w[(g + 2) & 3],
                        m3 = w[(g + 3) & 3];
                m = _mm_sha256msg2_epu32(
                    _mm_add_epi32(_mm_sha256msg1_epu32(m0, m1), _mm_alignr_epi8(m3, m2, 4)), m3);
            }
            w[g & 3] = m;
            __m128i k = _mm_add_epi32(m, _mm_loadu_si128((const __m128i*)&K256[4 * g]));
            s1 = _mm_sha256rnds2_epu32(s1, s0, k);
            k = _mm_shuffle_epi32(k, 0x0E);
            s0 = _mm_sha256rnds2_epu32(s0, s1, k);
        }
        s0 = _mm_add_epi32(s0, abef);
        s1 = _mm_add_epi32(s1, cdgh);
    }
    tmp = _mm_shuffle_epi32(s0, 0x1B);            /* FEBA */
    s1 = _mm_shuffle_epi32(s1, 0xB1);             /* DCHG */
    s0 = _mm_blend_epi16(tmp, s1, 0xF0);          /* DCBA */
    s1 = _mm_alignr_epi8(s1, tmp, 8);             /* HGFE */
    _mm_storeu_si128((__m128i*)&st[0], s0);
    _mm_storeu_si128((__m128i*)&st[4], s1);
}
#endif

int or_cpu_has_shani(void) {
#if defined(__x86_64__)
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return 0;
    if (!(b & (1u << 29))) return 0; /* SHA */
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & (1u << 19)) && (c & (1u << 9)); /* SSE4.1, SSSE3 */
#else
    return 0;
#endif
}

static void sha256_impl(const uint8_t* buf, size_t len, uint8_t out[32], int shani) {
    uint32_t st[8];
    memcpy(st, H0_256, sizeof st);
    size_t full = len / 64;
    void (*blocks)(uint32_t*, const uint8_t*, size_t) = sha256_blocks_scalar;
#if defined(__x86_64__)
    if (shani) blocks = sha256_blocks_shani;
#else
    (void)shani;
#endif
    if (full) blocks(st, buf, full);
    uint8_t tail[128];
    size_t rem = len - full * 64;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, buf + full * 64, rem);
    tail[rem] = 0x80;
    size_t tb = (rem + 9 <= 64) ? 1 : 2;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) tail[tb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    blocks(st, tail, tb);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* Sha256Hash::from_buf (sha256.rs:20-26) */
void or_sha256(const uint8_t* buf, size_t len, uint8_t out[32]) { sha256_impl(buf, len, out, 0); }

int or_sha256_shani(const uint8_t* buf, size_t len, uint8_t out[32]) {
    if (!or_cpu_has_shani()) return -1;
    sha256_impl(buf, len, out, 1);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Part-level restatement: FilePart::write_with_encoder compute (file_part.rs:150-185)        */
/* ------------------------------------------------------------------------------------------ */

/*
 * data_buf holds >= d*ceil(length/d) bytes (zero padded past `length`, like writer.rs:172).
 * parity_out: p*L bytes; digests_out: (d+p)*32 bytes, chunks in order (d data, then p parity).
 * Returns the chunk size L through *chunksize.
 */
int or_part_encode(size_t d, size_t p, const uint8_t* data_buf, size_t length,
                   uint8_t* parity_out, uint8_t* digests_out, size_t* chunksize) {
    size_t L = (length + d - 1) / d;
    const uint8_t* data[256];
    uint8_t* par[256];
    size_t dl[256], pl[256];
    for (size_t j = 0; j < d && j < 256; j++) { data[j] = data_buf + j * L; dl[j] = L; }
    for (size_t i = 0; i < p && i < 256; i++) { par[i] = parity_out + i * L; pl[i] = L; }
    int st = or_rs_encode_sep(d, p, data, dl, d, par, pl, p);
    if (st) return st;
    for (size_t j = 0; j < d; j++) or_sha256(data[j], L, digests_out + 32 * j);
    for (size_t i = 0; i < p; i++) or_sha256(par[i], L, digests_out + 32 * (d + i));
    *chunksize = L;
    return OR_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* CPU baseline: encode_sep + sha256 of all d+p chunks, one part per task, n_threads workers  */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    size_t d, p, L, total_parts, pool;
    int shani, hash;
    uint8_t** bufs; /* per worker: pool * (d+p)*L bytes */
    volatile size_t next;
    pthread_mutex_t mu;
    uint8_t sink;
} baseline_ctx;

typedef struct {
    baseline_ctx* ctx;
    int id;
} baseline_arg;

static void* baseline_worker(void* a_) {
    baseline_arg* a = (baseline_arg*)a_;
    baseline_ctx* c = a->ctx;
    size_t d = c->d, p = c->p, L = c->L;
    const uint8_t* rows[256];
    uint8_t* m = (uint8_t*)malloc((d + p) * d);
    or_rs_matrix(d, p, m);
    for (size_t i = 0; i < p; i++) rows[i] = m + (d + i) * d;
    uint8_t dig[32];
    uint8_t acc = 0;
    for (;;) {
        pthread_mutex_lock(&c->mu);
        size_t part = c->next++;
        pthread_mutex_unlock(&c->mu);
        if (part >= c->total_parts) break;
        uint8_t* base = c->bufs[a->id] + (part % c->pool) * (d + p) * L;
        const uint8_t* in[256];
        uint8_t* out[256];
        for (size_t j = 0; j < d; j++) in[j] = base + j * L;
        for (size_t i = 0; i < p; i++) out[i] = base + (d + i) * L;
        code_some_slices(rows, d, in, p, out, L);
        for (size_t k = 0; c->hash && k < d + p; k++) {
            sha256_impl(base + k * L, L, dig, c->shani);
            acc ^= dig[0];
        }
    }
    pthread_mutex_lock(&c->mu);
    c->sink ^= acc;
    pthread_mutex_unlock(&c->mu);
    free(m);
    return NULL;
}

/*
 * Times `total_parts` part encodes (+ sha256 of all d+p chunks when hash != 0) over n_threads
 * workers; each worker cycles over `pool` resident parts of pseudo-random data (generated
 * before the clock starts).  Returns wall seconds through *seconds.
 */
int or_baseline_encode_sha(size_t d, size_t p, size_t L, size_t total_parts, size_t pool,
                           int n_threads, int use_shani, int do_hash, double* seconds) {
    gf_ready();
    if (d == 0 || p == 0 || d + p > 256 || n_threads <= 0 || pool == 0) return OR_INVALID_ARGUMENT;
    baseline_ctx c;
    memset(&c, 0, sizeof c);
    c.d = d; c.p = p; c.L = L; c.total_parts = total_parts; c.pool = pool;
    c.shani = use_shani && or_cpu_has_shani();
    c.hash = do_hash;
    pthread_mutex_init(&c.mu, NULL);
    c.bufs = (uint8_t**)calloc((size_t)n_threads, sizeof(uint8_t*));
    uint64_t s = 0x9E3779B97F4A7C15ULL;
    for (int t = 0; t < n_threads; t++) {
        size_t n = pool * (d + p) * L;
        c.bufs[t] = (uint8_t*)malloc(n);
        if (!c.bufs[t]) return OR_INVALID_ARGUMENT;
        for (size_t i = 0; i < n; i++) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            c.bufs[t][i] = (uint8_t)(s >> 24);
        }
    }
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    baseline_arg* args = (baseline_arg*)calloc((size_t)n_threads, sizeof(baseline_arg));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < n_threads; t++) {
        args[t].ctx = &c;
        args[t].id = t;
        pthread_create(&th[t], NULL, baseline_worker, &args[t]);
    }
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    for (int t = 0; t < n_threads; t++) free(c.bufs[t]);
    free(c.bufs);
    free(th);
    free(args);
    pthread_mutex_destroy(&c.mu);
    return OR_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Checker: FilePart::write_with_encoder's digests for a whole batch of full parts            */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    size_t d, p, L, n_parts, part_stride;
    const uint8_t* data;
    uint8_t* digests;
    uint8_t* parity_match;
    int shani;
    int failed; /* a worker could not allocate its scratch */
    volatile size_t next;
    pthread_mutex_t mu;
} digest_ctx;

static void* digest_worker(void* a_) {
    digest_ctx* c = (digest_ctx*)a_;
    size_t d = c->d, p = c->p, L = c->L;
    const uint8_t* rows[256];
    uint8_t* m = (uint8_t*)malloc((d + p) * d);
    uint8_t* par = (uint8_t*)malloc(p * L);
    if (!m || !par) {
        free(par);
        free(m);
        pthread_mutex_lock(&c->mu);
        c->failed = 1;
        pthread_mutex_unlock(&c->mu);
        return NULL;
    }
    or_rs_matrix(d, p, m);
    for (size_t i = 0; i < p; i++) rows[i] = m + (d + i) * d;
    for (;;) {
        pthread_mutex_lock(&c->mu);
        size_t part = c->next++;
        pthread_mutex_unlock(&c->mu);
        if (part >= c->n_parts) break;
        const uint8_t* base = c->data + part * c->part_stride;
        const uint8_t* in[256];
        uint8_t* out[256];
        for (size_t j = 0; j < d; j++) in[j] = base + j * L;
        for (size_t i = 0; i < p; i++) out[i] = par + i * L;
        code_some_slices(rows, d, in, p, out, L);
        if (c->parity_match)
            c->parity_match[part] = memcmp(par, base + d * L, p * L) == 0;
        uint8_t* dig = c->digests + part * (d + p) * 32;
        for (size_t j = 0; j < d; j++) sha256_impl(in[j], L, dig + 32 * j, c->shani);
        for (size_t i = 0; i < p; i++) sha256_impl(out[i], L, dig + 32 * (d + i), c->shani);
    }
    free(par);
    free(m);
    return NULL;
}

/*
 * digests[n_parts][d+p][32] of n_parts full parts whose d data chunks (L bytes each, back to
 * back) start `part_stride` bytes apart in `data`: encode_sep (file_part.rs:161-165) then
 * Sha256Hash::from_buf of each chunk in order (:185), over n_threads workers.  With
 * parity_match != NULL the p chunks that follow the data chunks in `data` (part_stride >=
 * (d+p)*L) are compared with the computed parity: parity_match[part] = 1 if equal.  The bench's
 * cpu_baseline leg checks a whole device batch with it.
 */
int or_encode_hash_parts(size_t d, size_t p, size_t L, size_t n_parts, const uint8_t* data,
                         size_t part_stride, uint8_t* digests, uint8_t* parity_match,
                         int n_threads) {
    gf_ready();
    if (d == 0 || p == 0 || d + p > 256 || L == 0 || n_threads <= 0 || part_stride < d * L ||
        (parity_match && part_stride < (d + p) * L))
        return OR_INVALID_ARGUMENT;
    digest_ctx c;
    memset(&c, 0, sizeof c);
    c.d = d; c.p = p; c.L = L; c.n_parts = n_parts; c.part_stride = part_stride;
    c.data = data; c.digests = digests; c.parity_match = parity_match;
    c.shani = or_cpu_has_shani();
    pthread_mutex_init(&c.mu, NULL);
    pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
    if (!th) return OR_INVALID_ARGUMENT;
    int started = 0;
    for (int t = 0; t < n_threads; t++)
        if (pthread_create(&th[t], NULL, digest_worker, &c) == 0) started++;
        else break;
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&c.mu);
    /* every part was claimed by a worker that ran to completion, or the call fails */
    return (started == 0 || c.failed || c.next < n_parts) ? OR_INVALID_ARGUMENT : OR_OK;
}
