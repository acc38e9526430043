/*
 * kq_cpu_simd.c — CPU ORACLE companion (test infrastructure / CPU baseline only).
 *
 * AVX2 forms of the restated NEON vec_dots (kq_oracle.c), used for bench.py's
 * cpu_baseline leg so the host-side figure is a vectorised CPU path rather than
 * the scalar checker. The integer parts are computed with u8 x i8 pair products
 * (vpmaddubsw: |pair| <= 2*63*128 < 2^15, so no saturation for 4/5/6-bit quants)
 * and i16 x i16 pair sums (vpmaddwd) — exact, so they equal the scalar
 * restatement's int32 values; the fp32 update per superblock is the same fmaf
 * sequence (README.md:551 fmsub, :614 fmadd for Q4_K; the Q6_K / Q5_K
 * contractions of kq_oracle.c). Outputs are therefore bit-identical to the
 * scalar oracle (tests/test_oracle.py::test_simd_vec_dot_matches_scalar).
 * Never linked by the product path.
 */
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "kq_oracle.h"

static inline int32_t hsum_i32(__m256i v) {
    __m128i s = _mm_add_epi32(_mm256_castsi256_si128(v), _mm256_extracti128_si256(v, 1));
    s = _mm_add_epi32(s, _mm_shuffle_epi32(s, 0x4E));
    s = _mm_add_epi32(s, _mm_shuffle_epi32(s, 0xB1));
    return _mm_cvtsi128_si32(s);
}

/* 6-bit scales/mins of Q4_K/Q5_K (README.md:732-739; kmask1/2/3). */
static inline void unpack_sm(const uint8_t *q, uint8_t sc[8], uint8_t mn[8]) {
    for (int j = 0; j < 4; ++j) {
        sc[j] = q[j] & 63;
        mn[j] = q[j + 4] & 63;
        sc[j + 4] = (uint8_t)((q[j + 8] & 0xF) | ((q[j] >> 6) << 4));
        mn[j + 4] = (uint8_t)((q[j + 8] >> 4) | ((q[j + 4] >> 6) << 4));
    }
}

/* sum_g bsums[g] * m[g/2] over the 16 groups (int16 products summed in int32). */
static inline int32_t mins_dot(const int16_t *bsums, const uint8_t mn[8]) {
    const __m256i b = _mm256_loadu_si256((const __m256i *)bsums);
    const __m128i m8 = _mm_loadl_epi64((const __m128i *)mn);
    const __m128i m16 = _mm_unpacklo_epi8(m8, m8);  /* m0 m0 m1 m1 ... as bytes */
    const __m256i m = _mm256_cvtepu8_epi16(m16);
    return hsum_i32(_mm256_madd_epi16(b, m));
}

void kqo_vec_dot_q4_K_q8_K_simd(int n, float *s, size_t bs, const void *vx, size_t bx, const void *vy, size_t by,
                                int nrc) {
    (void)bs; (void)bx; (void)by; (void)nrc;
    const kqo_block_q4_K *x = (const kqo_block_q4_K *)vx;
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / KQO_QK_K;
    const __m256i m4 = _mm256_set1_epi8(0x0F);
    float sumf = 0;
    for (int i = 0; i < nb; ++i) {
        const float d = y[i].d * kqo_fp16_to_fp32(x[i].d);
        const float dmin = y[i].d * kqo_fp16_to_fp32(x[i].dmin);
        uint8_t sc[8], mn[8];
        unpack_sm(x[i].scales, sc, mn);
        const int32_t summins = mins_dot(y[i].bsums, mn);
        __m256i acc = _mm256_setzero_si256();
        const uint8_t *q4 = x[i].qs;
        const int8_t *q8 = y[i].qs;
        for (int j = 0; j < 4; ++j) {
            const __m256i q = _mm256_loadu_si256((const __m256i *)(q4 + 32 * j));
            const __m256i lo = _mm256_and_si256(q, m4);
            const __m256i hi = _mm256_and_si256(_mm256_srli_epi16(q, 4), m4);
            const __m256i a0 = _mm256_loadu_si256((const __m256i *)(q8 + 64 * j));
            const __m256i a1 = _mm256_loadu_si256((const __m256i *)(q8 + 64 * j + 32));
            const __m256i p0 = _mm256_madd_epi16(_mm256_maddubs_epi16(lo, a0), _mm256_set1_epi16(sc[2 * j]));
            const __m256i p1 = _mm256_madd_epi16(_mm256_maddubs_epi16(hi, a1), _mm256_set1_epi16(sc[2 * j + 1]));
            acc = _mm256_add_epi32(acc, _mm256_add_epi32(p0, p1));
        }
        const int32_t sumi = hsum_i32(acc);
        sumf = fmaf(-(float)summins, dmin, sumf); /* fmsub, README.md:551 */
        sumf = fmaf((float)sumi, d, sumf);        /* fmadd, README.md:614 */
    }
    *s = sumf;
}

void kqo_vec_dot_q5_K_q8_K_simd(int n, float *s, size_t bs, const void *vx, size_t bx, const void *vy, size_t by,
                                int nrc) {
    (void)bs; (void)bx; (void)by; (void)nrc;
    const kqo_block_q5_K *x = (const kqo_block_q5_K *)vx;
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / KQO_QK_K;
    const __m256i m4 = _mm256_set1_epi8(0x0F);
    const __m256i one = _mm256_set1_epi8(1);
    float sumf = 0;
    for (int i = 0; i < nb; ++i) {
        const float d = y[i].d * kqo_fp16_to_fp32(x[i].d);
        const float dmin = y[i].d * kqo_fp16_to_fp32(x[i].dmin);
        uint8_t sc[8], mn[8];
        unpack_sm(x[i].scales, sc, mn);
        const int32_t summins = mins_dot(y[i].bsums, mn);
        const __m256i qh = _mm256_loadu_si256((const __m256i *)x[i].qh);
        __m256i acc = _mm256_setzero_si256();
        for (int j = 0; j < 4; ++j) {
            const __m256i q = _mm256_loadu_si256((const __m256i *)(x[i].qs + 32 * j));
            /* bit 2j / 2j+1 of qh[l] -> 16 (bytes: shift in 16-bit lanes then mask the low bit) */
            const __m256i h0 = _mm256_and_si256(_mm256_srli_epi16(qh, 2 * j), one);
            const __m256i h1 = _mm256_and_si256(_mm256_srli_epi16(qh, 2 * j + 1), one);
            const __m256i lo = _mm256_or_si256(_mm256_and_si256(q, m4), _mm256_slli_epi16(h0, 4));
            const __m256i hi = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(q, 4), m4), _mm256_slli_epi16(h1, 4));
            const __m256i a0 = _mm256_loadu_si256((const __m256i *)(y[i].qs + 64 * j));
            const __m256i a1 = _mm256_loadu_si256((const __m256i *)(y[i].qs + 64 * j + 32));
            const __m256i p0 = _mm256_madd_epi16(_mm256_maddubs_epi16(lo, a0), _mm256_set1_epi16(sc[2 * j]));
            const __m256i p1 = _mm256_madd_epi16(_mm256_maddubs_epi16(hi, a1), _mm256_set1_epi16(sc[2 * j + 1]));
            acc = _mm256_add_epi32(acc, _mm256_add_epi32(p0, p1));
        }
        const int32_t sumi = hsum_i32(acc);
        const float t = fmaf(d, (float)sumi, -(dmin * (float)summins)); /* kq_oracle.c Q5_K contraction */
        sumf = sumf + t;
    }
    *s = sumf;
}

void kqo_vec_dot_q6_K_q8_K_simd(int n, float *s, size_t bs, const void *vx, size_t bx, const void *vy, size_t by,
                                int nrc) {
    (void)bs; (void)bx; (void)by; (void)nrc;
    const kqo_block_q6_K *x = (const kqo_block_q6_K *)vx;
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / KQO_QK_K;
    const __m256i m4 = _mm256_set1_epi8(0x0F);
    const __m256i m2 = _mm256_set1_epi8(0x03);
    float sum = 0;
    for (int i = 0; i < nb; ++i) {
        const float d_all = kqo_fp16_to_fp32(x[i].d);
        /* isum_mins = sum_g bsums[g] * scale[g] (signed 8-bit scales) */
        const __m256i b = _mm256_loadu_si256((const __m256i *)y[i].bsums);
        const __m256i scl16 = _mm256_cvtepi8_epi16(_mm_loadu_si128((const __m128i *)x[i].scales));
        const int32_t isum_mins = hsum_i32(_mm256_madd_epi16(b, scl16));
        __m256i acc = _mm256_setzero_si256();
        for (int j = 0; j < 2; ++j) {
            const uint8_t *ql = x[i].ql + 64 * j;
            const __m256i h = _mm256_loadu_si256((const __m256i *)(x[i].qh + 32 * j));
            const __m256i l0 = _mm256_loadu_si256((const __m256i *)ql);
            const __m256i l1 = _mm256_loadu_si256((const __m256i *)(ql + 32));
            __m256i qv[4];
            qv[0] = _mm256_or_si256(_mm256_and_si256(l0, m4), _mm256_slli_epi16(_mm256_and_si256(h, m2), 4));
            qv[1] = _mm256_or_si256(_mm256_and_si256(l1, m4),
                                    _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(h, 2), m2), 4));
            qv[2] = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(l0, 4), m4),
                                    _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(h, 4), m2), 4));
            qv[3] = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(l1, 4), m4),
                                    _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(h, 6), m2), 4));
            for (int part = 0; part < 4; ++part) {
                const __m256i a = _mm256_loadu_si256((const __m256i *)(y[i].qs + 128 * j + 32 * part));
                const int g = 8 * j + 2 * part; /* elements 16g .. 16g+31 */
                const __m256i sv = _mm256_setr_m128i(_mm_set1_epi16(x[i].scales[g]), _mm_set1_epi16(x[i].scales[g + 1]));
                acc = _mm256_add_epi32(acc, _mm256_madd_epi16(_mm256_maddubs_epi16(qv[part], a), sv));
            }
        }
        const int32_t isum = hsum_i32(acc);
        sum = fmaf(d_all * y[i].d, (float)(isum - 32 * isum_mins), sum); /* kq_oracle.c Q6_K contraction */
    }
    *s = sum;
}

/* ------------------------------------------------------------ binary16 arithmetic */
/* vfmaq_f16 lane c + a*b with one rounding (kq_ops_oracle.c kqo_f16_fma restates it
 * on 128-bit integers). Here: p = a*b is exact in double (22 significant bits),
 * s = p + c rounded to double with its exact error e (TwoSum); rounding s to binary16
 * equals rounding p + c unless s sits exactly on a binary16 midpoint and e != 0 —
 * then the tie is broken toward e. Finite inputs (the attention's values). */
static inline uint16_t f16_from_double(double s, double err) {
    uint64_t bits;
    memcpy(&bits, &s, 8);
    const uint16_t sign = (uint16_t)((bits >> 48) & 0x8000);
    bits &= 0x7fffffffffffffffull;
    if (bits == 0) return sign; /* signed zero: IEEE sum sign, as the restatement */
    const int up = (err != 0.0) && ((err > 0) == (sign == 0)); /* exact value above |s| */
    const int exp = (int)(bits >> 52) - 1023;                   /* finite, normal doubles here */
    const uint64_t mant = (bits & 0xfffffffffffffull) | (1ull << 52);
    int e = exp < -14 ? -14 : exp;
    const int shift = 42 + (e - exp); /* low bits of the 53-bit significand below the quantum */
    if (shift > 53) return sign;      /* < 2^-25: rounds to zero */
    uint64_t q = mant >> shift;
    const uint64_t rem = mant & ((1ull << shift) - 1), half = 1ull << (shift - 1);
    if (rem > half || (rem == half && (err != 0.0 ? up : (int)(q & 1)))) q++;
    if (q >= 2048) {
        q >>= 1;
        e++;
    }
    if (e > 15) return sign | 0x7c00;
    if (q < 1024) return sign | (uint16_t)q; /* subnormal */
    return sign | (uint16_t)(((e + 15) << 10) | (int)(q - 1024));
}

static inline double h2d(uint16_t h) { return (double)_cvtsh_ss(h); }

uint16_t kqo_f16_fma_fast(uint16_t a, uint16_t b, uint16_t c) {
    const double p = h2d(a) * h2d(b), cc = h2d(c);
    const double s = p + cc;
    const double bb = s - p;
    const double err = (p - (s - bb)) + (cc - bb);
    return f16_from_double(s, err);
}

uint16_t kqo_f16_add_fast(uint16_t a, uint16_t b) { return f16_from_double(h2d(a) + h2d(b), 0.0); /* exact */ }

static inline uint64_t xs64(uint64_t *s) {
    uint64_t x = *s;
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return *s = x;
}

long kqo_f16_fast_check(long n, uint64_t seed) {
    uint64_t st = seed | 1;
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        const uint64_t r = xs64(&st);
        uint16_t a = (uint16_t)r, b = (uint16_t)(r >> 16), c = (uint16_t)(r >> 32);
        /* finite operands only; bias some toward nearby exponents and exact midpoints */
        if (((a >> 10) & 0x1f) == 0x1f) a &= 0xbfff;
        if (((b >> 10) & 0x1f) == 0x1f) b &= 0xbfff;
        if (((c >> 10) & 0x1f) == 0x1f) c &= 0xbfff;
        if ((r >> 48) % 4 == 0) c = (uint16_t)((c & 0x83ff) | (a & 0x7c00));
        if (kqo_f16_fma_fast(a, b, c) != kqo_f16_fma(a, b, c)) ++bad;
        if (kqo_f16_add_fast(a, c) != kqo_f16_add(a, c)) ++bad;
    }
    return bad;
}

/* kqo_vec_dot_f16 with the fast binary16 ops (same structure and order). */
static float vec_dot_f16_fast(int n, const uint16_t *x, const uint16_t *y) {
    const int np = n & ~31;
    uint16_t sum[4][8];
    memset(sum, 0, sizeof(sum));
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; ++j)
            for (int l = 0; l < 8; ++l)
                sum[j][l] = kqo_f16_fma_fast(x[i + 8 * j + l], y[i + 8 * j + l], sum[j][l]);
    for (int l = 0; l < 8; ++l) {
        sum[0][l] = kqo_f16_add_fast(sum[0][l], sum[2][l]);
        sum[1][l] = kqo_f16_add_fast(sum[1][l], sum[3][l]);
    }
    for (int l = 0; l < 8; ++l) sum[0][l] = kqo_f16_add_fast(sum[0][l], sum[1][l]);
    float t[4];
    for (int k = 0; k < 4; ++k) t[k] = kqo_fp16_to_fp32(sum[0][k]) + kqo_fp16_to_fp32(sum[0][k + 4]);
    double sumf = (double)((t[0] + t[1]) + (t[2] + t[3]));
    for (int i = np; i < n; ++i) sumf += (double)(kqo_fp16_to_fp32(x[i]) * kqo_fp16_to_fp32(y[i]));
    return (float)sumf;
}

typedef struct {
    const float *q;
    const uint16_t *k_cache, *v_cache;
    int pos, n_ctx, n_kv, gsz, kvw, head_dim;
    float scale;
    float *out;
} attn_ctx;

static void attn_head(void *vc, int h) {
    const attn_ctx *a = (const attn_ctx *)vc;
    const int g = h / a->gsz, hd = a->head_dim, n_kv = a->n_kv;
    uint16_t q16[512];
    float kq[8192], mask[8192];
    uint16_t p16[8192];
    for (int c = 0; c < n_kv; ++c) mask[c] = c <= a->pos ? 0.0f : -INFINITY;
    kqo_fp32_to_fp16_row(a->q + (int64_t)h * hd, q16, hd);
    for (int c = 0; c < n_kv; ++c)
        kq[c] = vec_dot_f16_fast(hd, a->k_cache + (int64_t)c * a->kvw + (int64_t)g * hd, q16);
    kqo_soft_max_row(n_kv, kq, kq, mask, a->scale);
    kqo_fp32_to_fp16_row(kq, p16, n_kv);
    for (int d = 0; d < hd; ++d)
        a->out[(int64_t)h * hd + d] = vec_dot_f16_fast(n_kv, a->v_cache + (int64_t)(g * hd + d) * a->n_ctx, p16);
}

/* kqo_attn_decode (kq_ops_oracle.c) with the fast binary16 ops, heads spread over the
 * worker pool as ggml-cpu spreads the attention's rows over its threads. */
void kqo_attn_decode_fast(const float *q, const float *k, const float *v, uint16_t *k_cache, uint16_t *v_cache,
                          int pos, int n_ctx, int n_head, int n_head_kv, int head_dim, float scale, float *out,
                          int n_threads) {
    const int kvw = n_head_kv * head_dim;
    kqo_fp32_to_fp16_row(k, k_cache + (int64_t)pos * kvw, kvw);
    for (int ch = 0; ch < kvw; ++ch) v_cache[(int64_t)ch * n_ctx + pos] = kqo_fp32_to_fp16(v[ch]);
    attn_ctx a = {q, k_cache, v_cache, pos, n_ctx, kqo_attn_n_kv(pos, n_ctx), n_head / n_head_kv, kvw, head_dim,
                  scale, out};
    kqo_pool_run(n_threads, n_head, attn_head, &a);
}
