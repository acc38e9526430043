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
