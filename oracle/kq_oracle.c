/*
 * kq_oracle.c — CPU ORACLE for the Q4_K/Q5_K/Q6_K x Q8_K dot path.
 *
 * TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker. Never linked into, called by,
 * or substituted for the product path (ggml-neon-opt_amd/). See kq_oracle.h
 * for the parity status ("parity unpinned": no reference fixtures exist).
 *
 * Built with -ffp-contract=off: every fused multiply-add that the reference
 * build performs is written explicitly as fmaf(), every other product is
 * rounded on its own, so the float semantics do not depend on this host's
 * compiler flags.
 *
 * Sources restated (all in /root/reference):
 *   - NEON ggml_vec_dot_q4_K_q8_K, README.md:686-779 (optimized variant
 *     README.md:1455-1480 gives the identical value: the per-superblock int32
 *     sum is reassociated exactly, README.md:1101-1106)
 *   - FP contraction from the disassembly: `fmsub s21,s0,s2,s4` (README.md:551)
 *     = sumf - (float)summins*dmin with one rounding, and `fmadd s4,s0,s20,s21`
 *     (README.md:614) = sumf + (float)sumi*d with one rounding.
 *   - struct offsets: README.md:459-460, 472, 480, 488, 492, 507, 522, 529, 610-611.
 *   - quantize_row_q8_K -> quantize_row_q8_K_ref + nearest_int (out.folded:184-186);
 *     body restated from upstream ggml-quants.c @ a3cb0474 [U].
 *   - generic q4_K path (fallback named at README.md:626), Q6_K NEON (profiled at
 *     README.md:369, out.folded:160), Q5_K, dequantize_row_*: upstream @ a3cb0474 [U].
 *   - mul_mat dispatch/chunking: ggml-cpu.c:1389/:1194 as evidenced by
 *     README.md:136, :156 (64-row chunks, thread ith starts at chunk ith).
 */
#define _GNU_SOURCE
#include "kq_oracle.h"

#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define QK_K KQO_QK_K

/* ------------------------------------------------------------ fp16 helpers */
float kqo_fp16_to_fp32(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    const uint32_t exp = (h >> 10) & 0x1f;
    const uint32_t man = h & 0x3ffu;
    uint32_t bits;
    if (exp == 0) {
        if (man == 0) {
            bits = sign;
        } else { /* subnormal: normalise */
            int e = -1;
            uint32_t m = man;
            do { m <<= 1; e++; } while ((m & 0x400u) == 0);
            bits = sign | ((uint32_t)(127 - 15 - e) << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (exp == 31) {
        bits = sign | 0x7f800000u | (man << 13);
    } else {
        bits = sign | ((exp + 127 - 15) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

uint16_t kqo_fp32_to_fp16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t abs = x & 0x7fffffffu;
    if (abs >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (abs > 0x7f800000u ? 0x200u : 0));
    if (abs >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* overflow -> inf */
    if (abs < 0x38800000u) {                                   /* subnormal half */
        /* value = abs_float; half subnormal unit = 2^-24 */
        float af;
        memcpy(&af, &abs, 4);
        float scaled = af * 16777216.0f; /* exact: power-of-two scaling */
        /* round half to even */
        float r = nearbyintf(scaled);
        return (uint16_t)(sign | (uint32_t)r);
    }
    uint32_t e = (abs >> 23) - 127 + 15;
    uint32_t m = abs & 0x7fffffu;
    uint32_t half = (e << 10) | (m >> 13);
    uint32_t rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (half & 1u))) half++;
    return (uint16_t)(sign | half);
}

/* --------------------------------------------------------- Q8_K quantizer */
static inline int nearest_int_unfused(float fval) {
    float val = fval + 12582912.f;
    int i;
    memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

static inline int nearest_int_fused(float iscale, float x) {
    float val = fmaf(iscale, x, 12582912.f);
    int i;
    memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

void kqo_quantize_row_q8_K(const float *x, kqo_block_q8_K *y, int64_t k, int fused) {
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        float max = 0;
        float amax = 0;
        for (int j = 0; j < QK_K; ++j) {
            float ax = fabsf(x[j]);
            if (ax > amax) {
                amax = ax;
                max = x[j];
            }
        }
        if (!amax) {
            y[i].d = 0;
            memset(y[i].qs, 0, QK_K);
            /* upstream leaves bsums unwritten here; d == 0 makes them
             * irrelevant to every dot. Defined as 0 in this build. */
            memset(y[i].bsums, 0, sizeof(y[i].bsums));
            x += QK_K;
            continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < QK_K; ++j) {
            int v = fused ? nearest_int_fused(iscale, x[j]) : nearest_int_unfused(iscale * x[j]);
            y[i].qs[j] = (int8_t)(v < 127 ? v : 127);
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = (int16_t)sum;
        }
        y[i].d = 1 / iscale;
        x += QK_K;
    }
}

/* ------------------------------------------------------ scale/min unpack */
/* get_scale_min_k4 [U]; equals the kmask1/2/3 utmp shuffle of README.md:732-739. */
static inline void get_scale_min_k4(int j, const uint8_t *q, uint8_t *d, uint8_t *m) {
    if (j < 4) {
        *d = q[j] & 63;
        *m = q[j + 4] & 63;
    } else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

/* The NEON listing's own unpack (README.md:732-739), kept separately so tests
 * can check the two formulations agree on all 2^96... sampled byte patterns. */
static inline void unpack_scales_neon(const uint8_t *s12, uint8_t scales[8], uint8_t mins[8]) {
    static const uint32_t kmask1 = 0x3f3f3f3f, kmask2 = 0x0f0f0f0f, kmask3 = 0x03030303;
    uint32_t utmp[4];
    memcpy(utmp, s12, 12);
    uint32_t mins8[2];
    mins8[0] = utmp[1] & kmask1;
    mins8[1] = ((utmp[2] >> 4) & kmask2) | (((utmp[1] >> 6) & kmask3) << 4);
    utmp[1] = (utmp[2] & kmask2) | (((utmp[0] >> 6) & kmask3) << 4);
    utmp[0] &= kmask1;
    memcpy(scales, utmp, 8);
    memcpy(mins, mins8, 8);
}

/* ------------------------------------------------------------ dequant [U] */
void kqo_dequantize_row_q4_K(const kqo_block_q4_K *x, float *y, int64_t k) {
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        const uint8_t *q = x[i].qs;
        const float d = kqo_fp16_to_fp32(x[i].d);
        const float min = kqo_fp16_to_fp32(x[i].dmin);
        int is = 0;
        uint8_t sc, m;
        for (int j = 0; j < QK_K; j += 64) {
            get_scale_min_k4(is + 0, x[i].scales, &sc, &m);
            const float d1 = d * sc, m1 = min * m;
            get_scale_min_k4(is + 1, x[i].scales, &sc, &m);
            const float d2 = d * sc, m2 = min * m;
            for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
            for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
            q += 32;
            is += 2;
        }
    }
}

void kqo_dequantize_row_q5_K(const kqo_block_q5_K *x, float *y, int64_t k) {
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        const uint8_t *ql = x[i].qs;
        const uint8_t *qh = x[i].qh;
        const float d = kqo_fp16_to_fp32(x[i].d);
        const float min = kqo_fp16_to_fp32(x[i].dmin);
        int is = 0;
        uint8_t sc, m;
        uint8_t u1 = 1, u2 = 2;
        for (int j = 0; j < QK_K; j += 64) {
            get_scale_min_k4(is + 0, x[i].scales, &sc, &m);
            const float d1 = d * sc, m1 = min * m;
            get_scale_min_k4(is + 1, x[i].scales, &sc, &m);
            const float d2 = d * sc, m2 = min * m;
            for (int l = 0; l < 32; ++l) *y++ = d1 * ((ql[l] & 0xF) + (qh[l] & u1 ? 16 : 0)) - m1;
            for (int l = 0; l < 32; ++l) *y++ = d2 * ((ql[l] >> 4) + (qh[l] & u2 ? 16 : 0)) - m2;
            ql += 32;
            is += 2;
            u1 <<= 2;
            u2 <<= 2;
        }
    }
}

void kqo_dequantize_row_q6_K(const kqo_block_q6_K *x, float *y, int64_t k) {
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        const float d = kqo_fp16_to_fp32(x[i].d);
        const uint8_t *ql = x[i].ql;
        const uint8_t *qh = x[i].qh;
        const int8_t *sc = x[i].scales;
        for (int n = 0; n < QK_K; n += 128) {
            for (int l = 0; l < 32; ++l) {
                int is = l / 16;
                const int8_t q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                const int8_t q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                const int8_t q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                const int8_t q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                y[l + 0] = d * sc[is + 0] * q1;
                y[l + 32] = d * sc[is + 2] * q2;
                y[l + 64] = d * sc[is + 4] * q3;
                y[l + 96] = d * sc[is + 6] * q4;
            }
            y += 128;
            ql += 64;
            qh += 32;
            sc += 8;
        }
    }
}

/* ----------------------------------------------------- Q4_K integer core */
/* Exact integer partials of one superblock, in the NEON listing's structure:
 *   summins = vaddvq_s32(prod): sum_{t<8} (bsums[2t]+bsums[2t+1]) * mins[t]  (README.md:730, 741-744)
 *   sumi    = sum_{j<4} dot(q4 lo, q8[64j..+32])*sc[2j] + dot(q4 hi, q8[64j+32..+32])*sc[2j+1]
 *             (README.md:754-771; int32 arithmetic is exact and associative) */
static inline void q4K_block_ints(const kqo_block_q4_K *x, const kqo_block_q8_K *y,
                                  int32_t *sumi_out, int32_t *summins_out) {
    uint8_t scales[8], mins[8];
    unpack_scales_neon(x->scales, scales, mins);
    int32_t summins = 0;
    for (int t = 0; t < 8; ++t)
        summins += (int32_t)(int16_t)(y->bsums[2 * t] + y->bsums[2 * t + 1]) * (int32_t)mins[t];
    const uint8_t *q4 = x->qs;
    const int8_t *q8 = y->qs;
    int32_t sumi1 = 0, sumi2 = 0;
    for (int j = 0; j < QK_K / 64; ++j) {
        int32_t p1 = 0, p2 = 0;
        for (int l = 0; l < 32; ++l) p1 += (int32_t)(q4[l] & 0xF) * q8[l];
        for (int l = 0; l < 32; ++l) p2 += (int32_t)(q4[l] >> 4) * q8[l + 32];
        sumi1 += p1 * scales[2 * j + 0];
        sumi2 += p2 * scales[2 * j + 1];
        q4 += 32;
        q8 += 64;
    }
    *sumi_out = sumi1 + sumi2;
    *summins_out = summins;
}

static void check_nrc(int nrc, const char *fn) {
    if (nrc != 1) {
        fprintf(stderr, "%s: nrc=%d unsupported (reference config has nrows=1)\n", fn, nrc);
        abort();
    }
}

void kqo_vec_dot_q4_K_q8_K_neon(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc) {
    (void)bs; (void)bx; (void)by;
    check_nrc(nrc, __func__);
    const kqo_block_q4_K *x = (const kqo_block_q4_K *)vx;
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / QK_K;
    float sumf = 0;
    for (int i = 0; i < nb; ++i) {
        /* d = y.d * fp16(x.d); dmin = y.d * fp16(x.dmin): README.md:727-728, :538-540 */
        const float d = y[i].d * kqo_fp16_to_fp32(x[i].d);
        const float dmin = y[i].d * kqo_fp16_to_fp32(x[i].dmin);
        int32_t sumi, summins;
        q4K_block_ints(&x[i], &y[i], &sumi, &summins);
        sumf = fmaf(-(float)summins, dmin, sumf); /* fmsub, README.md:551 */
        sumf = fmaf((float)sumi, d, sumf);        /* fmadd, README.md:614 */
    }
    *s = sumf;
}

/* Upstream ggml_vec_dot_q4_K_q8_K_generic [U]: 8 float lanes `sums[8]`, a
 * different (also contracted) fp32 order; integer content identical. */
void kqo_vec_dot_q4_K_q8_K_generic(int n, float *s, size_t bs, const void *vx, size_t bx,
                                   const void *vy, size_t by, int nrc) {
    (void)bs; (void)bx; (void)by;
    check_nrc(nrc, __func__);
    const kqo_block_q4_K *x = (const kqo_block_q4_K *)vx;
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / QK_K;
    int8_t aux8[QK_K];
    int16_t aux16[8];
    float sums[8];
    int32_t aux32[8];
    memset(sums, 0, sizeof(sums));
    float sumf = 0;
    for (int i = 0; i < nb; ++i) {
        const uint8_t *q4 = x[i].qs;
        const int8_t *q8 = y[i].qs;
        memset(aux32, 0, sizeof(aux32));
        int8_t *a = aux8;
        for (int j = 0; j < QK_K / 64; ++j) {
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] & 0xF);
            a += 32;
            for (int l = 0; l < 32; ++l) a[l] = (int8_t)(q4[l] >> 4);
            a += 32;
            q4 += 32;
        }
        uint8_t scales[8], mins[8];
        unpack_scales_neon(x[i].scales, scales, mins);
        int sumi = 0;
        for (int j = 0; j < QK_K / 16; ++j) sumi += y[i].bsums[j] * mins[j / 2];
        a = aux8;
        int is = 0;
        for (int j = 0; j < QK_K / 32; ++j) {
            int32_t scale = scales[is++];
            for (int q = 0; q < 4; ++q) {
                for (int l = 0; l < 8; ++l) aux16[l] = (int16_t)(q8[l] * a[l]);
                for (int l = 0; l < 8; ++l) aux32[l] += scale * aux16[l];
                q8 += 8;
                a += 8;
            }
        }
        const float d = kqo_fp16_to_fp32(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] = fmaf(d, (float)aux32[l], sums[l]);
        const float dmin = kqo_fp16_to_fp32(x[i].dmin) * y[i].d;
        sumf = fmaf(-dmin, (float)sumi, sumf);
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    *s = sumf;
}

/* ----------------------------------------------------------------- Q5_K */
static inline void q5K_block_ints(const kqo_block_q5_K *x, const kqo_block_q8_K *y,
                                  int32_t *sumi_out, int32_t *summins_out) {
    uint8_t scales[8], mins[8];
    unpack_scales_neon(x->scales, scales, mins);
    int32_t summins = 0;
    for (int t = 0; t < 8; ++t)
        summins += (int32_t)(int16_t)(y->bsums[2 * t] + y->bsums[2 * t + 1]) * (int32_t)mins[t];
    const uint8_t *q5 = x->qs;
    const int8_t *q8 = y->qs;
    int32_t sumi = 0;
    for (int j = 0; j < QK_K / 64; ++j) {
        int32_t p1 = 0, p2 = 0;
        for (int l = 0; l < 32; ++l) {
            const int hb1 = (x->qh[l] >> (2 * j)) & 1;
            const int hb2 = (x->qh[l] >> (2 * j + 1)) & 1;
            p1 += (int32_t)((q5[l] & 0xF) | (hb1 << 4)) * q8[l];
            p2 += (int32_t)((q5[l] >> 4) | (hb2 << 4)) * q8[l + 32];
        }
        sumi += p1 * scales[2 * j + 0];
        sumi += p2 * scales[2 * j + 1];
        q5 += 32;
        q8 += 64;
    }
    *sumi_out = sumi;
    *summins_out = summins;
}

/* [U] contraction choices the reference's listings do not show: 0 is the
 * restatement's choice (gcc -O2 -std=gnu11, whose default -ffp-contract=fast fuses a
 * single-use product into the add/sub it feeds, README.md:649-677's compile line); the
 * other values are the alternatives, selectable only here, so tests can measure how often
 * each would change an output (tests/test_oracle.py::test_unpinned_choice_flip_rates).
 *   which 0 (Q5_K update): 1 = fma(-dmin, mins, d*sumi); 2 = no fma; 3 = Q4_K's two fmas
 *   which 1 (Q6_K update): 1 = sum + (d_all*y.d)*f, unfused */
static int g_q5_variant = 0, g_q6_variant = 0;
void kqo_set_contraction_variant(int which, int v) {
    if (which == 0) g_q5_variant = v;
    else g_q6_variant = v;
}

/* NEON ggml_vec_dot_q5_K_q8_K [U]: `sumf += d * sumi - dmin * sumi_mins;`
 * Contraction as gcc's FMA pass forms it (first product fused into the
 * subtraction, the add to sumf unfused) — tolerance-only: parity unpinned. */
void kqo_vec_dot_q5_K_q8_K_neon(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc) {
    (void)bs; (void)bx; (void)by;
    check_nrc(nrc, __func__);
    const kqo_block_q5_K *x = (const kqo_block_q5_K *)vx;
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / QK_K;
    float sumf = 0;
    for (int i = 0; i < nb; ++i) {
        const float d = y[i].d * kqo_fp16_to_fp32(x[i].d);
        const float dmin = y[i].d * kqo_fp16_to_fp32(x[i].dmin);
        int32_t sumi, summins;
        q5K_block_ints(&x[i], &y[i], &sumi, &summins);
        if (g_q5_variant == 0) {
            const float t = fmaf(d, (float)sumi, -(dmin * (float)summins));
            sumf = sumf + t;
        } else if (g_q5_variant == 1) {
            const float t = fmaf(-dmin, (float)summins, d * (float)sumi);
            sumf = sumf + t;
        } else if (g_q5_variant == 2) {
            const float t = d * (float)sumi - dmin * (float)summins;
            sumf = sumf + t;
        } else {
            sumf = fmaf(-(float)summins, dmin, sumf);
            sumf = fmaf((float)sumi, d, sumf);
        }
    }
    *s = sumf;
}

/* ----------------------------------------------------------------- Q6_K */
static inline void q6K_block_ints(const kqo_block_q6_K *x, const kqo_block_q8_K *y,
                                  int32_t *isum_out, int32_t *isum_mins_out) {
    const int8_t *scale = x->scales;
    int32_t isum_mins = 0;
    for (int g = 0; g < 16; ++g) isum_mins += (int32_t)y->bsums[g] * (int32_t)scale[g];
    const uint8_t *q6 = x->ql;
    const uint8_t *qh = x->qh;
    const int8_t *q8 = y->qs;
    int32_t isum = 0;
    for (int j = 0; j < QK_K / 128; ++j) {
        for (int part = 0; part < 4; ++part) {
            /* part 0: ql[0..31]&F | qh bits0-1 ; 1: ql[32..63]&F | bits2-3 ;
             * 2: ql[0..31]>>4 | bits4-5 ; 3: ql[32..63]>>4 | bits6-7 */
            for (int half = 0; half < 2; ++half) {
                int32_t dot = 0;
                for (int l = 0; l < 16; ++l) {
                    const int li = half * 16 + l;
                    const uint8_t b = q6[(part & 1) * 32 + li];
                    const int lo = (part < 2) ? (b & 0xF) : (b >> 4);
                    const int hi = (qh[li] >> (2 * part)) & 3;
                    dot += (int32_t)(lo | (hi << 4)) * q8[part * 32 + li];
                }
                isum += dot * scale[part * 2 + half];
            }
        }
        q6 += 64;
        qh += 32;
        q8 += 128;
        scale += 8;
    }
    *isum_out = isum;
    *isum_mins_out = isum_mins;
}

/* NEON ggml_vec_dot_q6_K_q8_K [U]: `sum += d_all * y[i].d * (isum - 32 * isum_mins);`
 * contracted: fma(d_all*y.d, (float)(isum - 32*isum_mins), sum). */
void kqo_vec_dot_q6_K_q8_K_neon(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc) {
    (void)bs; (void)bx; (void)by;
    check_nrc(nrc, __func__);
    const kqo_block_q6_K *x = (const kqo_block_q6_K *)vx;
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / QK_K;
    float sum = 0;
    for (int i = 0; i < nb; ++i) {
        const float d_all = kqo_fp16_to_fp32(x[i].d);
        int32_t isum, isum_mins;
        q6K_block_ints(&x[i], &y[i], &isum, &isum_mins);
        if (g_q6_variant == 0) sum = fmaf(d_all * y[i].d, (float)(isum - 32 * isum_mins), sum);
        else sum = sum + (d_all * y[i].d) * (float)(isum - 32 * isum_mins);
    }
    *s = sum;
}

void kqo_vec_dot_q6_K_q8_K_generic(int n, float *s, size_t bs, const void *vx, size_t bx,
                                   const void *vy, size_t by, int nrc) {
    (void)bs; (void)bx; (void)by;
    check_nrc(nrc, __func__);
    const kqo_block_q6_K *x = (const kqo_block_q6_K *)vx;
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / QK_K;
    int8_t aux8[QK_K];
    int16_t aux16[8];
    float sums[8];
    int32_t aux32[8];
    memset(sums, 0, sizeof(sums));
    float sumf = 0;
    for (int i = 0; i < nb; ++i) {
        const uint8_t *q4 = x[i].ql;
        const uint8_t *qh = x[i].qh;
        const int8_t *q8 = y[i].qs;
        memset(aux32, 0, sizeof(aux32));
        int8_t *a = aux8;
        for (int j = 0; j < QK_K; j += 128) {
            for (int l = 0; l < 32; ++l) {
                a[l + 0] = (int8_t)((q4[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                a[l + 32] = (int8_t)((q4[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                a[l + 64] = (int8_t)((q4[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                a[l + 96] = (int8_t)((q4[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
            }
            a += 128;
            q4 += 64;
            qh += 32;
        }
        a = aux8;
        int is = 0;
        for (int j = 0; j < QK_K / 16; ++j) {
            int scale = x[i].scales[is++];
            for (int q = 0; q < 2; ++q) {
                for (int l = 0; l < 8; ++l) aux16[l] = (int16_t)(q8[l] * a[l]);
                for (int l = 0; l < 8; ++l) aux32[l] += scale * aux16[l];
                q8 += 8;
                a += 8;
            }
        }
        const float d = kqo_fp16_to_fp32(x[i].d) * y[i].d;
        for (int l = 0; l < 8; ++l) sums[l] = fmaf(d, (float)aux32[l], sums[l]);
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    *s = sumf;
}

void kqo_block_partials(int type, int n, const void *vx, const void *vy, int32_t *out) {
    const kqo_block_q8_K *y = (const kqo_block_q8_K *)vy;
    const int nb = n / QK_K;
    for (int i = 0; i < nb; ++i) {
        int32_t a = 0, b = 0;
        if (type == 12) q4K_block_ints((const kqo_block_q4_K *)vx + i, &y[i], &a, &b);
        else if (type == 13) q5K_block_ints((const kqo_block_q5_K *)vx + i, &y[i], &a, &b);
        else if (type == 14) q6K_block_ints((const kqo_block_q6_K *)vx + i, &y[i], &a, &b);
        out[2 * i] = a;
        out[2 * i + 1] = b;
    }
}

/* --------------------------------------------------- mul_mat (restated) */
typedef void (*vec_dot_fn)(int, float *, size_t, const void *, size_t, const void *, size_t, int);

static size_t type_size(int type) {
    return type == 12 ? sizeof(kqo_block_q4_K) : type == 13 ? sizeof(kqo_block_q5_K)
         : type == 14 ? sizeof(kqo_block_q6_K) : 0;
}

/* variant: 0 = NEON order (scalar), 1 = generic, 2 = NEON order with AVX2 integer
 * parts (kq_cpu_simd.c; bit-identical to 0). */
static vec_dot_fn pick_vec_dot(int type, int variant) {
    if (variant == 2) {
        if (type == 12) return kqo_vec_dot_q4_K_q8_K_simd;
        if (type == 13) return kqo_vec_dot_q5_K_q8_K_simd;
        if (type == 14) return kqo_vec_dot_q6_K_q8_K_simd;
        return NULL;
    }
    if (type == 12) return variant ? kqo_vec_dot_q4_K_q8_K_generic : kqo_vec_dot_q4_K_q8_K_neon;
    if (type == 13) return kqo_vec_dot_q5_K_q8_K_neon;
    if (type == 14) return variant ? kqo_vec_dot_q6_K_q8_K_generic : kqo_vec_dot_q6_K_q8_K_neon;
    return NULL;
}

typedef struct {
    const char *src0; int64_t K, N; size_t nb01;
    const float *src1; size_t nb11; int64_t M;
    kqo_block_q8_K *wdata; int quantize;
    float *dst; vec_dot_fn vec_dot;
    int nth; atomic_int current_chunk;
    atomic_int arrived; /* ggml_barrier: threads past the quantization */
    /* generic parallel-for (kqo_pool_run): tasks handed out by current_chunk */
    void (*task_fn)(void *ctx, int task); void *task_ctx; int n_tasks;
} mm_plan;

typedef struct { mm_plan *p; int ith; } mm_arg;

/* ggml_compute_forward_mul_mat_one_chunk (ggml-cpu.c:1194): 16x16 blocking,
 * tmp[32], vec_dot per (row, col), memcpy of the 16-row strip into dst. */
static void mm_one_chunk(mm_plan *p, int64_t ir0_start, int64_t ir0_end, int64_t ir1_start,
                         int64_t ir1_end) {
    const int64_t nbq = p->K / QK_K;
    const size_t row_size = (size_t)nbq * sizeof(kqo_block_q8_K);
    const int64_t blck_0 = 16, blck_1 = 16;
    float tmp[32];
    for (int64_t iir1 = ir1_start; iir1 < ir1_end; iir1 += blck_1) {
        for (int64_t iir0 = ir0_start; iir0 < ir0_end; iir0 += blck_0) {
            for (int64_t ir1 = iir1; ir1 < iir1 + blck_1 && ir1 < ir1_end; ++ir1) {
                const char *src1_col = (const char *)p->wdata + ir1 * row_size;
                float *dst_col = p->dst + ir1 * p->N;
                int64_t ir0;
                for (ir0 = iir0; ir0 < iir0 + blck_0 && ir0 < ir0_end; ++ir0)
                    p->vec_dot((int)p->K, &tmp[ir0 - iir0], 0, p->src0 + ir0 * p->nb01, 0, src1_col, 0, 1);
                memcpy(&dst_col[iir0], tmp, (size_t)(ir0 - iir0) * sizeof(float));
            }
        }
    }
}

static void *mm_thread(void *arg) {
    mm_arg *a = (mm_arg *)arg;
    mm_plan *p = a->p;
    const int ith = a->ith, nth = p->nth;
    if (p->task_fn) { /* generic tasks: an atomic counter, no barrier */
        for (int t = atomic_fetch_add(&p->current_chunk, 1); t < p->n_tasks; t = atomic_fetch_add(&p->current_chunk, 1))
            p->task_fn(p->task_ctx, t);
        return NULL;
    }
    const int64_t nbq = p->K / QK_K;
    if (p->quantize) { /* every thread quantizes its block slice of every src1 row */
        for (int64_t i11 = 0; i11 < p->M; ++i11) {
            const int64_t b0 = (ith * nbq) / nth, b1 = ((ith + 1) * nbq) / nth;
            if (b1 > b0)
                kqo_quantize_row_q8_K((const float *)((const char *)p->src1 + i11 * p->nb11) + b0 * QK_K,
                                      p->wdata + i11 * nbq + b0, (b1 - b0) * QK_K, 1);
        }
    }
    if (ith == 0) atomic_store(&p->current_chunk, nth);
    /* ggml_barrier (spin): every src1 slice quantized before any chunk runs */
    atomic_fetch_add(&p->arrived, 1);
    for (int spins = 0; atomic_load(&p->arrived) < nth;)
        if (++spins < (1 << 16)) __builtin_ia32_pause();
        else sched_yield(); /* oversubscribed host: let the straggler run */

    const int64_t nr0 = p->N, nr1 = p->M;
    int64_t chunk_size = (nr0 == 1 || nr1 == 1) ? 64 : 16;
    int64_t nchunk0 = (nr0 + chunk_size - 1) / chunk_size;
    int64_t nchunk1 = (nr1 + chunk_size - 1) / chunk_size;
    if (nchunk0 * nchunk1 < nth * 4) {
        nchunk0 = nr0 > nr1 ? nth : 1;
        nchunk1 = nr0 > nr1 ? 1 : nth;
    }
    const int64_t dr0 = (nr0 + nchunk0 - 1) / nchunk0;
    const int64_t dr1 = (nr1 + nchunk1 - 1) / nchunk1;
    int64_t current_chunk = ith;
    while (current_chunk < nchunk0 * nchunk1) {
        const int64_t ith0 = current_chunk % nchunk0, ith1 = current_chunk / nchunk0;
        const int64_t ir0_start = dr0 * ith0, ir0_end = ir0_start + dr0 < nr0 ? ir0_start + dr0 : nr0;
        const int64_t ir1_start = dr1 * ith1, ir1_end = ir1_start + dr1 < nr1 ? ir1_start + dr1 : nr1;
        mm_one_chunk(p, ir0_start, ir0_end, ir1_start, ir1_end);
        if (nth >= nchunk0 * nchunk1) break;
        current_chunk = atomic_fetch_add(&p->current_chunk, 1);
    }
    return NULL;
}

/* Persistent worker pool, as ggml's threadpool: workers are created once per
 * thread count and spin (then yield) on a generation counter between graph nodes,
 * so a mul_mat call costs no thread creation. The caller is ith 0. */
static struct {
    int nth;
    pthread_t th[256];
    mm_arg args[256];
    atomic_int gen, done, quit;
    mm_plan *volatile plan;
} g_pool;
static pthread_mutex_t g_pool_mu = PTHREAD_MUTEX_INITIALIZER;

static void *pool_worker(void *arg) {
    mm_arg *a = (mm_arg *)arg;
    int seen = 0;
    for (;;) {
        int spins = 0, g;
        while ((g = atomic_load(&g_pool.gen)) == seen && !atomic_load(&g_pool.quit)) {
            if (++spins < 20000) __builtin_ia32_pause();
            else sched_yield();
        }
        if (atomic_load(&g_pool.quit)) return NULL;
        seen = g;
        a->p = g_pool.plan;
        mm_thread(a);
        atomic_fetch_add(&g_pool.done, 1);
    }
}

static void pool_resize(int nth) {
    if (g_pool.nth == nth) return;
    if (g_pool.nth > 1) {
        atomic_store(&g_pool.quit, 1);
        for (int t = 1; t < g_pool.nth; ++t) pthread_join(g_pool.th[t], NULL);
    }
    atomic_store(&g_pool.quit, 0);
    atomic_store(&g_pool.gen, 0);
    g_pool.nth = nth;
    for (int t = 1; t < nth; ++t) {
        g_pool.args[t].ith = t;
        pthread_create(&g_pool.th[t], NULL, pool_worker, &g_pool.args[t]);
    }
}

static int mm_run(mm_plan *p, int n_threads) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    p->nth = n_threads;
    atomic_init(&p->current_chunk, 0);
    atomic_init(&p->arrived, 0);
    mm_arg a0 = {p, 0};
    if (n_threads == 1) {
        mm_thread(&a0);
        return 0;
    }
    pthread_mutex_lock(&g_pool_mu); /* one graph node at a time per process */
    pool_resize(n_threads);
    g_pool.plan = p;
    atomic_store(&g_pool.done, 0);
    atomic_fetch_add(&g_pool.gen, 1);
    mm_thread(&a0); /* main thread is ith 0, as in ggml_graph_compute */
    for (int spins = 0; atomic_load(&g_pool.done) < n_threads - 1;)
        if (++spins < (1 << 16)) __builtin_ia32_pause();
        else sched_yield();
    pthread_mutex_unlock(&g_pool_mu);
    return 0;
}

void kqo_pool_run(int n_threads, int n_tasks, void (*fn)(void *ctx, int task), void *ctx) {
    mm_plan p;
    memset(&p, 0, sizeof(p));
    p.task_fn = fn;
    p.task_ctx = ctx;
    p.n_tasks = n_tasks;
    mm_run(&p, n_threads < n_tasks ? n_threads : (n_tasks > 0 ? n_tasks : 1));
}

int kqo_mul_mat(int type, const void *src0, int64_t K, int64_t N, size_t nb01,
                const float *src1, int64_t M, size_t nb11, float *dst, int n_threads, int variant) {
    if (K <= 0 || K % QK_K || N < 0 || M < 0 || !type_size(type)) return -1;
    if (N == 0 || M == 0) return 0;
    mm_plan p;
    memset(&p, 0, sizeof(p));
    p.src0 = (const char *)src0; p.K = K; p.N = N; p.nb01 = nb01;
    p.src1 = src1; p.nb11 = nb11; p.M = M; p.dst = dst;
    p.vec_dot = pick_vec_dot(type, variant);
    p.wdata = (kqo_block_q8_K *)malloc((size_t)M * (size_t)(K / QK_K) * sizeof(kqo_block_q8_K));
    if (!p.wdata) return -1;
    p.quantize = 1;
    mm_run(&p, n_threads);
    free(p.wdata);
    return 0;
}

int kqo_mul_mat_q8(int type, const void *src0, int64_t K, int64_t N, size_t nb01,
                   const void *src1_q8, int64_t M, float *dst, int n_threads, int variant) {
    if (K <= 0 || K % QK_K || N < 0 || M < 0 || !type_size(type)) return -1;
    if (N == 0 || M == 0) return 0;
    mm_plan p;
    memset(&p, 0, sizeof(p));
    p.src0 = (const char *)src0; p.K = K; p.N = N; p.nb01 = nb01;
    p.M = M; p.dst = dst;
    p.vec_dot = pick_vec_dot(type, variant);
    p.wdata = (kqo_block_q8_K *)src1_q8;
    p.quantize = 0;
    mm_run(&p, n_threads);
    return 0;
}
