/*
 * kq_ops_oracle.c — CPU ORACLE for the non-matmul decode ops of the llama graph
 * (rms_norm, mul/add, rope, f16 attention vec_dot,
 * soft_max, swiglu, set_rows, get_rows).
 *
 * TEST INFRASTRUCTURE ONLY (same contract as kq_oracle.c): used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker; never
 * linked into or called by the product path (ggml-neon-opt_amd/).
 *
 * The reference's profile shows which ggml-cpu functions run for these ops in
 * the measured tg128 (artifacts/perf/out.folded, un-vendored llama.cpp @ a3cb0474):
 *   get_rows  -> dequantize_row_q4_K                          out.folded:103-104
 *   swiglu    -> ggml_compute_forward_glu -> ggml_vec_swiglu_f32  :107-113
 *   mul       -> binary_op<op_mul> / apply_binary_op          :115-121
 *   add       -> binary_op<op_add>                            :91-99
 *   KQ / KQV  -> mul_mat_one_chunk -> ggml_vec_dot_f16 (vfmaq_f16, NEON FP16
 *                arithmetic: f16 accumulators)                :140-144
 *   src1->f16 -> ggml_cpu_fp32_to_fp16                        :176-178
 *   rms_norm  -> ggml_compute_forward_rms_norm_f32            :189-193
 *   rope      -> ggml_compute_forward_rope_f32, ggml_rope_cache_init, rope_yarn :196-208
 *   set_rows  -> ggml_compute_forward_set_rows_f32 (f32 -> f16 cache rows) :209-215
 *   soft_max  -> ggml_compute_forward_soft_max_f32, ggml_vec_soft_max_f32,
 *                ggml_v_expf (its slow path: vclezq_f32)      :216-234
 *   graph     -> llm_build_llama                              :249-251
 * The bodies are restated from upstream ggml-cpu at that build [U] (the source is
 * not in /root/reference): parity unpinned, as for the rest of the oracle.
 * Compiler contraction of the aarch64 gcc build (-std=gnu*: -ffp-contract=fast)
 * is written out with fmaf() where gcc fuses a multiply into an add [U]:
 * dequantize `d1*q - m1` -> fmaf(d1, q, -m1); rope `x0*c - x1*s` ->
 * fmaf(x0, c, -(x1*s)) and `x0*s + x1*c` -> fmaf(x0, s, x1*c) (the first product
 * of the expression is fused). NEON intrinsics keep their own fusion (vfmaq).
 *
 * f16 arithmetic (vfmaq_f16 / vaddq_f16) is computed exactly here: f16 operands
 * are integers times 2^-24, so a*b + c is an exact integer times 2^-48 held in
 * 128 bits, rounded once to binary16 (nearest-even, subnormals, overflow to inf).
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "kq_oracle.h"

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* ------------------------------------------------------------ exact binary16 */
/* finite f16 -> (sign, value in units of 2^-24) */
static inline int64_t f16_fixed24(uint16_t h) {
    const int64_t e = (h >> 10) & 0x1f, m = h & 0x3ff;
    const int64_t mag = e == 0 ? m : (m | 0x400) << (e - 1);
    return (h & 0x8000) ? -mag : mag;
}

static inline int clz128(unsigned __int128 u) {
    const uint64_t hi = (uint64_t)(u >> 64), lo = (uint64_t)u;
    return hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);
}

/* Round v * 2^-48 to binary16 (RNE). `neg_zero`: sign of an exact zero. */
static uint16_t f16_round48(__int128 v, int neg_zero) {
    if (v == 0) return neg_zero ? 0x8000 : 0;
    uint16_t sign = 0;
    if (v < 0) { sign = 0x8000; v = -v; }
    const unsigned __int128 u = (unsigned __int128)v;
    int e = (127 - clz128(u)) - 48;  /* floor(log2(value)) */
    if (e < -14) e = -14;            /* subnormal quantum 2^-24 */
    const int shift = e + 38;        /* quantum 2^(e-10) in units of 2^-48 */
    unsigned __int128 q = u >> shift;
    const unsigned __int128 rem = u & (((unsigned __int128)1 << shift) - 1);
    const unsigned __int128 half = (unsigned __int128)1 << (shift - 1);
    if (rem > half || (rem == half && (q & 1))) q++;
    if (q >= 2048) { q >>= 1; e++; }
    if (e > 15) return sign | 0x7c00;
    if (q < 1024) return sign | (uint16_t)q; /* subnormal */
    return sign | (uint16_t)(((e + 15) << 10) | (int)(q - 1024));
}

/* vfmaq_f16(c, a, b) lane: c + a*b, one rounding */
uint16_t kqo_f16_fma(uint16_t a, uint16_t b, uint16_t c) {
    const __int128 p = (__int128)f16_fixed24(a) * f16_fixed24(b);
    const __int128 s = p + ((__int128)f16_fixed24(c) << 24);
    const int pneg = ((a ^ b) & 0x8000) != 0, cneg = (c & 0x8000) != 0;
    return f16_round48(s, p == 0 && f16_fixed24(c) == 0 && pneg && cneg);
}

/* vaddq_f16 lane */
uint16_t kqo_f16_add(uint16_t a, uint16_t b) {
    const __int128 s = ((__int128)f16_fixed24(a) + f16_fixed24(b)) << 24;
    return f16_round48(s, (a & 0x8000) && (b & 0x8000) && f16_fixed24(a) == 0 && f16_fixed24(b) == 0);
}

/* ggml_cpu_fp32_to_fp16 (out.folded:176): row conversion, NEON vcvt = RNE */
void kqo_fp32_to_fp16_row(const float *x, uint16_t *y, int64_t n) {
    for (int64_t i = 0; i < n; ++i) y[i] = kqo_fp32_to_fp16(x[i]);
}

/* ggml_vec_dot_f16, NEON FP16 path (GGML_F16_STEP 32, GGML_F16_EPR 8: four f16x8
 * accumulators, vfmaq_f16), GGML_F16_VEC_REDUCE (sum[0]+=sum[2], sum[1]+=sum[3],
 * sum[0]+=sum[1] in f16, then vcvt to f32 halves, vaddq_f32, vaddvq_f32 =
 * (t0+t1)+(t2+t3)) into ggml_float; leftovers in ggml_float; *s = (float)sumf.
 * out.folded:140-144. */
float kqo_vec_dot_f16(int n, const uint16_t *x, const uint16_t *y) {
    const int np = n & ~31;
    uint16_t sum[4][8];
    memset(sum, 0, sizeof(sum));
    for (int i = 0; i < np; i += 32)
        for (int j = 0; j < 4; ++j)
            for (int l = 0; l < 8; ++l)
                sum[j][l] = kqo_f16_fma(x[i + 8 * j + l], y[i + 8 * j + l], sum[j][l]);
    for (int l = 0; l < 8; ++l) {
        sum[0][l] = kqo_f16_add(sum[0][l], sum[2][l]);
        sum[1][l] = kqo_f16_add(sum[1][l], sum[3][l]);
    }
    for (int l = 0; l < 8; ++l) sum[0][l] = kqo_f16_add(sum[0][l], sum[1][l]);
    float t[4];
    for (int k = 0; k < 4; ++k) t[k] = kqo_fp16_to_fp32(sum[0][k]) + kqo_fp16_to_fp32(sum[0][k + 4]);
    double sumf = (double)((t[0] + t[1]) + (t[2] + t[3]));
    for (int i = np; i < n; ++i) sumf += (double)(kqo_fp16_to_fp32(x[i]) * kqo_fp16_to_fp32(y[i]));
    return (float)sumf;
}

/* ------------------------------------------------------------ exp / silu */
/* one lane of ggml_v_expf (NEON, ggml-cpu vec.h [U]); vfmaq_f32(a,b,c) = fmaf(b,c,a),
 * vfmsq_f32(a,b,c) = fmaf(-b,c,a), vcagtq = |.|>, vclezq = <= 0 (out.folded:218). */
float kqo_v_expf(float x) {
    const float r = 0x1.8p23f;
    const float z = fmaf(x, 0x1.715476p+0f, r);
    const float n = z - r;
    const float b = fmaf(-n, 0x1.7f7d1cp-20f, fmaf(-n, 0x1.62e4p-1f, x));
    const uint32_t e = f2u(z) << 23;
    const float k = u2f(e + f2u(1.0f));
    const int c = fabsf(n) > 126.0f;
    const float u = b * b;
    const float j = fmaf(fmaf(fmaf(0x1.0e4020p-7f, b, 0x1.573e2ep-5f), u, fmaf(0x1.555e66p-3f, b, 0x1.fffdb6p-2f)), u,
                         0x1.ffffecp-1f * b);
    if (!c) return fmaf(k, j, k);
    const uint32_t d = n <= 0.0f ? 0x82000000u : 0u;
    const float s1 = u2f(d + 0x7f000000u);
    const float s2 = u2f(e - d);
    if (fabsf(n) > 192.0f) return s1 * s1;
    return fmaf(s2, j, s2) * s1;
}

/* ggml_v_silu lane: x / (1 + v_expf(0 - x)) */
static inline float v_silu(float x) { return x / (1.0f + kqo_v_expf(0.0f - x)); }

/* ggml_vec_swiglu_f32 (out.folded:107-113): NEON body for i+3 < n, scalar tail
 * ggml_silu_f32(x) = x/(1.0f+expf(-x)) (libm). y = silu(x) * g. */
void kqo_vec_swiglu_f32(int n, float *y, const float *x, const float *g) {
    int i = 0;
    for (; i + 3 < n; i += 4)
        for (int k = 0; k < 4; ++k) y[i + k] = v_silu(x[i + k]) * g[i + k];
    for (; i < n; ++i) y[i] = (x[i] / (1.0f + expf(-x[i]))) * g[i];
}

/* ggml_compute_forward_soft_max_f32 for one row (out.folded:216-234): wp = sp*scale
 * (ggml_vec_scale_f32), wp += slope*mask (slope 1: max_bias 0), max (ggml_vec_max_f32),
 * ggml_vec_soft_max_f32 (NEON: 4 lanes of v_expf(x-max), sum += (ggml_float)vaddvq_f32;
 * scalar tail expf), sum = 1.0/sum, ggml_vec_scale_f32(dp, (float)sum). */
void kqo_soft_max_row(int n, float *dp, const float *sp, const float *mask, float scale) {
    float max = -INFINITY;
    for (int i = 0; i < n; ++i) {
        float w = sp[i] * scale;
        if (mask) w += mask[i];
        dp[i] = w;
        max = max > w ? max : w;  /* MAX(max, x[i]) */
    }
    double sum = 0.0;
    int i = 0;
    for (; i + 3 < n; i += 4) {
        float v[4];
        for (int k = 0; k < 4; ++k) v[k] = kqo_v_expf(dp[i + k] - max);
        for (int k = 0; k < 4; ++k) dp[i + k] = v[k];
        sum += (double)((v[0] + v[1]) + (v[2] + v[3]));
    }
    for (; i < n; ++i) {
        const float v = expf(dp[i] - max);
        sum += (double)v;
        dp[i] = v;
    }
    sum = 1.0 / sum;
    const float inv = (float)sum;
    for (int k = 0; k < n; ++k) dp[k] *= inv;
}

/* ------------------------------------------------------------ norm / binary */
/* ggml_compute_forward_rms_norm_f32 (out.folded:189-193): sum += (ggml_float)(x*x)
 * sequentially, mean = sum/ne00 (to float), y = x * (1.0f/sqrtf(mean + eps)). */
void kqo_rms_norm_f32(const float *x, float *y, int64_t n, float eps) {
    double sum = 0.0;
    for (int64_t i = 0; i < n; ++i) sum += (double)(x[i] * x[i]);
    const float mean = (float)(sum / (double)n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int64_t i = 0; i < n; ++i) y[i] = x[i] * scale;
}

void kqo_mul_f32(const float *a, const float *b, float *y, int64_t n) {
    for (int64_t i = 0; i < n; ++i) y[i] = a[i] * b[i];
}

void kqo_add_f32(const float *a, const float *b, float *y, int64_t n) {
    for (int64_t i = 0; i < n; ++i) y[i] = a[i] + b[i];
}

/* ------------------------------------------------------------ rope (NORM mode) */
/* theta_scale = powf(freq_base, -2.0f/n_dims) (ggml_compute_forward_rope_f32). */
float kqo_rope_theta_scale(float freq_base, int n_dims) { return powf(freq_base, -2.0f / (float)n_dims); }

/* ggml_rope_cache_init + rope_yarn with ext_factor 0, attn_factor (mscale) 1, no
 * freq_factors, sin_sign 1 (out.folded:201-208): theta = p; per pair i0:
 * cos = cosf(freq_scale*theta)*1, sin = sinf(...)*1; theta *= theta_scale.
 * table[(p*(n_dims/2) + i)*2 + {0,1}] = {cos, sin} for p in [0, n_pos). */
void kqo_rope_table(float *table, int n_pos, int n_dims, float freq_base, float freq_scale) {
    const float theta_scale = kqo_rope_theta_scale(freq_base, n_dims);
    for (int p = 0; p < n_pos; ++p) {
        float theta = (float)p;
        for (int i = 0; i < n_dims / 2; ++i) {
            const float t = freq_scale * theta;
            table[((int64_t)p * (n_dims / 2) + i) * 2 + 0] = cosf(t) * 1.0f;
            table[((int64_t)p * (n_dims / 2) + i) * 2 + 1] = sinf(t) * 1.0f;
            theta *= theta_scale;
        }
    }
}

/* rotate_pairs<float>(n_dims, 1, cache, ...) for GGML_ROPE_TYPE_NORMAL, one token,
 * n_heads rows of head_dim floats; dims >= n_dims copied. */
void kqo_rope_norm(const float *x, float *y, int head_dim, int n_dims, int n_heads, int pos, const float *table) {
    const float *c = table + (int64_t)pos * (n_dims / 2) * 2;
    for (int h = 0; h < n_heads; ++h) {
        const float *s = x + (int64_t)h * head_dim;
        float *d = y + (int64_t)h * head_dim;
        for (int i0 = 0; i0 < n_dims; i0 += 2) {
            const float ct = c[i0], st = c[i0 + 1];
            const float x0 = s[i0], x1 = s[i0 + 1];
            d[i0] = fmaf(x0, ct, -(x1 * st));
            d[i0 + 1] = fmaf(x0, st, x1 * ct);
        }
        for (int i0 = n_dims; i0 < head_dim; ++i0) d[i0] = s[i0];
    }
}

/* ------------------------------------------------------------ get_rows */
/* ggml_compute_forward_get_rows_q -> dequantize_row_q4_K (out.folded:103-104) with
 * gcc's contraction y = fmaf(d1, q, -m1) [U]; Q6_K: y = d*sc*q (no add: nothing to
 * fuse); F32 rows copied. */
static inline void scale_min_k4(int j, const uint8_t *q, uint8_t *d, uint8_t *m) {
    if (j < 4) {
        *d = q[j] & 63;
        *m = q[j + 4] & 63;
    } else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

void kqo_get_rows(int type, const void *table, int64_t k, size_t row_stride, const int32_t *ids, int64_t n_ids,
                  float *out) {
    for (int64_t r = 0; r < n_ids; ++r) {
        const uint8_t *row = (const uint8_t *)table + (int64_t)ids[r] * row_stride;
        float *y = out + r * k;
        if (type == 0) {
            memcpy(y, row, (size_t)k * 4);
        } else if (type == 12) {
            const kqo_block_q4_K *x = (const kqo_block_q4_K *)row;
            for (int64_t i = 0; i < k / 256; i++) {
                const uint8_t *q = x[i].qs;
                const float d = kqo_fp16_to_fp32(x[i].d), min = kqo_fp16_to_fp32(x[i].dmin);
                int is = 0;
                uint8_t sc, m;
                for (int j = 0; j < 256; j += 64) {
                    scale_min_k4(is + 0, x[i].scales, &sc, &m);
                    const float d1 = d * sc, m1 = min * m;
                    scale_min_k4(is + 1, x[i].scales, &sc, &m);
                    const float d2 = d * sc, m2 = min * m;
                    for (int l = 0; l < 32; ++l) *y++ = fmaf(d1, (float)(q[l] & 0xF), -m1);
                    for (int l = 0; l < 32; ++l) *y++ = fmaf(d2, (float)(q[l] >> 4), -m2);
                    q += 32;
                    is += 2;
                }
            }
        } else if (type == 13) {  /* dequantize_row_q5_K [U], the same contraction as Q4_K */
            const kqo_block_q5_K *x = (const kqo_block_q5_K *)row;
            for (int64_t i = 0; i < k / 256; i++) {
                const uint8_t *ql = x[i].qs, *qh = x[i].qh;
                const float d = kqo_fp16_to_fp32(x[i].d), min = kqo_fp16_to_fp32(x[i].dmin);
                int is = 0;
                uint8_t sc, m, u1 = 1, u2 = 2;
                for (int j = 0; j < 256; j += 64) {
                    scale_min_k4(is + 0, x[i].scales, &sc, &m);
                    const float d1 = d * sc, m1 = min * m;
                    scale_min_k4(is + 1, x[i].scales, &sc, &m);
                    const float d2 = d * sc, m2 = min * m;
                    for (int l = 0; l < 32; ++l) *y++ = fmaf(d1, (float)((ql[l] & 0xF) + (qh[l] & u1 ? 16 : 0)), -m1);
                    for (int l = 0; l < 32; ++l) *y++ = fmaf(d2, (float)((ql[l] >> 4) + (qh[l] & u2 ? 16 : 0)), -m2);
                    ql += 32;
                    is += 2;
                    u1 <<= 2;
                    u2 <<= 2;
                }
            }
        } else if (type == 14) {
            kqo_dequantize_row_q6_K((const kqo_block_q6_K *)row, y, k);
        }
    }
}

/* ------------------------------------------------------------ attention (decode) */
/* The non-flash-attention block of llm_build_llama (out.folded:249) for ONE token at
 * position `pos`, one sequence:
 *   Kcur/Vcur rows -> f16 cache cells (set_rows, out.folded:209-215): K row-major
 *   [cell][n_head_kv*hd], V transposed [n_head_kv*hd][n_ctx] (non-FA v_trans);
 *   q -> f16 (ggml_cpu_fp32_to_fp16, src1 of the KQ mul_mat);
 *   kq[h][c] = vec_dot_f16(k_cache[c][g], q16[h]), g = h / (n_head/n_head_kv);
 *   soft_max_ext(kq, mask, scale) with mask 0 for c <= pos, -INF above, over n_kv cells;
 *   kqv[h][d] = vec_dot_f16(v_cache[g*hd+d][0..n_kv), f16(kq_soft[h]));
 *   out[h*hd + d] (permute + cont). q, k must already be roped.
 * n_kv = min(n_ctx, max(32, GGML_PAD(pos+1, 32))) (kv-cache padding 32 without flash
 * attention [U]). */
int kqo_attn_n_kv(int pos, int n_ctx) {
    int n = (pos + 1 + 31) / 32 * 32;
    if (n < 32) n = 32;
    return n < n_ctx ? n : n_ctx;
}

void kqo_attn_decode(const float *q, const float *k, const float *v, uint16_t *k_cache, uint16_t *v_cache, int pos,
                     int n_ctx, int n_head, int n_head_kv, int head_dim, float scale, float *out) {
    const int kvw = n_head_kv * head_dim;
    kqo_fp32_to_fp16_row(k, k_cache + (int64_t)pos * kvw, kvw);
    for (int ch = 0; ch < kvw; ++ch) v_cache[(int64_t)ch * n_ctx + pos] = kqo_fp32_to_fp16(v[ch]);
    const int n_kv = kqo_attn_n_kv(pos, n_ctx);
    const int gsz = n_head / n_head_kv;
    uint16_t q16[512];
    float kq[8192], mask[8192];
    uint16_t p16[8192];
    for (int c = 0; c < n_kv; ++c) mask[c] = c <= pos ? 0.0f : -INFINITY;
    for (int h = 0; h < n_head; ++h) {
        const int g = h / gsz;
        kqo_fp32_to_fp16_row(q + (int64_t)h * head_dim, q16, head_dim);
        for (int c = 0; c < n_kv; ++c)
            kq[c] = kqo_vec_dot_f16(head_dim, k_cache + (int64_t)c * kvw + (int64_t)g * head_dim, q16);
        kqo_soft_max_row(n_kv, kq, kq, mask, scale);
        kqo_fp32_to_fp16_row(kq, p16, n_kv);
        for (int d = 0; d < head_dim; ++d)
            out[(int64_t)h * head_dim + d] =
                kqo_vec_dot_f16(n_kv, v_cache + (int64_t)(g * head_dim + d) * n_ctx, p16);
    }
}
