// kq_ops_device.h — device arithmetic of the non-matmul decode ops, written to give
// the same bits as ggml-cpu's aarch64 build (restated for the tests on the CPU side):
//   * ggml_v_expf (NEON) lane by lane: same constants, same fused ops (vfmaq_f32 ->
//     fmaf, vfmsq_f32 -> fmaf(-b, c, a)), same integer exponent tricks;
//   * ggml_v_silu: x / (1 + v_expf(0 - x)) with a correctly rounded divide;
//   * binary16 FMA / add (vfmaq_f16 / vaddq_f16) on the f16 ALU (v_fma_f16, v_add_f16:
//     IEEE, one rounding, f16 denormals kept);
//   * the RMS-norm sum of squares: a fast FIXED order shared by every kernel that
//     computes it (kq_rms_norm and the kq_rows norm prologue): per 16 consecutive
//     elements a sequential double sum, a balanced tree over the 16 groups of a
//     256-element superblock, then superblocks in order. ggml sums sequentially in
//     double (ggml_compute_forward_rms_norm_f32); the two orders can differ only in
//     the last bits of the double, which reach the float mean only when it lies
//     within ~2^-40 (relative) of a rounding boundary — detected exactly
//     (rms_mean_ambiguous), and then the sum is redone in ggml's sequential order,
//     so the float mean is the reference's in every case.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kq {

__device__ __forceinline__ float v_expf(float x) {
    const float r = 0x1.8p23f;
    const float z = __builtin_fmaf(x, 0x1.715476p+0f, r);
    const float n = z - r;
    const float b = __builtin_fmaf(-n, 0x1.7f7d1cp-20f, __builtin_fmaf(-n, 0x1.62e4p-1f, x));
    const uint32_t e = __float_as_uint(z) << 23;
    const float k = __uint_as_float(e + 0x3f800000u);
    const float u = b * b;
    const float j = __builtin_fmaf(
        __builtin_fmaf(__builtin_fmaf(0x1.0e4020p-7f, b, 0x1.573e2ep-5f), u, __builtin_fmaf(0x1.555e66p-3f, b, 0x1.fffdb6p-2f)),
        u, 0x1.ffffecp-1f * b);
    const float an = __builtin_fabsf(n);
    if (!(an > 126.0f)) return __builtin_fmaf(k, j, k);
    const uint32_t d = n <= 0.0f ? 0x82000000u : 0u;
    const float s1 = __uint_as_float(d + 0x7f000000u);
    const float s2 = __uint_as_float(e - d);
    if (an > 192.0f) return s1 * s1;
    return __builtin_fmaf(s2, j, s2) * s1;
}

__device__ __forceinline__ float v_silu(float x) { return x / (1.0f + v_expf(0.0f - x)); }

// rotate_pairs (GGML_ROPE_TYPE_NORMAL) with the position's cos/sin row of the table;
// x0*c - x1*s -> fmaf(x0, c, -(x1*s)), x0*s + x1*c -> fmaf(x0, s, x1*c) [U].
__device__ __forceinline__ float2 rope_pair(float x0, float x1, float c, float s) {
    return make_float2(__builtin_fmaf(x0, c, -(x1 * s)), __builtin_fmaf(x0, s, x1 * c));
}

typedef _Float16 h16;

__device__ __forceinline__ h16 hfma(h16 a, h16 b, h16 c) { return __builtin_fmaf16(a, b, c); }
__device__ __forceinline__ h16 u2h(uint16_t u) { return __builtin_bit_cast(h16, u); }
__device__ __forceinline__ uint16_t h2u(h16 h) { return __builtin_bit_cast(uint16_t, h); }
// f32 -> f16 round-to-nearest-even (v_cvt_f16_f32) of an f32 VALUE: the asm pin keeps
// the compiler from folding the producing f32 op into a mixed-precision instruction
// (v_fma_mixlo_f16 rounds the exact result to f16 once; ggml rounds to f32 first).
__device__ __forceinline__ h16 f2h_rne(float f) {
    asm volatile("" : "+v"(f));
    return (h16)f;
}

// GGML_F16_VEC_REDUCE tail: 8 f16 lanes (after sum[0]+=sum[2], sum[1]+=sum[3],
// sum[0]+=sum[1]) -> vcvt halves, vaddq_f32, vaddvq_f32 = (t0+t1)+(t2+t3).
__device__ __forceinline__ float f16x8_reduce(const h16 s[8]) {
    float t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = (float)s[k] + (float)s[k + 4];
    return (t[0] + t[1]) + (t[2] + t[3]);
}

// Two f16 lanes per 32-bit word: one v_pk_fma_f16 runs the NEON lanes 2k and 2k+1 (each
// half an IEEE f16 fma, the scalar v_fma_f16's result), so the lanes stay in their words.
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h16x2 w2h(uint32_t w) { return __builtin_bit_cast(h16x2, w); }
__device__ __forceinline__ uint32_t h2w(h16x2 h) { return __builtin_bit_cast(uint32_t, h); }
__device__ __forceinline__ uint32_t pk_fma_w(uint32_t a, uint32_t b, uint32_t c) {
    return h2w(__builtin_elementwise_fma(w2h(a), w2h(b), w2h(c)));
}
__device__ __forceinline__ h16 lane_of(const uint32_t w[4], int l) {
    return u2h((uint16_t)(w[l >> 1] >> (16 * (l & 1))));
}

__device__ __forceinline__ uint32_t pk_add_w(uint32_t a, uint32_t b) { return h2w(w2h(a) + w2h(b)); }
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_w(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// The GGML_F16_VEC_REDUCE of 4 accumulators held by the 4 lanes of a quad (lane j of the
// quad: accumulator j, 8 f16 lanes in 4 words): sum[0] += sum[2], sum[1] += sum[3],
// sum[0] += sum[1] per f16 lane (IEEE adds, commutative), then the f32 tail; the result
// is valid in the quad's lane 0. Every lane of the wave must be active.
__device__ __forceinline__ float f16x8_reduce_quad(const uint32_t acc[4]) {
    uint32_t s[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t t = pk_add_w(acc[k], dpp_w<0x4E>(acc[k]));  // j0: a0 + a2, j1: a1 + a3
        s[k] = pk_add_w(t, dpp_w<0xB1>(t));                        // j0: (a0 + a2) + (a1 + a3)
    }
    h16 v[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) v[l] = lane_of(s, l);
    return f16x8_reduce(v);
}

// ggml_vec_dot_f16 (NEON FP16) of two f16 rows held as 8-element vectors of 16-B:
// x[v], y[v] for v in [0, n/8); n % 32 == 0. Returns the f32 result. Accumulator j of
// the 4 (vfmaq_f16 on sum[j]) holds lanes 2k, 2k+1 in word acc[j][k].
template <int N>
__device__ __forceinline__ float vec_dot_f16_rows(const uint4 *x, const uint4 *y) {
    static_assert(N % 32 == 0, "n % 32");
    uint32_t acc[4][4] = {};
#pragma unroll
    for (int it = 0; it < N / 32; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 xv = x[4 * it + j], yv = y[4 * it + j];
            acc[j][0] = pk_fma_w(xv.x, yv.x, acc[j][0]);
            acc[j][1] = pk_fma_w(xv.y, yv.y, acc[j][1]);
            acc[j][2] = pk_fma_w(xv.z, yv.z, acc[j][2]);
            acc[j][3] = pk_fma_w(xv.w, yv.w, acc[j][3]);
        }
    h16 s[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const h16 s0 = lane_of(acc[0], l) + lane_of(acc[2], l);
        const h16 s1 = lane_of(acc[1], l) + lane_of(acc[3], l);
        s[l] = s0 + s1;
    }
    return f16x8_reduce(s);
}

// Sum of squares of 16 consecutive floats, sequential in double (x*x rounded to float
// first, as `(ggml_float)(x[i00] * x[i00])`).
__device__ __forceinline__ double sumsq16(const float v[16]) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += (double)(v[k] * v[k]);
    return s;
}

// Balanced tree over the 16 lanes of an aligned 16-lane row (xor 1, 2, 4, 8): every
// lane of the row ends with the same value. By DPP: quad permutes for xor 1 and 2;
// after them every lane of a quad holds the quad's sum, so the half-row mirror
// brings the other quad's sum (= the xor-4 partner's value) and the row mirror the
// other half's (= xor 8); float addition is commutative, so every lane's sum has
// the same bits as the xor tree. Every lane of the wave must be active.
template <int CTRL>
__device__ __forceinline__ double dpp_mov_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double row16_sum(double v) {
    v += dpp_mov_f64<0xB1>(v);   // xor 1
    v += dpp_mov_f64<0x4E>(v);   // xor 2
    v += dpp_mov_f64<0x141>(v);  // the other quad of the half-row (xor 4)
    v += dpp_mov_f64<0x140>(v);  // the other half of the row (xor 8)
    return v;
}

// In-order double sum of the first n values of sums[] (LDS), the same adds as
// `for (b < n) tot += sums[b]`: lane i loads sums[c0 + i] for a chunk of 64 and the
// dependent adds read the lanes in order (one LDS round trip per 64 values).
__device__ __forceinline__ double seq_sum_lanes(const double *sums, int n, int lane) {
    double tot = 0.0;
    for (int c0 = 0; c0 < n; c0 += 64) {
        const double v = c0 + lane < n ? sums[c0 + lane] : 0.0;
        const uint64_t b = __builtin_bit_cast(uint64_t, v);
        const int m = n - c0 < 64 ? n - c0 : 64;
        for (int i = 0; i < m; ++i) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, i);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), i);
            tot += __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
        }
    }
    return tot;
}

// Max over a wave (order-free: fmaxf is exact): quad xor 1 / 2, half-row and row
// mirrors by DPP, then the four rows by readlane. Every lane must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_mov_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_fmax(float v) {
    v = fmaxf(v, dpp_mov_f32<0xB1>(v));   // quad_perm [1,0,3,2]
    v = fmaxf(v, dpp_mov_f32<0x4E>(v));   // quad_perm [2,3,0,1]
    v = fmaxf(v, dpp_mov_f32<0x141>(v));  // row_half_mirror
    v = fmaxf(v, dpp_mov_f32<0x140>(v));  // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// The wave's sum of v, for callers whose every partial sum is exact (then any order gives
// the same bits): DPP within rows of 16, then the four row sums.
__device__ __forceinline__ double wave_sum_exact_f64(double v) {
    v = row16_sum(v);
    return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// sum / n in double, correctly rounded (ggml_float mean = sum/ne00): for n a power of
// two the quotient is the exact product sum * 2^-k (both correctly rounded results of
// the same real value), so the f64 divide sequence is skipped.
__device__ __forceinline__ double div_by_count(double sum, int64_t n) {
    if ((n & (n - 1)) == 0) return sum * (1.0 / (double)n);
    return sum / (double)n;
}

// ---------------------------------------------------------------- rms_norm exactness guard
// The fast sum of squares above runs in a fixed tree order; ggml sums
// (ggml_float)(x*x) sequentially (ggml_compute_forward_rms_norm_f32). Both are sums of
// non-negative terms with one rounding per add, so each is within (n + 32) * 2^-53 * S
// of the exact S (partial sums never exceed S), and after the correctly rounded
// division by n the two doubles md_tree, md_seq differ by less than
// delta = (2n + 64) * 2^-53 * md. The float mean (float)md can therefore differ only
// when md_tree lies within delta of a float rounding midpoint (the ones next to
// f = (float)md_tree: delta is ~2^-39 relative even at n = 8192, a float ulp 2^-23).
// Then, and for inf/NaN, the caller recomputes the sum in ggml's sequential order:
// the mean is bit-exact by construction, and the slow path runs for about one row in
// 10^4-10^5 of random data (tests/test_gpu_ops.py builds inputs that take it).
__device__ __forceinline__ bool rms_mean_ambiguous(double md, int64_t n) {
    const float f = (float)md;
    if (!(f >= 0.0f && f <= 3.402823466e+38f)) return true;  // a sum of squares: >= 0, else inf/NaN
    const double delta = (double)(2 * n + 64) * 0x1p-53 * md;
    const uint32_t fb = __float_as_uint(f);                  // neighbours of f >= 0 by its bits
    const double fu = (double)__uint_as_float(fb + 1u);
    const double fd = fb ? (double)__uint_as_float(fb - 1u) : -(double)__uint_as_float(1u);
    const double mid_up = ((double)f + fu) * 0.5, mid_dn = ((double)f + fd) * 0.5;  // exact in double
    return __builtin_fabs(md - mid_up) <= delta || __builtin_fabs(md - mid_dn) <= delta;
}

// ggml's order, one wave: sum += (ggml_float)(x[i] * x[i]) for i = 0 .. n-1. Lane l
// squares x[c0 + l] (a float product, as in C), then the dependent double adds read
// the lanes in order. Every lane of the wave returns the same sum.
__device__ __forceinline__ double seq_sumsq_wave(const float *x, int64_t n, int lane) {
    double tot = 0.0;
    for (int64_t c0 = 0; c0 < n; c0 += 64) {
        const float v = c0 + lane < n ? x[c0 + lane] : 0.0f;
        const float p = v * v;
        const double sq = (double)p;
        const uint64_t b = __builtin_bit_cast(uint64_t, sq);
        const int m = n - c0 < 64 ? (int)(n - c0) : 64;
        for (int i = 0; i < m; ++i) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, i);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), i);
            tot += __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
        }
    }
    return tot;
}

// In-order double sum of n LDS doubles (p 16-B aligned): sum = ((0 + p[0]) + p[1]) + ...,
// the dependent adds fed by 16-B reads issued 8 values ahead instead of one LDS
// round trip per value.
__device__ __forceinline__ double seq_sum_lds(const double *p, int n) {
    double sum = 0.0;
    int i = 0;
    if (n >= 8) {
        const double2 *p2 = (const double2 *)p;
        double2 c0 = p2[0], c1 = p2[1], c2 = p2[2], c3 = p2[3];
        for (; i + 8 <= n; i += 8) {
            double2 n0 = c0, n1 = c1, n2 = c2, n3 = c3;
            if (i + 16 <= n) {
                const int h = (i + 8) / 2;
                n0 = p2[h], n1 = p2[h + 1], n2 = p2[h + 2], n3 = p2[h + 3];
            }
            sum += c0.x;
            sum += c0.y;
            sum += c1.x;
            sum += c1.y;
            sum += c2.x;
            sum += c2.y;
            sum += c3.x;
            sum += c3.y;
            c0 = n0, c1 = n1, c2 = n2, c3 = n3;
        }
    }
    for (; i < n; ++i) sum += p[i];
    return sum;
}

#ifndef KQ_SEQ_SUM_WAVE
#define KQ_SEQ_SUM_WAVE 0  // soft_max's in-order fallback: seq_sum_wave (0: seq_sum_lds, one dependent add per term)
#endif
// ggml's in-order `sum += g[i]` over n LDS doubles g[i] >= 0 (or non-finite), bit for bit, by
// one whole wave, 64 terms a round instead of one dependent add per term (soft_max's group
// sums; not for signed terms). While the running sum s stays in one binade [2^E, 2^(E+1)), s
// is a multiple of u = 2^(E-52) and s + g rounds to s + RN(g / u) u whatever s's other bits
// are, unless g / u is an exact tie (the even neighbour then depends on s). Lane l takes term
// i0 + l: RN(g / u) as an integer, an inclusive scan over the lanes (DPP; exact below 2^53,
// >= 2^53 when it is not), and the first lane whose s would reach 2^(E+1), or that holds a tie
// or a non-finite term, is added as is after the exact sum of the lanes before it; the next
// round starts after it. A sum that changes binade too often finishes in order.
// (tests/test_ops_oracle.py mirrors this in numpy against the plain loop.)
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64_or0(double v) {  // lanes without a source: +0
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, ROWS, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, ROWS, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double seq_sum_wave(const double *g, int n, int lane) {
    double s = 0.0;
    int i0 = 0;
    const int max_rounds = (n >> 6) + 48;
    for (int round = 0; i0 < n && round < max_rounds; ++round) {
        if (!(s < INFINITY)) break;  // inf / NaN: the rest in order
        const int len = n - i0 < 64 ? n - i0 : 64;
        const double v = lane < len ? g[i0 + lane] : 0.0;
        int k;  // the lane added as is
        if (s == 0.0) {  // no binade yet: zeros add nothing, the first nonzero term as is
            const uint64_t bl = __ballot(v != 0.0);
            if (bl == 0) {
                i0 += len;
                continue;
            }
            k = __builtin_ctzll(bl);
        } else {
            const int ex = (int)((__double_as_longlong(s) >> 52) & 0x7ff);  // s normal: >= 2^-149
            const double sc = __longlong_as_double((long long)(2098 - ex) << 52);  // 1 / u
            const double uu = __longlong_as_double((long long)(ex - 52) << 52);    // u
            const double su = s * sc;                                              // in [2^52, 2^53)
            const double x = v * sc;  // exact (a power of two)
            const bool fin = x < INFINITY;
            const double xf = fin ? x : 0.0;
            bool fl = !fin || xf - __builtin_floor(xf) == 0.5;
            double q = __builtin_rint(xf);
            q += dpp_f64_or0<0x111, 0xF>(q);  // row_shr:1
            q += dpp_f64_or0<0x112, 0xF>(q);  // row_shr:2
            q += dpp_f64_or0<0x114, 0xF>(q);  // row_shr:4
            q += dpp_f64_or0<0x118, 0xF>(q);  // row_shr:8
            q += dpp_f64_or0<0x142, 0xA>(q);  // row_bcast:15 (rows 1, 3)
            q += dpp_f64_or0<0x143, 0xC>(q);  // row_bcast:31 (rows 2, 3)
            fl = lane < len && (fl || su + q >= 0x1p53);
            const uint64_t bl = __ballot(fl);
            if (bl == 0) {
                s = (su + readlane_f64(q, 63)) * uu;  // (lanes >= len add 0)
                i0 += len;
                continue;
            }
            k = __builtin_ctzll(bl);
            s = (su + (k > 0 ? readlane_f64(q, k - 1) : 0.0)) * uu;
        }
        s += readlane_f64(v, k);
        i0 += k + 1;
    }
    for (; i0 < n; ++i0) s += g[i0];
    return s;
}

// soft_max's double sum of the n vaddvq group sums g[0..n) (LDS doubles, each a float
// (e0 + e1) + (e2 + e3) >= 0, e <= 1: every g <= 4), with the bits of ggml's in-order
// `sum += (ggml_float)g` (ggml_vec_soft_max_f32), computed by one whole wave.
// Every nonzero float g is a multiple of 2^G(g) (G: the exponent of its last mantissa bit,
// max(biased exponent, 1) - 150), so every partial sum of such terms, in ANY order, is a
// multiple of 2^Gmin no larger than the total T: exactly representable in double while
// T < 2^(Gmin + 53). Then the in-order sum never rounds and equals the exact sum, which a tree
// over the wave computes in 6 steps instead of n dependent f64 adds. The test uses the tree's
// own total S (within 2^-48 of T, so S <= (1 - 2^-40) 2^(Gmin + 53) proves T < 2^(Gmin + 53)):
// exact whenever the smallest group sum is within ~2^-30 of the total (round 6; rounds 1-5
// bounded T by 4n, 2^-29 of it, up to 9 binades stricter at 1024 groups). A more peaked
// soft_max, or a non-finite g, takes the in-order sum itself.
struct SumExact {
    double part = 0.0;  // this lane's terms, any order
    int gmin = 1 << 20; // min G over its nonzero terms (none: 2^20)
    bool bad = false;   // a non-finite term
    __device__ __forceinline__ void add(float gf) {
        const int ef = (__float_as_int(gf) >> 23) & 0xff;
        bad = bad || ef == 255;
        const int G = (ef > 1 ? ef : 1) - 150;
        gmin = gf != 0.0f && G < gmin ? G : gmin;
        part += (double)gf;
    }
};
// the bound test for a total s of terms with min G gmin: true = every partial sum is exact
__device__ __forceinline__ bool sum_exact_ok(double s, int gmin, bool bad) {
    if (bad) return false;
    if (gmin >= (1 << 20)) return true;  // every term zero
    return s <= __longlong_as_double((long long)(gmin + 53 + 1023) << 52) * (1.0 - 0x1p-40);
}
__device__ __forceinline__ int wave_imin(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int y = __shfl_xor(v, o, 64);
        v = y < v ? y : v;
    }
    return v;
}
// The wave tree alone: the sum and whether it is provably ggml's in-order sum (ok; wave-uniform)
__device__ __forceinline__ double softmax_group_tree(const double *g, int n, int lane, bool &ok) {
    SumExact se;
    for (int i = lane; i < n; i += 64) se.add((float)g[i]);  // (float)g is exact: g holds a float
    double part = se.part;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    const double p0 = readlane_f64(part, 0);  // (one value for the whole wave's decision)
    ok = sum_exact_ok(p0, wave_imin(se.gmin), __any(se.bad));
    return p0;
}
__device__ __forceinline__ double softmax_group_sum(const double *g, int n, int lane) {
    if (n <= 0) return 0.0;
    bool ok;
    const double p0 = softmax_group_tree(g, n, lane, ok);
    if (ok) return p0;
    return KQ_SEQ_SUM_WAVE ? seq_sum_wave(g, n, lane) : seq_sum_lds(g, n);
}

}  // namespace kq
