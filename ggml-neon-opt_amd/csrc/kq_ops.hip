// kq_ops.hip — the non-matmul ops of a llama decode token on gfx950 (SURVEY.md §8f
// rank 4): get_rows, rms_norm (+ its weight MUL), add, mul, swiglu, rope and the
// decode attention block (rope + f16 KV-cache write + KQ + soft_max + KQV).
//
// Reference functions (ggml-cpu @ a3cb0474 [U], as profiled in
// artifacts/perf/out.folded; restated for the tests on the CPU side):
//   get_rows  ggml_compute_forward_get_rows_q -> dequantize_row_q4_K   :103-104
//   rms_norm  ggml_compute_forward_rms_norm_f32                        :189-193
//   mul/add   binary_op<op_mul>/<op_add>                               :91-99, :115-121
//   swiglu    ggml_vec_swiglu_f32 (ggml_v_silu)                        :107-113
//   rope      ggml_compute_forward_rope_f32 (ggml_rope_cache_init, rope_yarn) :196-208
//   attention set_rows (f32->f16), mul_mat(f16) -> ggml_vec_dot_f16, soft_max_f32
//             (ggml_vec_soft_max_f32, ggml_v_expf), mul_mat(f16)       :140-144, :176, :209-234
// Every kernel reproduces the reference's arithmetic op for op (see kq_ops_device.h);
// these ops are HBM/latency-bound and tiny at decode, so the layout work is about
// launch count (they fuse into the GEMVs where the graph allows, kq_rows.hip).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <vector>

#include <hip/hip_ext.h>

#include "kq_common.h"
#include "kq_internal.h"
#include "kq_attn_device.h"
#include "kq_attn_head.h"
#include "kq_device.h"
#include "kq_ops_device.h"
#include "kq_rows_device.h"

#ifndef KQ_ATTN_BATCH_CTX
#define KQ_ATTN_BATCH_CTX 256  // caches above this many cells take kq_attn_decode<HD, true>
#endif
#ifndef KQ_ATTN_OSC1
#define KQ_ATTN_OSC1 0  // experiment build: the decode attention's output stored write-through (sc1)
#endif

namespace kq {

// ------------------------------------------------------------ get_rows
// One workgroup per (id, 2048-element chunk); thread t dequantizes 8 consecutive
// elements. Q4_K / Q5_K: y = fmaf(d*sc, q, -(dmin*m)) (gcc contracts `d1*q - m1` [U]; Q5_K's
// q is the nibble + 16 * its qh bit); Q6_K: y = (d*sc)*q; F32: copy.
__global__ void __launch_bounds__(256) kq_get_rows(int type, const uint8_t *__restrict__ table, int64_t k,
                                                   int64_t row_stride, int64_t n_rows,
                                                   const int32_t *__restrict__ ids, float *__restrict__ out) {
    const int64_t r = blockIdx.y;
    const int64_t e0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (e0 >= k) return;
    const int64_t id = ids[r];
    float *y = out + r * k + e0;
    if (id < 0 || id >= n_rows) {  // ggml asserts 0 <= i01 < ne01: never read outside the table
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = __builtin_nanf("");
        return;
    }
    const uint8_t *row = table + id * row_stride;
    if (type == MI355X_TYPE_F32) {
        const float *s = (const float *)row + e0;
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = s[i];
        return;
    }
    const int64_t b = e0 / QK;
    const int e = (int)(e0 % QK);
    if (type == MI355X_TYPE_Q4_K || type == MI355X_TYPE_Q5_K) {
        const bool q5 = type == MI355X_TYPE_Q5_K;
        const uint8_t *blk = row + b * (q5 ? 176 : 144);
        const float d = h2f(*(const uint16_t *)blk), dmin = h2f(*(const uint16_t *)(blk + 2));
        const uint8_t *sc = blk + 4;
        const int j = e / 64, h = (e / 32) & 1, l0 = e % 32;
        const int is = 2 * j + h;
        int s, m;
        if (is < 4) {
            s = sc[is] & 63;
            m = sc[is + 4] & 63;
        } else {
            s = (sc[is + 4] & 0xF) | ((sc[is - 4] >> 6) << 4);
            m = (sc[is + 4] >> 4) | ((sc[is] >> 6) << 4);
        }
        const float d1 = d * (float)s, m1 = dmin * (float)m;
        const uint8_t *q = blk + (q5 ? 48 : 16) + 32 * j + l0;
        const uint8_t *qh = blk + 16 + l0;  // Q5_K: bit 2j + h of qh[l] is the fifth bit
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int hb = q5 ? ((qh[i] >> (2 * j + h)) & 1) << 4 : 0;
            y[i] = __builtin_fmaf(d1, (float)(((q[i] >> (4 * h)) & 0xF) + hb), -m1);
        }
    } else {  // Q6_K
        const uint8_t *blk = row + b * 210;
        const float d = h2f((uint16_t)(blk[208] | (blk[209] << 8)));
        const int half = e / 128, rr = e % 128, quarter = rr / 32, l0 = rr % 32;
        const uint8_t *ql = blk + 64 * half, *qh = blk + 128 + 32 * half;
        const int8_t *sc = (const int8_t *)(blk + 192) + 8 * half;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int l = l0 + i;
            int q;
            if (quarter == 0) q = (ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4);
            else if (quarter == 1) q = (ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4);
            else if (quarter == 2) q = (ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4);
            else q = (ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4);
            y[i] = d * (float)sc[l / 16 + 2 * quarter] * (float)(q - 32);
        }
    }
}

// ------------------------------------------------------------ rms_norm (+ mul)
// One workgroup per row, 256 threads = 16 rows of 16 lanes; lane l of a row owns
// elements [16l, 16l+16) of one superblock per pass. Sum order: kq_ops_device.h.
__global__ void __launch_bounds__(256) kq_rms_norm(const float *__restrict__ x, const float *__restrict__ w,
                                                   float *__restrict__ y, int64_t n, float eps) {
    extern __shared__ __attribute__((aligned(16))) double sb_sum[];
    const int64_t row = blockIdx.x;
    const float *xr = x + row * n;
    float *yr = y + row * n;
    const int nb = (int)(n / QK);
    const int rid = threadIdx.x >> 4, l = threadIdx.x & 15;
    for (int b0 = 0; b0 < nb; b0 += 16) {
        const int b = b0 + rid;
        double s = 0.0;
        if (b < nb) {
            float v[16];
            const float4 *p = (const float4 *)(xr + (int64_t)b * QK + 16 * l);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 t = p[k];
                v[4 * k] = t.x, v[4 * k + 1] = t.y, v[4 * k + 2] = t.z, v[4 * k + 3] = t.w;
            }
            s = sumsq16(v);
        }
        s = row16_sum(s);
        if (b < nb && l == 0) sb_sum[b] = s;
    }
    __syncthreads();
    double total = seq_sum_lds(sb_sum, nb);  // superblocks in order
    if (rms_mean_ambiguous(div_by_count(total, n), n)) {  // block-uniform: every thread has the same total
        __syncthreads();                                  // sb_sum[0] is reused below
        if (threadIdx.x < 64) {
            const double s = seq_sumsq_wave(xr, n, threadIdx.x);  // ggml's sequential order
            if (threadIdx.x == 0) sb_sum[0] = s;
        }
        __syncthreads();
        total = sb_sum[0];
    }
    const float mean = (float)div_by_count(total, n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const float v = xr[i] * scale;
        yr[i] = w ? v * w[i] : v;
    }
}

// ------------------------------------------------------------ elementwise
// b has nb elements, repeated over a's rows (ggml_add / ggml_mul broadcast of src1 over
// ne1: the norm weights of a batch); nb == n is the plain element-wise op.
__global__ void __launch_bounds__(256) kq_binary(int op, const float *__restrict__ a, const float *__restrict__ b,
                                                 float *__restrict__ y, int64_t n, int64_t nb) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const float bv = b[nb == n ? i : i % nb];
        y[i] = op == 0 ? a[i] + bv : a[i] * bv;
    }
}

// ggml_vec_swiglu_f32: NEON body for the first n & ~3 elements, libm tail otherwise.
__global__ void __launch_bounds__(256) kq_swiglu(const float *__restrict__ g, const float *__restrict__ u,
                                                 float *__restrict__ y, int64_t n) {
    const int64_t n4 = n & ~(int64_t)3;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        y[i] = i < n4 ? v_silu(g[i]) * u[i] : (g[i] / (1.0f + expf(-g[i]))) * u[i];
}

__global__ void __launch_bounds__(256) kq_rope(const float *__restrict__ x, float *__restrict__ y, int head_dim,
                                               int n_dims, int n_heads, const int32_t *__restrict__ pos_p,
                                               const float *__restrict__ table, int n_pos) {
    const int pos = *pos_p;
    const int per = head_dim / 2;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // pair index
    if (i >= (int64_t)n_heads * per) return;
    const int h = (int)(i / per), p = (int)(i % per);
    const float *s = x + (int64_t)h * head_dim + 2 * p;
    float *d = y + (int64_t)h * head_dim + 2 * p;
    if (pos < 0 || pos >= n_pos) {  // outside the table: NaN, never a silent result
        d[0] = d[1] = __builtin_nanf("");
        return;
    }
    if (2 * p >= n_dims) {
        d[0] = s[0];
        d[1] = s[1];
        return;
    }
    const float *cs = table + ((int64_t)pos * (n_dims / 2) + p) * 2;
    const float2 r = rope_pair(s[0], s[1], cs[0], cs[1]);
    d[0] = r.x;
    d[1] = r.y;
}

// ------------------------------------------------------------ decode attention
// One workgroup per query head (kq_attn_head.h).
// BATCH: the cache loads past the prefetched cells requested in batches (kq_attn_head.h); the
// launch takes it for caches of more than KQ_ATTN_BATCH_CTX cells only: at short context its
// code costs the head_dim-128 launch ~0.3 us (profiles/r05_attn_ab_batch_ctx.txt).
// DS > 1: DS workgroups per head, one slice of the head's outputs each (kq_attn_head.h).
// TPH: threads per head (experiment builds: KQ_ATTN_TPH64 = 128 for the short-context head_dim
// 64 launch; the register path then holds 128 cells, the fused attention + o-proj's shape).
#ifndef KQ_ATTN_TPH64
#define KQ_ATTN_TPH64 256
#endif
#ifndef KQ_ATTN_KDMA1  // 1: experiment build, caches of <= 256 cells on the LDS-DMA path (attn_head KD1)
#define KQ_ATTN_KDMA1 0
#endif
template <int HD, bool BATCH, int DS = 1, int TPH = 256, bool KD1 = false>
__global__ void __launch_bounds__(TPH) kq_attn_decode(const AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // XCD-aware head order (speed only): workgroup b runs on XCD b % 8, so XCD x takes the
    // consecutive heads [x*n_head/8, (x+1)*n_head/8) (every slice of a head on one XCD) and a
    // KV group's cells are fetched into the L2 of 8*gsz/n_head XCDs (TinyLlama: 2, Llama-3: 1)
    // instead of all 8.
    int h = blockIdx.x / DS, ds = blockIdx.x % DS;
    if ((a.n_head & 7) == 0) {
        const int x = blockIdx.x & 7, i = blockIdx.x >> 3;
        h = x * (a.n_head >> 3) + i / DS;
        ds = i % DS;
    }
    attn_head<HD, TPH, 0, KQ_ATTN_OSC1 != 0, false, BATCH, DS, KD1>(a, h, threadIdx.x, smem, a.out + (int64_t)h * HD,
                                                                     true, ds);
}

// ------------------------------------------------------------ long caches: KQ split over cells
// The output split (kq_attn_decode<HD, true, DS>) keeps the head's scores and its V slice in
// one workgroup and scores every cell in every slice; past what its LDS holds (~3000 cells at
// head_dim 64) the one-workgroup-per-head kernel streams every K and V row of a head through
// one CU (tg4096: ~21 us per layer). For caches of more than KQ_ATTN_CELLS_MIN cells where the
// split would need 8 slices or does not fit (attn_path), the head's KQ splits over cells
// instead, in two launches (DESIGN.md §4 "KQ split over cells", profiles/r06_cells_ab.txt):
//  A kq_attn_cells: workgroup (chunk, g) scores ATTN_CHUNK cells of kv group g for EVERY query
//    head of the group (each K row read once for the gsz heads) into a score workspace
//    [n_head][n_ctx]; the workgroup whose chunk holds the position writes the new cell to both
//    caches (rope'd k, f16 v) and scores that cell from its own copy;
//  B kq_attn_cells_kqv: workgroup (h, ds): soft_max over the head's scores held in registers
//    and KQV for its RS = HD / DS outputs (16 threads per output) from its V rows, LDS-DMA'd
//    under soft_max (the new cell included: A wrote it, a kernel boundary before).
// Every score is the same NEON-FP16 vec_dot as the one-launch kernels', soft_max's max, exps,
// group sums and in-order double sum and the KQV accumulator chains are theirs: bit-exact.
constexpr int ATTN_CHUNK = 64;
#ifndef KQ_ATTN_CELLS_OVER_SPLIT
#define KQ_ATTN_CELLS_OVER_SPLIT 0  // experiment builds: the two launches also where the output split fits
#endif
#ifndef KQ_ATTN_CELLS_SLICES
#define KQ_ATTN_CELLS_SLICES 8  // ... and where it needs this many slices (tg3072 +5 %, 8B tg2048 +5.5 %; 4: equal)
#endif
#ifndef KQ_ATTN_CELLS_MIN
#define KQ_ATTN_CELLS_MIN 1024  // only caches of more cells than this take the two launches
#endif
#ifndef KQ_ATTN_CELLS_OVERLAP
#define KQ_ATTN_CELLS_OVERLAP 1  // B's soft_max waits for the scores only, the V rows land meanwhile
#endif
#ifndef KQ_ATTN_CELLS_RS64
#define KQ_ATTN_CELLS_RS64 8  // B's outputs per workgroup at head_dim 64 (8: 256 workgroups for 32 heads)
#endif
#ifndef KQ_ATTN_CELLS_RS128
#define KQ_ATTN_CELLS_RS128 16  // at head_dim 128 (16: 256 workgroups for 32 heads, one round)
#endif
#ifndef KQ_ATTN_CELLS_STOP
#define KQ_ATTN_CELLS_STOP 0  // diagnostic builds: B stops after its loads (1) or soft_max (2)
#endif
#ifndef KQ_ATTN_CELLS_VPAD
#define KQ_ATTN_CELLS_VPAD 64  // bytes past 2 n_ctx per V row in B's LDS (a multiple of 16)
#endif
constexpr int ATTN_CELLS_VPAD = KQ_ATTN_CELLS_VPAD;
constexpr int ATTN_CELLS_GMAX = 8;  // B's soft_max: 4-cell groups per thread in registers (n_ctx <= 8192)

template <int HD>
__global__ void __launch_bounds__(256) kq_attn_cells(const AttnArgs a, float *scores) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int KV4 = HD / 8;                        // 16-B pieces of a K row
    constexpr int KPT = ATTN_CHUNK * KV4 / 256;        // pieces per thread
    const int g = blockIdx.y, c0 = blockIdx.x * ATTN_CHUNK, t = threadIdx.x;
    const int gsz = a.n_head / a.n_head_kv;
    const int kvw = a.n_head_kv * HD;
    // every load that does not depend on the position goes out with it: the chunk's K rows
    // (cells < n_ctx: valid memory whatever the position; cell pos's row is stale and unused)
    uint4 kr[KPT];
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
        const int i = t + 256 * u, r = i / KV4, k = i % KV4;
        kr[u] = *(const uint4 *)(a.k_cache + (int64_t)(c0 + r) * kvw + (int64_t)g * HD + 8 * k);
    }
    const int pos_in = *a.pos;
    const bool bad = pos_in < 0 || pos_in >= a.n_ctx;  // no cache cell: caches untouched, B outputs NaN
    const int pos = bad ? 0 : pos_in;
    int n_kv = (pos + 1 + 31) / 32 * 32;
    n_kv = n_kv < a.n_ctx ? n_kv : a.n_ctx;
    if (c0 >= n_kv) return;  // (uniform)
    // LDS: q16 [gsz][HD] | k16 [HD] | K rows [ATTN_CHUNK][KV4] (piece k of row r at k ^ (r % KV4))
    uint16_t *q16 = (uint16_t *)smem;
    uint16_t *k16 = q16 + gsz * HD;
    uint4 *krow = (uint4 *)(k16 + HD);
    const bool holds = pos >= c0 && pos < c0 + ATTN_CHUNK;
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
        const int i = t + 256 * u, r = i / KV4, k = i % KV4;
        krow[r * KV4 + (k ^ (r % KV4))] = kr[u];
    }
    // rope(q) of the group's heads at pos (kq_attn_head.h step 1), and the new cell where held
    const float *tc = a.rope_table + (a.rope_row ? 0 : (int64_t)pos * (HD / 2) * 2);
    for (int i = t; i < gsz * (HD / 2); i += 256) {
        const int hh = i / (HD / 2), p2 = i % (HD / 2);
        const float *qp = a.q + (int64_t)(g * gsz + hh) * HD + 2 * p2;
        const float2 rq = rope_pair(qp[0], qp[1], tc[2 * p2], tc[2 * p2 + 1]);
        q16[hh * HD + 2 * p2] = h2u(f2h_rne(rq.x));
        q16[hh * HD + 2 * p2 + 1] = h2u(f2h_rne(rq.y));
    }
    if (holds) {
        for (int p2 = t; p2 < HD / 2; p2 += 256) {
            const float *kp = a.k + (int64_t)g * HD + 2 * p2;
            const float2 rk = rope_pair(kp[0], kp[1], tc[2 * p2], tc[2 * p2 + 1]);
            const uint16_t k0 = h2u(f2h_rne(rk.x)), k1 = h2u(f2h_rne(rk.y));
            k16[2 * p2] = k0;
            k16[2 * p2 + 1] = k1;
            if (!bad) *(uint32_t *)(a.k_cache + (int64_t)pos * kvw + (int64_t)g * HD + 2 * p2) = k0 | ((uint32_t)k1 << 16);
        }
        for (int d = t; d < HD && !bad; d += 256)
            a.v_cache[(int64_t)(g * HD + d) * a.n_ctx + pos] = h2u(f2h_rne(a.v[(int64_t)g * HD + d]));
    }
    __syncthreads();
    for (int i = t; i < ATTN_CHUNK * gsz; i += 256) {  // lane <-> cell, waves <-> heads
        const int r = i % ATTN_CHUNK, hh = i / ATTN_CHUNK, c = c0 + r;
        if (c >= n_kv) continue;
        float sc = -INFINITY;  // cells past pos: masked
        if (c <= pos) {
            uint4 kv[KV4];
            if (c == pos) {
#pragma unroll
                for (int k = 0; k < KV4; ++k) kv[k] = ((const uint4 *)k16)[k];
            } else {
#pragma unroll
                for (int k = 0; k < KV4; ++k) kv[k] = krow[r * KV4 + (k ^ (r % KV4))];
            }
            sc = vec_dot_f16_rows<HD>(kv, (const uint4 *)(q16 + hh * HD)) * a.scale;
        }
        scores[(int64_t)(g * gsz + hh) * a.n_ctx + c] = sc;
    }
}

// B: every input of the workgroup — the head's n_kv scores and its RS = HD / DS V rows over
// cells [0, n_kv) — arrives by LDS-DMA issued at entry, all in flight at once (a thread's KQV
// chain runs over n_kv / 32 iterations in order: loading them from global memory as it goes
// paid one memory latency per batch). soft_max waits for the scores only (a counted vmcnt: the
// V rows were issued after them), so the V rows land while it runs; KQV reads LDS only.
// LDS: the scores (n_ctx f32; once in registers the region holds the group sums, then p16) |
// red (KQV words, RS x 16 u32) | scal (24 f32: wave maxima, wave ok flags, wave sums as f64) |
// the V rows (RS x VSTR).
template <int VM>
__device__ __forceinline__ void waitcnt_vm_le() {  // s_waitcnt vmcnt(VM) (expcnt, lgkmcnt free)
    static_assert(VM >= 0 && VM < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((VM & 15) | ((VM >> 4) << 14) | 0x0F70);
}
__device__ __forceinline__ void waitcnt_vm_floor8(int n) {  // vmcnt(8 floor(min(n, 63) / 8)) <= n
    switch ((n > 63 ? 63 : n) >> 3) {
    case 0: waitcnt_vm_le<0>(); break;
    case 1: waitcnt_vm_le<8>(); break;
    case 2: waitcnt_vm_le<16>(); break;
    case 3: waitcnt_vm_le<24>(); break;
    case 4: waitcnt_vm_le<32>(); break;
    case 5: waitcnt_vm_le<40>(); break;
    case 6: waitcnt_vm_le<48>(); break;
    default: waitcnt_vm_le<56>(); break;
    }
}
template <int HD, int DS>
__global__ void __launch_bounds__(256) kq_attn_cells_kqv(const AttnArgs a, const float *scores) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int RS = HD / DS;  // outputs of this workgroup
    static_assert(RS * 16 <= 256 && (RS & (RS - 1)) == 0 && RS >= 4, "16 threads per output, whole rows per wave");
    int h = blockIdx.x / DS, ds = blockIdx.x % DS;
    if ((a.n_head & 7) == 0) {  // XCD-aware order, as kq_attn_decode (speed only)
        const int x = blockIdx.x & 7, i = blockIdx.x >> 3;
        h = x * (a.n_head >> 3) + i / DS;
        ds = i % DS;
    }
    const int t = threadIdx.x, ln = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int g = h / (a.n_head / a.n_head_kv);
    const int pos_in = *a.pos;
    const bool bad = pos_in < 0 || pos_in >= a.n_ctx;
    const int pos = bad ? 0 : pos_in;
    int n_kv = (pos + 1 + 31) / 32 * 32;
    n_kv = n_kv < a.n_ctx ? n_kv : a.n_ctx;
    const int n_it = (pos + 32) / 32;  // 32-cell iterations holding a cell <= pos
    float *w = (float *)smem;
    double *gsum = (double *)smem;
    uint16_t *p16 = (uint16_t *)smem;
    uint32_t *red = (uint32_t *)(w + a.n_ctx);
    float *scal = (float *)(red + RS * 16);
    uint8_t *vlds = (uint8_t *)(scal + 24);
    const int VSTR = 2 * a.n_ctx + ATTN_CELLS_VPAD;  // rows 16 words apart in the banks
    int nv = 0;  // this wave's V-row DMAs (issued after its score DMAs)
    {
        const uint8_t *src = (const uint8_t *)(scores + (int64_t)h * a.n_ctx);
        const int sg = n_kv / 4;
        for (int i = wv; 64 * i < sg; i += 4) {
            const int n = sg - 64 * i < 64 ? sg - 64 * i : 64;
            attn_dma16_lanes(src + 1024 * i + 16 * ln,
                             __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS void *)((uint8_t *)w + 1024 * i)), ln, n);
        }
        const int vg = n_kv / 8;
        for (int r = wv; r < RS; r += 4) {
            const uint8_t *vsrc = (const uint8_t *)(a.v_cache + (int64_t)(g * HD + ds * RS + r) * a.n_ctx);
            for (int i = 0; 64 * i < vg; ++i, ++nv) {
                const int n = vg - 64 * i < 64 ? vg - 64 * i : 64;
                attn_dma16_lanes(vsrc + 1024 * i + 16 * ln,
                                 __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS void *)(vlds + r * VSTR + 1024 * i)),
                                 ln, n);
            }
        }
    }
#if KQ_ATTN_CELLS_OVERLAP
    waitcnt_vm_floor8(nv);  // this wave's score granules have landed (loads complete in order)
#else
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#endif
    __syncthreads();
#if KQ_ATTN_CELLS_STOP == 1
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    if (t < RS) a.out[(int64_t)h * HD + ds * RS + t] = w[t] + (float)vlds[t * VSTR];
    return;
#endif
    // soft_max (kq_attn_head.h, the general path): max (order-free), exps and the vaddvq group
    // sums, ggml's in-order double sum, p = e * (float)(1 / sum) -> f16. Thread t holds the
    // 4-cell groups t + 256 k in registers (one LDS read each, all issued together); the double
    // sum is a tree over the block where that is exact (softmax_group_sum's condition: every
    // group sum a float >= 2^(floor(log2(4 ng)) - 29), or zero), else the in-order sum of gsum.
    const int ng = n_kv >> 2;
    float4 ev[ATTN_CELLS_GMAX];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < ATTN_CELLS_GMAX; ++k) {
        const int gi = t + 256 * k;
        ev[k] = gi < ng ? ((const float4 *)w)[gi] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
        m = fmaxf(m, fmaxf(fmaxf(ev[k].x, ev[k].y), fmaxf(ev[k].z, ev[k].w)));
    }
    const float wmx = wave_fmax(m);
    if (ln == 0) scal[wv] = wmx;
    __syncthreads();  // (also: every score is in registers, the region is free)
    const float mx = fmaxf(fmaxf(scal[0], scal[1]), fmaxf(scal[2], scal[3]));
    SumExact se;
#pragma unroll
    for (int k = 0; k < ATTN_CELLS_GMAX; ++k) {
        const int gi = t + 256 * k;
        if (gi < ng) {
            float4 e = ev[k];
            e.x = e.x == -INFINITY ? 0.0f : v_expf(e.x - mx);
            e.y = e.y == -INFINITY ? 0.0f : v_expf(e.y - mx);
            e.z = e.z == -INFINITY ? 0.0f : v_expf(e.z - mx);
            e.w = e.w == -INFINITY ? 0.0f : v_expf(e.w - mx);
            ev[k] = e;
            const float gs = (e.x + e.y) + (e.z + e.w);
            gsum[gi] = (double)gs;
            se.add(gs);  // (exact when the total passes the bound: a subset's sum)
        }
    }
    const bool wbad = __any(se.bad);
    const int wgmin = wave_imin(se.gmin);
    double part = se.part;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    double *scald = (double *)(scal + 8);
    if (ln == 0) {
        scald[wv] = part;
        ((int *)scal)[4 + wv] = wgmin;
        ((int *)scal)[20 + wv] = wbad;
    }
    __syncthreads();
    const int *sgm = (const int *)scal + 4, *sbad = (const int *)scal + 20;
    const int gmin = min(min(sgm[0], sgm[1]), min(sgm[2], sgm[3]));
    const double st = (scald[0] + scald[1]) + (scald[2] + scald[3]);
    double sum;
    if (sum_exact_ok(st, gmin, (sbad[0] | sbad[1] | sbad[2] | sbad[3]) != 0)) {  // (uniform)
        sum = st;
    } else {
        if (t < 64) {
            const double s = KQ_SEQ_SUM_WAVE ? seq_sum_wave(gsum, ng, t) : seq_sum_lds(gsum, ng);
            if (t == 0) scald[4] = s;
        }
        __syncthreads();
        sum = scald[4];
    }
    __syncthreads();  // gsum's readers are done before p16 overwrites it
    const float inv = (float)(1.0 / sum);
#pragma unroll
    for (int k = 0; k < ATTN_CELLS_GMAX; ++k) {
        const int gi = t + 256 * k;
        if (gi < ng) {
            const uint32_t lo = (uint32_t)h2u(f2h_rne(ev[k].x * inv)) | ((uint32_t)h2u(f2h_rne(ev[k].y * inv)) << 16);
            const uint32_t hi = (uint32_t)h2u(f2h_rne(ev[k].z * inv)) | ((uint32_t)h2u(f2h_rne(ev[k].w * inv)) << 16);
            ((uint2 *)p16)[gi] = make_uint2(lo, hi);
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's V rows have landed
    __syncthreads();
#if KQ_ATTN_CELLS_STOP == 2
    if (t < RS) a.out[(int64_t)h * HD + ds * RS + t] = (float)p16[t] + (float)vlds[t * VSTR];
    return;
#endif
    // KQV: word q (f16 lanes 2q, 2q + 1) of accumulator j of output vr over cells 32 it + 8 j +
    // 2 q + {0, 1}, in order: 16 threads per output, each one chain of pk_fmas
    {
        const int vr = t >> 4, jq = t & 15;
        uint32_t acc1 = 0;
        if (vr < RS) {
            const uint32_t *vrow = (const uint32_t *)(vlds + vr * VSTR) + jq;
            const uint32_t *prow = (const uint32_t *)p16 + jq;
            int it = 0;
            for (; it + 16 <= n_it; it += 16) {
                uint32_t vb[16], pb[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    vb[k] = vrow[16 * (it + k)];
                    pb[k] = prow[16 * (it + k)];
                }
#pragma unroll
                for (int k = 0; k < 16; ++k) acc1 = pk_fma_w(vb[k], pb[k], acc1);
            }
            for (; it < n_it; ++it) acc1 = pk_fma_w(vrow[16 * it], prow[16 * it], acc1);
            red[t] = acc1;
        }
        __syncthreads();
    }
    // the GGML_F16_VEC_REDUCE of output vr_l's 4 accumulators: quad (vr_l, j = 0..3)
    const int vr_l = (t >> 2) & (RS - 1), j = t & 3;
    const bool kt = t < 4 * RS;
    uint32_t acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = red[16 * vr_l + 4 * j + k];
    const float o = f16x8_reduce_quad(acc);  // every lane active; quad (4 vr_l .. +3) holds output vr_l
    if (kt && j == 0) a.out[(int64_t)h * HD + ds * RS + vr_l] = bad ? __builtin_nanf("") : o;
}

// One workgroup per kv group (kq_attn_device.h): the group's cells [0, n_kv) are read
// once into LDS and serve its n_head/n_head_kv query heads, one wave each.
template <int HD>
__global__ void __launch_bounds__(1024) kq_attn_group(const AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    attn_group<HD>(a, blockIdx.x, smem, wave, (int)(blockDim.x >> 6), lane);
}

// ------------------------------------------------------------ prompt (batched) attention
// A prompt of T tokens in one graph (llama-bench pp: ggml's batched non-flash block —
// SET_ROWS writes the batch's T new cells, then KQ, soft_max with the causal mask and KQV
// for every query), two launches:
//  kq_kv_store: rope(k) -> f16 K cell, v -> f16 V cell (transposed) per (token, kv head);
//  kq_attn_prompt: one workgroup per (query head, token): the decode kernel's per-query
//  arithmetic (the general path of kq_attn_decode: KQ with the NEON FP16 structure, max,
//  ggml_v_expf, vaddvq group sums, the in-order double sum, KQV, the f16 reduce) reading
//  every cell from the caches. Cells after the query's position are masked: they add exact
//  zeros whatever they hold, so each query's output is the decode token's bit for bit.
template <int HD>
__global__ void __launch_bounds__(256) kq_kv_store(const AttnArgs a) {
    const int i = blockIdx.x, g = blockIdx.y, t = threadIdx.x;
    const int pos = a.pos[i];
    if (pos < 0 || pos >= a.n_ctx) return;  // no cell for this position (its output is NaN)
    const int kvw = a.n_head_kv * HD;
    const float *tc = a.rope_table + (int64_t)pos * (HD / 2) * 2;
    if (t < HD / 2) {
        const float *kp = a.k + (int64_t)i * kvw + (int64_t)g * HD + 2 * t;
        const float2 rk = rope_pair(kp[0], kp[1], tc[2 * t], tc[2 * t + 1]);
        const uint16_t k0 = h2u(f2h_rne(rk.x)), k1 = h2u(f2h_rne(rk.y));
        *(uint32_t *)(a.k_cache + (int64_t)pos * kvw + (int64_t)g * HD + 2 * t) = k0 | ((uint32_t)k1 << 16);
    } else if (t < HD / 2 + HD) {
        const int d = t - HD / 2;
        a.v_cache[(int64_t)(g * HD + d) * a.n_ctx + pos] = h2u(f2h_rne(a.v[(int64_t)i * kvw + (int64_t)g * HD + d]));
    }
}

// LDS: q16 (HD f16) | w (n_ctx f32) | p16 (n_ctx f16) | scal (4 f32) | gsum (n_ctx/4 f64)
size_t attn_prompt_lds(int hd, int n_ctx) {
    return (size_t)2 * hd + (size_t)n_ctx * 6 + 16 + (size_t)(n_ctx / 4) * 8;
}

template <int HD>
__global__ void __launch_bounds__(256) kq_attn_prompt(const AttnArgs a) {
    constexpr int KV4 = HD / 8;          // 16-B pieces of one K-cache row
    constexpr int ITEMS = HD * 4 / 256;  // KQV (d, j) items per thread
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int h = blockIdx.x, i = (int)gridDim.y - 1 - (int)blockIdx.y, t = threadIdx.x;  // latest tokens first
    const int g = h / (a.n_head / a.n_head_kv);
    const int kvw = a.n_head_kv * HD;
    const int64_t qrow = (int64_t)i * a.n_head * HD;
    const int pos_in = a.pos[i];
    const bool bad = pos_in < 0 || pos_in >= a.n_ctx;
    const int pos = bad ? 0 : pos_in;
    int n_kv = (pos + 1 + 31) / 32 * 32;
    n_kv = n_kv < a.n_ctx ? n_kv : a.n_ctx;
    uint16_t *q16 = (uint16_t *)smem;
    float *w = (float *)(smem + 2 * HD);
    uint16_t *p16 = (uint16_t *)(w + a.n_ctx);
    float *scal = (float *)(p16 + a.n_ctx);
    double *gsum = (double *)(scal + 4);

    if (t < HD / 2) {  // rope(q) at the query's position -> f16
        const float *qp = a.q + qrow + (int64_t)h * HD + 2 * t;
        const float *tc = a.rope_table + (int64_t)pos * (HD / 2) * 2;
        const float2 rq = rope_pair(qp[0], qp[1], tc[2 * t], tc[2 * t + 1]);
        q16[2 * t] = h2u(f2h_rne(rq.x));
        q16[2 * t + 1] = h2u(f2h_rne(rq.y));
    }
    __syncthreads();
    // KQ + scale + causal mask
    for (int c = t; c < n_kv; c += 256) {
        float sc = -INFINITY;
        if (c <= pos) {
            uint4 kv[KV4];
            const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)c * kvw + (int64_t)g * HD);
#pragma unroll
            for (int k = 0; k < KV4; ++k) kv[k] = kr[k];
            sc = vec_dot_f16_rows<HD>(kv, (const uint4 *)q16) * a.scale;
        }
        w[c] = sc;
    }
    __syncthreads();
    // soft_max: max (order-free), v_expf and the vaddvq group sums, the in-order double sum
    if (t < 64) {
        float m = -INFINITY;
        for (int c = t; c < n_kv; c += 64) m = fmaxf(m, w[c]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        if (t == 0) scal[0] = m;
    }
    __syncthreads();
    const float mx = scal[0];
    for (int gi = t; gi < n_kv / 4; gi += 256) {
        float e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float wv = w[4 * gi + k];
            e[k] = wv == -INFINITY ? 0.0f : v_expf(wv - mx);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) w[4 * gi + k] = e[k];
        gsum[gi] = (double)((e[0] + e[1]) + (e[2] + e[3]));
    }
    __syncthreads();
    if (t < 64) {  // ggml's in-order double sum (a tree where exact: softmax_group_sum)
        const float inv = (float)(1.0 / softmax_group_sum(gsum, n_kv / 4, t));
        if (t == 0) scal[1] = inv;
    }
    __syncthreads();
    const float inv = scal[1];
    for (int c = t; c < n_kv; c += 256) p16[c] = h2u(f2h_rne(w[c] * inv));
    __syncthreads();
    // KQV: thread (d, j) -> accumulator j of output d (cells 32it + 8j + l)
    const int n_it = (pos + 32) / 32;
#pragma unroll
    for (int ii = 0; ii < ITEMS; ++ii) {
        const int item = t + 256 * ii;
        const int d = item >> 2, j = item & 3;
        const uint16_t *vr = a.v_cache + (int64_t)(g * HD + d) * a.n_ctx;
        uint32_t acc[4] = {};  // lanes 2k, 2k+1 of accumulator j in word k
        for (int it0 = 0; it0 < n_it; it0 += 4) {  // 4 V chunks in flight per round trip
            uint4 vq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) vq[k] = it0 + k < n_it ? *(const uint4 *)(vr + 32 * (it0 + k) + 8 * j) : uint4{};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (it0 + k >= n_it) break;
                const uint4 pp = *(const uint4 *)(p16 + 32 * (it0 + k) + 8 * j);
                acc[0] = pk_fma_w(vq[k].x, pp.x, acc[0]);
                acc[1] = pk_fma_w(vq[k].y, pp.y, acc[1]);
                acc[2] = pk_fma_w(vq[k].z, pp.z, acc[2]);
                acc[3] = pk_fma_w(vq[k].w, pp.w, acc[3]);
            }
        }
        const float o = f16x8_reduce_quad(acc);  // accumulators j = 0..3 of output d: one quad
        if (j == 0) a.out[qrow + (int64_t)h * HD + d] = bad ? __builtin_nanf("") : o;
    }
}

// The same per-query arithmetic with one workgroup per (kv group, TPW tokens): the group's gsz
// query heads of TPW tokens share every K row and V chunk the workgroup loads (1/(gsz TPW) of
// the cache reads of kq_attn_prompt) and every barrier; each (token, head) row keeps its own
// scores, soft_max and accumulators.
constexpr int PROMPT_GMAX = 8;  // query heads per kv group handled by kq_attn_prompt_group
#ifndef KQ_PROMPT_SUMLANES
#define KQ_PROMPT_SUMLANES 1  // soft_max's in-order fallback sums: one lane per row, all rows at once
#endif
#ifndef KQ_PROMPT_TPW
#define KQ_PROMPT_TPW 1  // tokens per workgroup where the LDS holds them (2: measured 1.37x slower, profiles/r06_prompt_ab.txt)
#endif
#ifndef KQ_PROMPT_DIAG
#define KQ_PROMPT_DIAG 0  // timing-only builds: 1 no KQ dots, 2 no soft_max sums, 4 no KQV
#endif

// LDS: q16 [R][HD] | w [R][n_ctx] f32 | p16 [R][n_ctx] | scal [R][4] f32 (R = rows = gsz TPW),
//      with gsum [R][n_ctx/4] f64 over p16 (same bytes; read before p16 is written); the KQV
//      accumulators are reduced across lanes, not in LDS
size_t attn_prompt_group_lds(int hd, int n_ctx, int rows) {
    return (size_t)rows * ((size_t)2 * hd + (size_t)n_ctx * 6 + 16);
}

// GSZ: the group size fixed at compile time (4: Llama-3-8B, 8: TinyLlama / 70B), or 0 for
// any gsz <= PROMPT_GMAX: with it fixed, the per-head loops have no exits and hipcc keeps
// several LDS reads of KQV in flight (with the run-time exit it waited lgkmcnt(0) before
// every probability read). Every per-token loop runs over a compile-time TPW (unrolled: no
// array indexed at run time).
template <int HD, int GSZ = 0, int TPW = 1>
__global__ void __launch_bounds__(256) kq_attn_prompt_group(const AttnArgs a) {
    constexpr int KV4 = HD / 8;
    constexpr int ITEMS = HD * 4 / 256;
    constexpr int GM = GSZ > 0 ? GSZ : PROMPT_GMAX;  // heads the unrolled loops cover
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // tokens [i0, i0 + TPW), the latest first (the most cells: a shorter tail); i0 + tt < 0: none
    const int g = blockIdx.x, t = threadIdx.x;
    const int i0 = a.n_tok - TPW * (1 + (int)blockIdx.y);
    const int gsz = GSZ > 0 ? GSZ : a.n_head / a.n_head_kv;  // <= PROMPT_GMAX (host check)
    const int kvw = a.n_head_kv * HD;
    const int nc = a.n_ctx;
    int posv[TPW], nkv[TPW];
    bool badv[TPW], live[TPW];
    int nkv_max = 0, pos_max = -1;
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
        live[tt] = i0 + tt >= 0;
        const int pos_in = live[tt] ? a.pos[i0 + tt] : 0;
        badv[tt] = pos_in < 0 || pos_in >= nc;
        posv[tt] = badv[tt] ? 0 : pos_in;
        int n = (posv[tt] + 1 + 31) / 32 * 32;
        nkv[tt] = !live[tt] ? 0 : n < nc ? n : nc;
        nkv_max = nkv[tt] > nkv_max ? nkv[tt] : nkv_max;
        pos_max = live[tt] && posv[tt] > pos_max ? posv[tt] : pos_max;
    }
    const int R = TPW * gsz;                                // rows r = tt gsz + hh
    uint16_t *q16 = (uint16_t *)smem;                       // [R][HD]
    float *w = (float *)(q16 + R * HD);                     // [R][nc]
    uint16_t *p16 = (uint16_t *)(w + R * nc);               // [R][nc]
    float *scal = (float *)(p16 + R * nc);                  // [R][4]: max, 1 / sum, tree exact
    double *gsum = (double *)p16;                           // [R][nc/4], before p16

#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {  // rope(q) of the group's heads -> f16
        if (!live[tt]) continue;
        const int64_t qrow = (int64_t)(i0 + tt) * a.n_head * HD;
        const float *tc = a.rope_table + (int64_t)posv[tt] * (HD / 2) * 2;
        for (int u = t; u < gsz * (HD / 2); u += 256) {
            const int hh = u / (HD / 2), pr = u - hh * (HD / 2);
            const float *qp = a.q + qrow + (int64_t)(g * gsz + hh) * HD + 2 * pr;
            const float2 rq = rope_pair(qp[0], qp[1], tc[2 * pr], tc[2 * pr + 1]);
            q16[(tt * gsz + hh) * HD + 2 * pr] = h2u(f2h_rne(rq.x));
            q16[(tt * gsz + hh) * HD + 2 * pr + 1] = h2u(f2h_rne(rq.y));
        }
    }
    __syncthreads();
    // KQ: thread t owns cells t, t + 256, ...: one K row load serves every row of the workgroup
    for (int c = t; c < nkv_max; c += 256) {
        if (c <= pos_max) {
            uint4 kv[KV4];
            const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)c * kvw + (int64_t)g * HD);
#pragma unroll
            for (int k = 0; k < KV4; ++k) kv[k] = kr[k];
#pragma unroll
            for (int tt = 0; tt < TPW; ++tt) {
                const bool on = c <= posv[tt] && live[tt];
#pragma unroll
                for (int hh = 0; hh < GM; ++hh)
                    if (GSZ > 0 || hh < gsz)
                        w[(tt * gsz + hh) * nc + c] =
                            !on ? -INFINITY
                                : (KQ_PROMPT_DIAG & 1) ? __uint_as_float(kv[0].x ^ kv[KV4 - 1].w) * 1e-30f
                                                       : vec_dot_f16_rows<HD>(kv, (const uint4 *)(q16 + (tt * gsz + hh) * HD)) * a.scale;
            }
        } else {
            for (int r = 0; r < TPW * gsz; ++r) w[r * nc + c] = -INFINITY;
        }
    }
    __syncthreads();
    // soft_max per row: max (one wave per row, order-free), exp + vaddvq group sums
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
        for (int hh = t >> 6; hh < gsz; hh += 4) {
            const int l = t & 63, r = tt * gsz + hh;
            float m = -INFINITY;
            for (int c = l; c < nkv[tt]; c += 64) m = fmaxf(m, w[r * nc + c]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
            if (l == 0) scal[4 * r] = m;
        }
    __syncthreads();
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
        const int ng = nkv[tt] / 4;
        for (int u = t; u < gsz * ng; u += 256) {
            const int hh = u / ng, gi = u - hh * ng, r = tt * gsz + hh;
            const float mx = scal[4 * r];
            float e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float wv = w[r * nc + 4 * gi + k];
                e[k] = wv == -INFINITY ? 0.0f : v_expf(wv - mx);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) w[r * nc + 4 * gi + k] = e[k];
            gsum[r * (nc / 4) + gi] = (double)((e[0] + e[1]) + (e[2] + e[3]));
        }
    }
    __syncthreads();
    if (KQ_PROMPT_DIAG & 2) {
        if (t < R) scal[4 * t + 1] = (float)gsum[t * (nc / 4)];
    } else {
        // ggml's in-order double sums: a wave tree per row where that is provably exact; the
        // other rows' in-order chains then run one lane per row, all at once (a wave per row
        // ran them one after another)
#pragma unroll
        for (int tt = 0; tt < TPW; ++tt)
            for (int hh = t >> 6; hh < gsz; hh += 4) {
                const int r = tt * gsz + hh, ng = nkv[tt] / 4;
                bool ok = true;
                const double s = ng > 0 ? softmax_group_tree(gsum + r * (nc / 4), ng, t & 63, ok) : 0.0;
                if ((t & 63) == 0) {
                    scal[4 * r + 1] = (float)(1.0 / s);
                    ((int *)scal)[4 * r + 2] = ok;
                }
            }
        __syncthreads();
        int ngr = 0;  // row t's groups (t < R)
#pragma unroll
        for (int tt = 0; tt < TPW; ++tt) ngr = t / gsz == tt ? nkv[tt] / 4 : ngr;
        if (KQ_PROMPT_SUMLANES) {
            if (t < R && !((const int *)scal)[4 * t + 2]) scal[4 * t + 1] = (float)(1.0 / seq_sum_lds(gsum + t * (nc / 4), ngr));
        } else {  // (A/B builds: a wave per row, in turn)
#pragma unroll
            for (int tt = 0; tt < TPW; ++tt)
                for (int hh = t >> 6; hh < gsz; hh += 4) {
                    const int r = tt * gsz + hh;
                    if (!((const int *)scal)[4 * r + 2]) {
                        const double s = seq_sum_lds(gsum + r * (nc / 4), nkv[tt] / 4);
                        if ((t & 63) == 0) scal[4 * r + 1] = (float)(1.0 / s);
                    }
                }
        }
    }
    __syncthreads();
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt)
        for (int u = t; u < gsz * nkv[tt]; u += 256) {
            const int hh = u / nkv[tt], c = u - hh * nkv[tt], r = tt * gsz + hh;
            p16[r * nc + c] = h2u(f2h_rne(w[r * nc + c] * scal[4 * r + 1]));
        }
    __syncthreads();
    // KQV: thread (d, j) -> accumulator j of output d of every row; one V chunk per (d, j, it)
    // serves them all. A token's iterations past its own cells are computed and discarded (a
    // select: the V cells there need not be finite), so every accumulator sees exactly its
    // token's iterations, in order.
    int nit[TPW], nit_max = 0;
#pragma unroll
    for (int tt = 0; tt < TPW; ++tt) {
        nit[tt] = !live[tt] ? 0 : (KQ_PROMPT_DIAG & 4) ? 1 : (posv[tt] + 32) / 32;
        nit_max = nit[tt] > nit_max ? nit[tt] : nit_max;
    }
#pragma unroll
    for (int ii = 0; ii < ITEMS; ++ii) {
        const int item = t + 256 * ii;
        const int d = item >> 2, j = item & 3;
        const uint16_t *vr = a.v_cache + (int64_t)(g * HD + d) * nc;
        uint32_t acc[TPW][GM][4] = {};  // lanes 2k, 2k+1 of row (tt, hh)'s accumulator j in word k
        // one 32-cell iteration: its V chunk against every row's probabilities
        auto step = [&](const uint4 &vv, int it) {
            const int c0 = 32 * it + 8 * j;
            const uint32_t vw[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
            for (int tt = 0; tt < TPW; ++tt) {
                const bool on = TPW == 1 || it < nit[tt];
#pragma unroll
                for (int hh = 0; hh < GM; ++hh) {
                    if (GSZ == 0 && hh >= gsz) break;
                    const uint4 pp = *(const uint4 *)(p16 + (tt * gsz + hh) * nc + c0);
                    const uint32_t n0 = pk_fma_w(vw[0], pp.x, acc[tt][hh][0]);
                    const uint32_t n1 = pk_fma_w(vw[1], pp.y, acc[tt][hh][1]);
                    const uint32_t n2 = pk_fma_w(vw[2], pp.z, acc[tt][hh][2]);
                    const uint32_t n3 = pk_fma_w(vw[3], pp.w, acc[tt][hh][3]);
                    acc[tt][hh][0] = on ? n0 : acc[tt][hh][0];
                    acc[tt][hh][1] = on ? n1 : acc[tt][hh][1];
                    acc[tt][hh][2] = on ? n2 : acc[tt][hh][2];
                    acc[tt][hh][3] = on ? n3 : acc[tt][hh][3];
                }
            }
        };
        int it = 0;
        for (; it + 4 <= nit_max; it += 4) {  // whole batches: 4 V chunks in flight, no guards
            uint4 vq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) vq[k] = *(const uint4 *)(vr + 32 * (it + k) + 8 * j);
#pragma unroll
            for (int k = 0; k < 4; ++k) step(vq[k], it + k);
        }
        for (; it < nit_max; ++it) step(*(const uint4 *)(vr + 32 * it + 8 * j), it);
        // the 4 accumulators of output d sit in the 4 lanes of a quad (j = t & 3)
#pragma unroll
        for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
            for (int hh = 0; hh < GM; ++hh) {
                if (GSZ == 0 && hh >= gsz) break;
                const float o = badv[tt] ? __builtin_nanf("") : f16x8_reduce_quad(acc[tt][hh]);
                if (j == 0 && live[tt]) {
                    a.out[(int64_t)(i0 + tt) * a.n_head * HD + (int64_t)(g * gsz + hh) * HD + d] = o;
                    if (a.q8_out) w[(tt * gsz + hh) * HD + d] = o;  // staged for the Q8L blocks (w is free now)
                }
            }
    }
    if (a.q8_out) {  // each token's gsz*HD outputs (whole superblocks of its row) -> Q8L
        __syncthreads();
        const int nsb = gsz * HD / QK, l = t & 15;
        for (int rid = t >> 4; rid < TPW * nsb; rid += 16) {  // uniform over each 16-lane row (quant16_store's DPP row)
            const int tt = rid / nsb, sb = rid - tt * nsb;
            if (i0 + tt < 0) continue;
            const float *src = w + rid * QK + 16 * l;
            u32x4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 f = ((const float4 *)src)[k];
                v[k] = u32x4{__float_as_uint(f.x), __float_as_uint(f.y), __float_as_uint(f.z), __float_as_uint(f.w)};
            }
            const int64_t nbr = (int64_t)a.n_head * HD / QK;  // superblocks per row
            quant16_store<true>(v, l, a.q8_out + ((int64_t)(i0 + tt) * nbr + (int64_t)g * nsb + sb) * Q8L_STRIDE);
        }
    }
}

size_t attn_lds(int hd, int n_ctx) {
    const size_t gsum = (size_t)(n_ctx / 4) * 8 <= (size_t)hd * 64 ? 0 : (size_t)(n_ctx / 4) * 8;
    return (size_t)6 * hd + (size_t)n_ctx * 6 + (size_t)hd * 64 + 16 + gsum;
}
// ... plus the head's V rows (v_lds, or a 1/ds slice of them): rows of n_ctx f16, 16 B of
// padding each
size_t attn_lds_v(int hd, int n_ctx, int ds = 1, bool ring = false) {
    return (attn_lds(hd, n_ctx) + 15) / 16 * 16 + (size_t)(hd / ds) * ((size_t)n_ctx * 2 + 16) +
           (ds > 1 || ring ? (size_t)4 * KQ_ATTN_KD * ATTN_KSLOT : 0);  // + the K ring (KDMA)
}
#ifndef KQ_ATTN_DSMIN
#define KQ_ATTN_DSMIN 4  // (experiment builds: 8)
#endif
// Output slices per head for a cache of n_ctx cells (1: no split): past the register path's
// KQ_ATTN_BATCH_CTX cells, the fewest of 4 / 8 whose V slice fits the LDS beside the rest.
// Every slice scores every cell, so the K reads grow with the slices: 16 slices at 4096 cells
// (head_dim 64) measured slower than one workgroup per head (tg4096 894 against 925 tok/s,
// profiles/r05_attn_split_ab.txt).
// The split path LDS-DMAs whole K-cache rows and V rows (16-B pieces at 16-B offsets from the
// cache bases: both caches must be 16-B aligned, else the per-head kernel runs) and stages q / k
// / v and the rope row with 16-B transfers from 4-B aligned f32 vectors: the global side of an
// LDS-DMA need not be 16-B aligned on this device (the decode graph's staged rope row sits 8 B
// into its input tensor: every decode-graph test past 256 cells runs that way).
int attn_slices(const AttnArgs &a) {
    const uintptr_t mis16 = (uintptr_t)a.v_cache | (uintptr_t)a.k_cache;
    const uintptr_t mis4 = (uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v | (uintptr_t)a.rope_table;
    if (attn_impl() != MI355X_ATTN_SPLIT || a.n_ctx <= KQ_ATTN_BATCH_CTX || a.n_ctx % 8 || (mis16 & 15u) ||
        (mis4 & 3u))
        return 1;
    for (int ds = KQ_ATTN_DSMIN; ds <= 8; ds *= 2)
        if (attn_lds_v(a.head_dim, a.n_ctx, ds) <= 160 * 1024) return ds;
    return 1;
}

// ------------------------------------------------------------ launch helpers
int check_launch() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

template <typename K, typename... Args>
int timed_launch(const char *name, double bytes, K kern, dim3 grid, dim3 block, size_t lds, hipStream_t s,
                 Args... args) {
    hipEvent_t e0, e1;
    if (timing_slot(s, e0, e1)) {
        hipExtLaunchKernelGGL(kern, grid, block, (uint32_t)lds, s, e0, e1, 0, args...);
        timing_log(name, bytes, e0, e1);
    } else {
        hipLaunchKernelGGL(kern, grid, block, lds, s, args...);
    }
    return check_launch();
}

int elem_grid(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

int launch_rms_norm(const float *x, const float *w, float *y, int64_t n, int64_t nrows, float eps, hipStream_t s) {
    if (nrows == 0) return MI355X_OK;
    return timed_launch("kq::kq_rms_norm", (double)nrows * n * 8 + (w ? n * 4.0 : 0.0), kq_rms_norm,
                        dim3((unsigned)nrows), dim3(256), (size_t)(n / QK) * 8 + 8, s, x, w, y, n, eps);
}

int launch_binary(int op, const float *a, const float *b, float *y, int64_t n, hipStream_t s, int64_t nb) {
    if (n == 0) return MI355X_OK;
    if (nb <= 0) nb = n;
    if (n % nb) return MI355X_E_INVAL;
    return timed_launch(op == 0 ? "kq::kq_add" : "kq::kq_mul", n * 8.0 + nb * 4.0, kq_binary, dim3(elem_grid(n)),
                        dim3(256), 0, s, op, a, b, y, n, nb);
}

int launch_swiglu(const float *g, const float *u, float *y, int64_t n, hipStream_t s) {
    if (n == 0) return MI355X_OK;
    return timed_launch("kq::kq_swiglu", n * 12.0, kq_swiglu, dim3(elem_grid(n)), dim3(256), 0, s, g, u, y, n);
}

int attn_group_waves(const AttnArgs &a) {
    const int gsz = a.n_head / a.n_head_kv;
    return gsz < 4 ? 4 : gsz > 16 ? 16 : gsz;
}

size_t attn_group_bytes(const AttnArgs &a, int nwaves) {
    const int gsz = a.n_head / a.n_head_kv;
    return (size_t)attn_group_lds(a.head_dim, a.n_ctx, gsz < nwaves ? gsz : nwaves).total;
}

bool attn_group_ok(const AttnArgs &a, int nwaves) {
    const uintptr_t m = (uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v;  // 8-B pair loads
    return (m & 7u) == 0 && a.diag == 0 && attn_group_bytes(a, nwaves) <= 160 * 1024;
}

// MI355X_ATTN_SPLIT (the default: one workgroup per query head, split by output past 256
// cells: profiles/r05_attn_split_ab.txt), MI355X_ATTN_HEAD (one workgroup per query head at
// every size) or MI355X_ATTN_GROUP (one workgroup per kv group: each group's cells read
// once, 1/gsz of the cache traffic, +2.3 us per launch on the TinyLlama token:
// profiles/r02_attention_ab.md). Set only through mi355x_attn_impl().
#ifndef KQ_ATTN_DEFAULT_IMPL  // (experiment builds: the selector's initial value)
#define KQ_ATTN_DEFAULT_IMPL MI355X_ATTN_SPLIT
#endif
std::atomic<int> g_attn_impl{KQ_ATTN_DEFAULT_IMPL};
int attn_impl() { return g_attn_impl.load(); }

size_t attn_cells_lds_a(int hd, int gsz) { return (size_t)gsz * hd * 2 + (size_t)hd * 2 + (size_t)ATTN_CHUNK * hd * 2; }
// B's LDS: the scores region (p16 and the group sums reuse it), red, 96 B of scalars, and RS V
// rows of 2 n_ctx + VPAD bytes
size_t attn_cells_lds_b(int n_ctx, int rs) {
    return (size_t)n_ctx * 4 + (size_t)rs * 64 + 96 + (size_t)rs * (2 * (size_t)n_ctx + ATTN_CELLS_VPAD);
}
// head_dim 128: RS 16 (one round of workgroups) where its V rows fit the LDS, else 8
int attn_cells_rs(int hd, int n_ctx) {
    if (hd == 64) return KQ_ATTN_CELLS_RS64;
    return attn_cells_lds_b(n_ctx, KQ_ATTN_CELLS_RS128) <= 160 * 1024 ? KQ_ATTN_CELLS_RS128 : 8;
}

// The score workspace [n_head][n_ctx] f32: one grow-only buffer per (device, stream), so two
// streams' attentions never share one, allocated outside any stream capture (the backend
// reserves before it captures: attn_cells_reserve). An older, smaller buffer stays allocated:
// a captured graph may still point at it.
struct CellsScratch {
    struct Entry {
        int dev;
        hipStream_t stream;
        void *p;
        size_t bytes;
    };
    std::mutex mu;
    std::vector<Entry> cur;
};
CellsScratch &cells_scratch() {
    static CellsScratch s;
    return s;
}
void *attn_cells_buffer(size_t bytes, hipStream_t stream, bool may_alloc) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    CellsScratch &cs = cells_scratch();
    std::lock_guard<std::mutex> lk(cs.mu);
    for (auto &e : cs.cur)
        if (e.dev == dev && e.stream == stream) {
            if (e.bytes >= bytes) return e.p;
            if (!may_alloc) return nullptr;
            void *p = nullptr;
            if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
            e.p = p, e.bytes = bytes;  // (the old one is kept: graphs may read it)
            return p;
        }
    if (!may_alloc) return nullptr;
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    cs.cur.push_back({dev, stream, p, bytes});
    return p;
}

bool attn_cells_applies(const AttnArgs &a) {
    const int gsz = a.n_head_kv > 0 ? a.n_head / a.n_head_kv : 0;
    return attn_impl() == MI355X_ATTN_SPLIT && a.n_ctx > KQ_ATTN_CELLS_MIN && a.n_ctx % ATTN_CHUNK == 0 &&
           a.n_ctx <= 1024 * ATTN_CELLS_GMAX &&
           (a.head_dim == 64 || a.head_dim == 128) && gsz >= 1 && gsz <= 16 &&
           (KQ_ATTN_CELLS_OVER_SPLIT || attn_slices(a) == 1 || attn_slices(a) >= KQ_ATTN_CELLS_SLICES) &&
           attn_cells_lds_b(a.n_ctx, attn_cells_rs(a.head_dim, a.n_ctx)) <= 160 * 1024 && ((uintptr_t)a.k_cache & 15u) == 0 &&
           ((uintptr_t)a.v_cache & 15u) == 0;
}

// The workspace of a decode attention that will take the two launches, allocated now (callers
// that capture graphs call this first; an eager launch allocates on its own)
int attn_cells_reserve(const AttnArgs &a, hipStream_t stream) {
    if (!attn_cells_applies(a)) return MI355X_OK;
    return attn_cells_buffer((size_t)a.n_head * a.n_ctx * 4, stream, true) ? MI355X_OK : MI355X_E_WORKSPACE;
}

template <int HD, int RS>
int launch_attn_cells_t(const AttnArgs &a, float *ws, hipStream_t s, const char *na, const char *nb) {
    const int gsz = a.n_head / a.n_head_kv;
    const size_t la = attn_cells_lds_a(HD, gsz), lb = attn_cells_lds_b(a.n_ctx, RS);
    const dim3 ga((unsigned)(a.n_ctx / ATTN_CHUNK), (unsigned)a.n_head_kv);
    const int rc = timed_launch(na, 0.0, kq_attn_cells<HD>, ga, dim3(256), la, s, a, ws);
    if (rc) return rc;
    allow_lds((const void *)kq_attn_cells_kqv<HD, HD / RS>, lb);
    return timed_launch(nb, 0.0, kq_attn_cells_kqv<HD, HD / RS>, dim3((unsigned)(a.n_head * (HD / RS))), dim3(256), lb, s,
                        a, (const float *)ws);
}
int launch_attn_cells(const AttnArgs &a, float *ws, hipStream_t s) {
    if (a.head_dim == 64)
        return launch_attn_cells_t<64, KQ_ATTN_CELLS_RS64>(a, ws, s, "kq::kq_attn_cells<64>", "kq::kq_attn_cells_kqv<64>");
    if (attn_cells_rs(128, a.n_ctx) == KQ_ATTN_CELLS_RS128)
        return launch_attn_cells_t<128, KQ_ATTN_CELLS_RS128>(a, ws, s, "kq::kq_attn_cells<128>", "kq::kq_attn_cells_kqv<128>");
    return launch_attn_cells_t<128, 8>(a, ws, s, "kq::kq_attn_cells<128>", "kq::kq_attn_cells_kqv<128>");
}

// The kernel launch_attn runs for these arguments (mi355x_attn_path; a captured launch without
// a reserved workspace takes MI355X_ATTN_PATH_HEAD_BATCH instead of the cells split).
int attn_path(const AttnArgs &a) {
    if (attn_impl() == MI355X_ATTN_GROUP && attn_group_ok(a, attn_group_waves(a))) return MI355X_ATTN_PATH_GROUP;
    const int ds = attn_slices(a);
    if (ds > 1 && !attn_cells_applies(a)) return ds == 4 ? MI355X_ATTN_PATH_SPLIT4 : MI355X_ATTN_PATH_SPLIT8;
    if (attn_cells_applies(a)) return MI355X_ATTN_PATH_CELLS;
    if (KQ_ATTN_KDMA1 && a.n_ctx <= KQ_ATTN_BATCH_CTX && a.n_ctx % 8 == 0 && ((uintptr_t)a.v_cache & 15u) == 0 &&
        ((uintptr_t)a.k_cache & 15u) == 0)
        return MI355X_ATTN_PATH_KD1;
    return a.n_ctx > KQ_ATTN_BATCH_CTX ? MI355X_ATTN_PATH_HEAD_BATCH : MI355X_ATTN_PATH_HEAD;
}

int launch_attn(const AttnArgs &a, hipStream_t s) {
    const double bytes = 0;  // context-dependent; not a roofline kernel
    const int path = attn_path(a);
    if (path == MI355X_ATTN_PATH_GROUP) {
        const int nw = attn_group_waves(a);
        const size_t glds = attn_group_bytes(a, nw);
        if (a.head_dim == 64) {
            allow_lds((const void *)kq_attn_group<64>, glds);
            return timed_launch("kq::kq_attn_group<64>", bytes, kq_attn_group<64>, dim3(a.n_head_kv), dim3(64 * nw),
                                glds, s, a);
        }
        allow_lds((const void *)kq_attn_group<128>, glds);
        return timed_launch("kq::kq_attn_group<128>", bytes, kq_attn_group<128>, dim3(a.n_head_kv), dim3(64 * nw),
                            glds, s, a);
    }
    // Past the register path's 256 cells the V rows go to LDS by LDS-DMA as soon as the position
    // is known (all of them in flight under KQ and soft_max) where they fit; shorter caches keep
    // the register prefetch, which issues V with the position itself.
    AttnArgs b = a;
    const int ds = attn_slices(a);
    if (path == MI355X_ATTN_PATH_SPLIT4 || path == MI355X_ATTN_PATH_SPLIT8) {
        const size_t lds = attn_lds_v(a.head_dim, a.n_ctx, ds);
        const dim3 grid((unsigned)(a.n_head * ds));
#define KQ_ATTN_SPLIT_LAUNCH(HD, DS)                                                                        \
    if (a.head_dim == HD && ds == DS) {                                                                    \
        allow_lds((const void *)kq_attn_decode<HD, true, DS>, lds);                                        \
        return timed_launch("kq::kq_attn_decode<" #HD ", true, " #DS ">", bytes, kq_attn_decode<HD, true, DS>, \
                            grid, dim3(256), lds, s, b);                                                   \
    }
        KQ_ATTN_SPLIT_LAUNCH(64, 4)
        KQ_ATTN_SPLIT_LAUNCH(64, 8)
        KQ_ATTN_SPLIT_LAUNCH(128, 4)
        KQ_ATTN_SPLIT_LAUNCH(128, 8)
#undef KQ_ATTN_SPLIT_LAUNCH
        return MI355X_E_INVAL;
    }
    if (path == MI355X_ATTN_PATH_CELLS) {  // long caches past the output split: KQ split over cells, two launches
        hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
        const bool capturing = hipStreamIsCapturing(s, &cst) == hipSuccess && cst != hipStreamCaptureStatusNone;
        void *ws = attn_cells_buffer((size_t)a.n_head * a.n_ctx * 4, s, !capturing);
        if (ws) return launch_attn_cells(a, (float *)ws, s);
        // (captured without a reserved workspace: the one-launch kernel below)
    }
    if (path == MI355X_ATTN_PATH_KD1) {
        const size_t lds = attn_lds_v(a.head_dim, a.n_ctx, 1, true);
        if (a.head_dim == 64) {
            allow_lds((const void *)kq_attn_decode<64, true, 1, 256, true>, lds);
            return timed_launch("kq::kq_attn_decode<64, true, 1, kd1>", bytes, kq_attn_decode<64, true, 1, 256, true>,
                                dim3(a.n_head), dim3(256), lds, s, b);
        }
        allow_lds((const void *)kq_attn_decode<128, true, 1, 256, true>, lds);
        return timed_launch("kq::kq_attn_decode<128, true, 1, kd1>", bytes, kq_attn_decode<128, true, 1, 256, true>,
                            dim3(a.n_head), dim3(256), lds, s, b);
    }
    b.v_lds = a.n_ctx > KQ_ATTN_BATCH_CTX && a.n_ctx % 8 == 0 && attn_lds_v(a.head_dim, a.n_ctx) <= 160 * 1024 &&
              ((uintptr_t)a.v_cache & 15u) == 0 && KQ_ATTN_VLDS;
    const size_t lds = b.v_lds ? attn_lds_v(a.head_dim, a.n_ctx) : attn_lds(a.head_dim, a.n_ctx);
    const bool batch = a.n_ctx > KQ_ATTN_BATCH_CTX;
    if (a.head_dim == 64) {
        if (!batch)
            return timed_launch("kq::kq_attn_decode<64, false>", bytes, kq_attn_decode<64, false, 1, KQ_ATTN_TPH64>,
                                dim3(a.n_head), dim3(KQ_ATTN_TPH64), lds, s, b);
        if (b.v_lds) allow_lds((const void *)kq_attn_decode<64, true>, lds);
        return timed_launch("kq::kq_attn_decode<64, true>", bytes, kq_attn_decode<64, true>, dim3(a.n_head), dim3(256), lds, s, b);
    }
    if (!batch) return timed_launch("kq::kq_attn_decode<128, false>", bytes, kq_attn_decode<128, false>, dim3(a.n_head), dim3(256), lds, s, b);
    if (b.v_lds) allow_lds((const void *)kq_attn_decode<128, true>, lds);
    return timed_launch("kq::kq_attn_decode<128, true>", bytes, kq_attn_decode<128, true>, dim3(a.n_head), dim3(256), lds, s, b);
}

// mi355x_attn_prompt_impl: MI355X_ATTN_GROUP (default: one workgroup per kv group and token
// where the group fits) or MI355X_ATTN_HEAD (one per query head and token)
std::atomic<int> g_prompt_impl{MI355X_ATTN_GROUP};

bool attn_prompt_group_ok(const AttnArgs &a) {
    const int gsz = a.n_head / a.n_head_kv;
    return gsz <= PROMPT_GMAX && attn_prompt_group_lds(a.head_dim, a.n_ctx, gsz) <= 160 * 1024 &&
           g_prompt_impl.load() == MI355X_ATTN_GROUP;
}
// tokens per workgroup: KQ_PROMPT_TPW where its rows fit the LDS (fixed group sizes), else 1
int attn_prompt_tpw(const AttnArgs &a) {
    const int gsz = a.n_head / a.n_head_kv;
    return KQ_PROMPT_TPW > 1 && (gsz == 4 || gsz == 8) &&
                   attn_prompt_group_lds(a.head_dim, a.n_ctx, gsz * KQ_PROMPT_TPW) <= 160 * 1024
               ? KQ_PROMPT_TPW
               : 1;
}

// Q8L rows written by the group kernel: its slice (gsz*head_dim) must be whole superblocks
bool attn_prompt_q8_ok(const AttnArgs &a) {
    return attn_prompt_group_ok(a) && ((a.n_head / a.n_head_kv) * a.head_dim) % QK == 0 &&
           a.n_ctx >= a.head_dim;  // staged in the score rows: gsz*head_dim floats
}

int launch_attn_prompt(const AttnArgs &a0, int n_tok, hipStream_t s) {
    if (n_tok <= 0) return MI355X_OK;
    AttnArgs a = a0;
    a.n_tok = n_tok;
    const size_t lds = attn_prompt_lds(a.head_dim, a.n_ctx);
    const int gsz = a.n_head / a.n_head_kv;
    // one workgroup per (kv group, TPW tokens) where the rows fit: 1/(gsz TPW) of the cache reads
    const bool group = attn_prompt_group_ok(a);
    if (a.q8_out && !group) return MI355X_E_INVAL;  // only the group kernel writes the Q8L rows
    const int tpw = group ? attn_prompt_tpw(a) : 1;
    const size_t glds = attn_prompt_group_lds(a.head_dim, a.n_ctx, gsz * tpw);
    const dim3 gs((unsigned)n_tok, (unsigned)a.n_head_kv), ga((unsigned)a.n_head, (unsigned)n_tok);
    const dim3 gg((unsigned)a.n_head_kv, (unsigned)((n_tok + tpw - 1) / tpw));
    int rc;
#define KQ_PROMPT_GROUP_LAUNCH(HD, G, T)                                                                  \
    {                                                                                                   \
        allow_lds((const void *)kq_attn_prompt_group<HD, G, T>, glds);                                  \
        return timed_launch("kq::kq_attn_prompt_group<" #HD ">", 0.0, kq_attn_prompt_group<HD, G, T>, gg, \
                            dim3(256), glds, s, a);                                                     \
    }
    if (a.head_dim == 64) {
        rc = a.no_store ? 0 : timed_launch("kq::kq_kv_store<64>", 0.0, kq_kv_store<64>, gs, dim3(256), 0, s, a);
        if (rc) return rc;
        if (group) {
            if (gsz == 8 && tpw > 1) KQ_PROMPT_GROUP_LAUNCH(64, 8, KQ_PROMPT_TPW)
            if (gsz == 4 && tpw > 1) KQ_PROMPT_GROUP_LAUNCH(64, 4, KQ_PROMPT_TPW)
            if (gsz == 8) KQ_PROMPT_GROUP_LAUNCH(64, 8, 1)
            if (gsz == 4) KQ_PROMPT_GROUP_LAUNCH(64, 4, 1)
            KQ_PROMPT_GROUP_LAUNCH(64, 0, 1)
        }
        allow_lds((const void *)kq_attn_prompt<64>, lds);
        return timed_launch("kq::kq_attn_prompt<64>", 0.0, kq_attn_prompt<64>, ga, dim3(256), lds, s, a);
    }
    rc = a.no_store ? 0 : timed_launch("kq::kq_kv_store<128>", 0.0, kq_kv_store<128>, gs, dim3(256), 0, s, a);
    if (rc) return rc;
    if (group) {
        if (gsz == 8 && tpw > 1) KQ_PROMPT_GROUP_LAUNCH(128, 8, KQ_PROMPT_TPW)
        if (gsz == 4 && tpw > 1) KQ_PROMPT_GROUP_LAUNCH(128, 4, KQ_PROMPT_TPW)
        if (gsz == 8) KQ_PROMPT_GROUP_LAUNCH(128, 8, 1)
        if (gsz == 4) KQ_PROMPT_GROUP_LAUNCH(128, 4, 1)
        KQ_PROMPT_GROUP_LAUNCH(128, 0, 1)
    }
#undef KQ_PROMPT_GROUP_LAUNCH
    allow_lds((const void *)kq_attn_prompt<128>, lds);
    return timed_launch("kq::kq_attn_prompt<128>", 0.0, kq_attn_prompt<128>, ga, dim3(256), lds, s, a);
}

int check_attn(const AttnArgs &a) {
    if (!a.q || !a.k || !a.v || !a.pos || !a.rope_table || !a.k_cache || !a.v_cache || !a.out) return MI355X_E_INVAL;
    if (a.head_dim != 64 && a.head_dim != 128) return MI355X_E_UNSUPPORTED;
    if (a.n_head <= 0 || a.n_head_kv <= 0 || a.n_head % a.n_head_kv) return MI355X_E_INVAL;
    if (a.n_ctx < 32 || a.n_ctx % 32 || a.n_ctx > 8192) return MI355X_E_UNSUPPORTED;
    if (((uintptr_t)a.k_cache & 15u) || ((uintptr_t)a.v_cache & 15u)) return MI355X_E_INVAL;
    if (attn_lds(a.head_dim, a.n_ctx) > 64 * 1024) return MI355X_E_UNSUPPORTED;
    return MI355X_OK;
}

uint64_t ops_selector_key() {
    return (uint64_t)(uint32_t)attn_impl() | ((uint64_t)(uint32_t)g_prompt_impl.load() << 8);
}

}  // namespace kq

using namespace kq;

extern "C" {

int mi355x_get_rows(int type, const void *table, int64_t ne0, size_t row_stride, int64_t n_rows, const int32_t *ids,
                    int64_t n_ids, float *dst, void *stream) {
    if (!table || !ids || !dst || ne0 <= 0 || n_ids < 0 || n_rows < 0) return MI355X_E_INVAL;
    if (type != MI355X_TYPE_F32 && type != MI355X_TYPE_Q4_K && type != MI355X_TYPE_Q5_K && type != MI355X_TYPE_Q6_K)
        return MI355X_E_UNSUPPORTED;
    if (ne0 % (type == MI355X_TYPE_F32 ? 8 : QK)) return MI355X_E_INVAL;
    if (row_stride < mi355x_row_size(type, ne0) && type != MI355X_TYPE_F32) return MI355X_E_INVAL;
    if (n_ids == 0) return MI355X_OK;
    if (!device_ok()) return MI355X_E_NODEVICE;
    const dim3 grid((unsigned)((ne0 / 8 + 255) / 256), (unsigned)n_ids);
    return timed_launch("kq::kq_get_rows", (double)n_ids * (ne0 * 4.0 + (double)mi355x_row_size(type, ne0)),
                        kq_get_rows, grid, dim3(256), 0, (hipStream_t)stream, type, (const uint8_t *)table, ne0,
                        (int64_t)row_stride, n_rows, ids, dst);
}

int mi355x_rms_norm(const float *x, const float *w, float *y, int64_t n, int64_t nrows, float eps, void *stream) {
    if (!x || !y || n <= 0 || nrows < 0 || !(eps >= 0.0f)) return MI355X_E_INVAL;
    if (n % QK || ((uintptr_t)x & 15u)) return MI355X_E_UNSUPPORTED;
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_rms_norm(x, w, y, n, nrows, eps, (hipStream_t)stream);
}

int mi355x_add(const float *a, const float *b, float *y, int64_t n, void *stream) {
    if (!a || !b || !y || n < 0) return MI355X_E_INVAL;
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_binary(0, a, b, y, n, (hipStream_t)stream);
}

int mi355x_mul(const float *a, const float *b, float *y, int64_t n, void *stream) {
    if (!a || !b || !y || n < 0) return MI355X_E_INVAL;
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_binary(1, a, b, y, n, (hipStream_t)stream);
}

int mi355x_swiglu(const float *gate, const float *up, float *y, int64_t n, void *stream) {
    if (!gate || !up || !y || n < 0) return MI355X_E_INVAL;
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_swiglu(gate, up, y, n, (hipStream_t)stream);
}

size_t mi355x_rope_table_size(int n_pos, int n_dims) {
    if (n_pos <= 0 || n_dims <= 0 || n_dims % 2) return 0;
    return (size_t)n_pos * (size_t)(n_dims / 2) * 2 * sizeof(float);
}

// ggml_rope_cache_init / rope_yarn (ext_factor 0, attn_factor 1, no freq_factors) for
// every position, built on the host with the C library's powf/cosf/sinf (the
// functions the CPU path calls) and copied to the device table.
int mi355x_rope_table(float *table, int n_pos, int n_dims, float freq_base, float freq_scale, void *stream) {
    const size_t bytes = mi355x_rope_table_size(n_pos, n_dims);
    if (!table || !bytes || !(freq_base > 0.0f)) return MI355X_E_INVAL;
    if (!device_ok()) return MI355X_E_NODEVICE;
    std::vector<float> host(bytes / sizeof(float));
    const float theta_scale = powf(freq_base, -2.0f / (float)n_dims);
    for (int p = 0; p < n_pos; ++p) {
        float theta = (float)p;
        for (int i = 0; i < n_dims / 2; ++i) {
            const float th = freq_scale * theta;
            host[((size_t)p * (n_dims / 2) + i) * 2 + 0] = cosf(th) * 1.0f;
            host[((size_t)p * (n_dims / 2) + i) * 2 + 1] = sinf(th) * 1.0f;
            theta *= theta_scale;
        }
    }
    hipError_t e = hipMemcpyAsync(table, host.data(), bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? MI355X_OK : (int)e;
}

int mi355x_rope(const float *x, float *y, int head_dim, int n_dims, int n_heads, const int32_t *pos,
                const float *table, int n_pos, void *stream) {
    if (!x || !y || !pos || !table || head_dim <= 0 || head_dim % 2 || n_dims % 2 || n_dims > head_dim ||
        n_heads < 0 || n_pos <= 0)
        return MI355X_E_INVAL;
    if (n_heads == 0) return MI355X_OK;
    if (!device_ok()) return MI355X_E_NODEVICE;
    const int64_t pairs = (int64_t)n_heads * (head_dim / 2);
    return timed_launch("kq::kq_rope", pairs * 16.0, kq_rope, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0,
                        (hipStream_t)stream, x, y, head_dim, n_dims, n_heads, pos, table, n_pos);
}

int mi355x_attn_path(const mi355x_attn_desc *d) {
    AttnArgs a = {};
    const int rc = attn_args_from(d, a);
    return rc != MI355X_OK ? rc : attn_path(a);
}

int mi355x_attn_decode(const mi355x_attn_desc *d, void *stream) {
    if (!d) return MI355X_E_INVAL;
    AttnArgs a;
    const int rc = attn_args_from(d, a);
    if (rc) return rc;
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_attn(a, (hipStream_t)stream);
}

int mi355x_attn_prompt(const mi355x_attn_desc *d, int n_tokens, void *stream) {
    if (!d || n_tokens < 0) return MI355X_E_INVAL;
    if (d->rope_row) return MI355X_E_INVAL;  // per-token positions: the whole rope table
    AttnArgs a;
    const int rc = attn_args_from(d, a);
    if (rc) return rc;
    if (attn_prompt_lds(a.head_dim, a.n_ctx) > 160 * 1024) return MI355X_E_UNSUPPORTED;
    if (n_tokens == 0) return MI355X_OK;
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_attn_prompt(a, n_tokens, (hipStream_t)stream);
}

int mi355x_attn_prompt_impl(int impl) {
    if (impl != MI355X_ATTN_GROUP && impl != MI355X_ATTN_HEAD) return MI355X_E_INVAL;
    return g_prompt_impl.exchange(impl);
}

int mi355x_attn_impl(int impl) {
    if (impl != MI355X_ATTN_GROUP && impl != MI355X_ATTN_HEAD && impl != MI355X_ATTN_SPLIT) return MI355X_E_INVAL;
    const int prev = attn_impl();
    g_attn_impl.store(impl);
    return prev;
}

}  // extern "C"

namespace kq {

int attn_args_from(const mi355x_attn_desc *d, AttnArgs &a) {
    if (!d) return MI355X_E_INVAL;
    a.q = d->q;
    a.k = d->k;
    a.v = d->v;
    a.pos = d->pos;
    a.rope_table = d->rope_table;
    a.k_cache = d->k_cache;
    a.v_cache = d->v_cache;
    a.out = d->out;
    a.n_ctx = d->n_ctx;
    a.n_head = d->n_head;
    a.n_head_kv = d->n_head_kv;
    a.head_dim = d->head_dim;
    a.scale = d->scale;
    a.rope_row = d->rope_row ? 1 : 0;
    a.q8_out = nullptr;
    a.no_store = 0;
    a.v_lds = 0;  // launch_attn decides
    a.diag = (int)knob(KNOB_ATTN_DIAG);  // KQ_ATTN_DIAG builds only
    return check_attn(a);
}

}  // namespace kq
