// kq_attn_device.h — decode attention of ONE kv group (its gsz query heads), the work
// unit of kq_attn_group (kq_ops.hip). Same arithmetic as kq_attn_decode (one workgroup
// per query head), op for op, so every output bit is the reference's:
//   rope(q_h), rope(k_g) at pos -> f16; v_g -> f16; the new cell written to both caches
//   (set_rows, V transposed); KQ = ggml_vec_dot_f16 (NEON FP16 structure) * scale,
//   causal mask; soft_max: max, ggml_v_expf, vaddvq group sums of 4, the sequential
//   double sum over groups; KQV = ggml_vec_dot_f16(v_cache row, p16)
//   (ggml-cpu @ a3cb0474 [U]; artifacts/perf/out.folded:140-144, :176, :209-234).
//
// Layout (MI355X-first): the group's K and V cells [0, n_kv) are fetched ONCE per
// workgroup by LDS-DMA (every wave issues a share), n_kv = pad32(pos + 1) — only the
// live cells, never the whole cache — and stored "transposed by 16 B" so that lane c
// of a KQ pass (cell c) and lane d of KQV (channel d) read consecutive 16-B words
// (conflict-free ds_read_b128):
//   Ks: granule (p, c) = K[c][8p .. 8p+8)  at Ks + (p * n_ctx + c) * 16
//   Vs: granule (s, d) = V[d][8s .. 8s+8)  at Vs + (s * HD + d) * 16
// Latency: cells [0, ATTN_PF) (every position has them) are requested together with
// the position, q/k/v and the rope row; only a position past them costs a second
// round trip for cells [ATTN_PF, n_kv).
// Head h = g*gsz + i runs on wave i (and i + nwaves, ...): KQ over 64-cell passes,
// scores / exps / group sums in the wave's LDS slot, KQV from Vs with p16 broadcast.
// The new cell comes from the group's LDS copy (kn / vn), never from a cache line
// written in this launch.
#pragma once

#include "kq_device.h"
#include "kq_ops_device.h"

namespace kq {

// Byte offsets (16-B aligned) of the group attention's LDS, from `base`.
struct AttnLds {
    int ks, vs, kn, vn, slot, slot_stride, total;
};
__host__ __device__ inline AttnLds attn_group_lds(int hd, int n_ctx, int slots) {
    AttnLds L;
    L.ks = 0;
    L.vs = L.ks + 2 * hd * n_ctx;
    L.kn = L.vs + 2 * hd * n_ctx;
    L.vn = L.kn + 2 * hd;
    L.slot = L.vn + 2 * hd;
    L.slot_stride = 2 * hd + 8 * n_ctx;  // q16 [hd] | w f32 [n_ctx] | p16 [n_ctx] | gsum f64 [n_ctx/4]
    L.total = L.slot + slots * L.slot_stride;
    return L;
}

// ggml_vec_dot_f16 of a K cell held as KV4 16-B granules `stride` apart in LDS with q
// (contiguous): the same accumulators, in the same order, as vec_dot_f16_rows.
template <int N>
__device__ __forceinline__ float vec_dot_f16_lds(const uint4 *x, int stride, const uint4 *y) {
    h16 acc[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int l = 0; l < 8; ++l) acc[j][l] = (h16)0.0f;
#pragma unroll
    for (int it = 0; it < N / 32; ++it)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 xv = x[(4 * it + j) * stride], yv = y[4 * it + j];
            const uint32_t xw[4] = {xv.x, xv.y, xv.z, xv.w}, yw[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
            for (int l = 0; l < 8; ++l)
                acc[j][l] = hfma(u2h((uint16_t)(xw[l >> 1] >> (16 * (l & 1)))),
                                 u2h((uint16_t)(yw[l >> 1] >> (16 * (l & 1)))), acc[j][l]);
        }
    h16 s[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const h16 s0 = acc[0][l] + acc[2][l];
        const h16 s1 = acc[1][l] + acc[3][l];
        s[l] = s0 + s1;
    }
    return f16x8_reduce(s);
}

constexpr int ATTN_PF = 64;  // cells fetched before the position is known

// Loads issued by inline asm, so that the compiler tracks none of them: with a
// compiler-visible load in flight hipcc puts an s_waitcnt vmcnt(0) in front of every
// later DMA of a loop (its address registers look busy), which serialised the slice
// fetch into one round trip per instruction. Every address must be valid for every lane
// (no branch may join a register whose load is in flight); the caller waits with one
// s_waitcnt vmcnt(0) and pins the registers.
__device__ __forceinline__ uint64_t ld8_asm(const void *p) {
    uint64_t v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint32_t ld4_asm(const void *p) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ float2 pair_of(uint64_t v) {
    return make_float2(__uint_as_float((uint32_t)v), __uint_as_float((uint32_t)(v >> 32)));
}

// The K/V cells [c0, c1) of group g into the slices (c0 % 64 == 0, c1 % 32 == 0). One
// LDS-DMA instruction fills 64 consecutive granules: K, 64 cells of one 16-B column p
// (lanes past c1 masked); V, 64 channels of one 8-cell column s.
template <int HD>
__device__ __forceinline__ void attn_fetch(const AttnArgs &a, int g, int c0, int c1, uint8_t *Ks, uint8_t *Vs,
                                           int wave, int nwaves, int lane) {
    constexpr int KV4 = HD / 8;  // 16-B granules of one K cell of the group
    const int kvw = a.n_head_kv * HD;
    const int nck = (c1 - c0 + 63) / 64;  // 64-cell chunks per column
    for (int j = wave; j < KV4 * nck; j += nwaves) {
        const int p = j / nck, c = c0 + 64 * (j - p * nck) + lane;
        if (c < c1) dma16(a.k_cache + (int64_t)c * kvw + g * HD + 8 * p, (LDS void *)(Ks + 16 * (p * a.n_ctx + c - lane)));
    }
    constexpr int DH = HD / 64;  // instructions per 8-cell column
    for (int j = wave; j < DH * (c1 - c0) / 8; j += nwaves) {
        const int s = c0 / 8 + j / DH, d = 64 * (j % DH) + lane;
        dma16(a.v_cache + (int64_t)(g * HD + d) * a.n_ctx + 8 * s, (LDS void *)(Vs + 16 * (s * HD + d - lane)));
    }
}

// The whole group g, by the `nwaves` waves of the calling workgroup (each calls with
// its wave index). `base`: 16-B aligned LDS of attn_group_lds(HD, n_ctx, min(gsz,
// nwaves)).total bytes.
template <int HD>
__device__ void attn_group(const AttnArgs &a, int g, uint8_t *base, int wave, int nwaves, int lane) {
    static_assert(HD == 64 || HD == 128, "head_dim");
    const int gsz = a.n_head / a.n_head_kv;
    const int kvw = a.n_head_kv * HD;
    const int n_ctx = a.n_ctx;
    const int slots = gsz < nwaves ? gsz : nwaves;
    const AttnLds L = attn_group_lds(HD, n_ctx, slots);
    uint8_t *const Ks = base + L.ks;
    uint8_t *const Vs = base + L.vs;
    uint16_t *const kn = (uint16_t *)(base + L.kn);
    uint16_t *const vn = (uint16_t *)(base + L.vn);

    // ---- A. one round trip: the position, cells [0, ATTN_PF), k_g / v_g, the q of the
    //         wave's first head (a valid head for every wave) and the staged rope row
    const int pf = n_ctx < ATTN_PF ? n_ctx : ATTN_PF;
    const int lp = lane & (HD / 2 - 1);
    uint32_t r_pos = ld4_asm(a.pos);
    attn_fetch<HD>(a, g, 0, pf, Ks, Vs, wave, nwaves, lane);
    uint64_t r_cs = ld8_asm(a.rope_table + 2 * lp);  // the row itself when rope_row, else row 0
    uint64_t r_k = ld8_asm(a.k + (int64_t)g * HD + 2 * lp);
    uint32_t r_v0 = ld4_asm(a.v + (int64_t)g * HD + lane);
    uint32_t r_v1 = ld4_asm(a.v + (int64_t)g * HD + (HD == 128 ? 64 : 0) + lane);
    uint64_t r_q = ld8_asm(a.q + (int64_t)(g * gsz + (wave < gsz ? wave : 0)) * HD + 2 * lp);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(r_pos), "+v"(r_cs), "+v"(r_k), "+v"(r_v0), "+v"(r_v1), "+v"(r_q));
    const int pos_in = __builtin_amdgcn_readfirstlane((int)r_pos);
    const bool bad = pos_in < 0 || pos_in >= n_ctx;  // no cache cell for this position
    const int pos = bad ? 0 : pos_in;
    int n_kv = (pos + 1 + 31) / 32 * 32;
    n_kv = n_kv < n_ctx ? n_kv : n_ctx;
    if (n_kv > pf || (!a.rope_row && pos > 0)) {  // a second round trip: later cells, the table's row
        if (n_kv > pf) attn_fetch<HD>(a, g, pf, n_kv, Ks, Vs, wave, nwaves, lane);
        r_cs = ld8_asm(a.rope_table + (a.rope_row ? 0 : (int64_t)pos * HD) + 2 * lp);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(r_cs));
    }
    const float2 cs = pair_of(r_cs), kp = pair_of(r_k);
    const float v0 = __uint_as_float(r_v0), v1 = __uint_as_float(r_v1);
    float2 qp = pair_of(r_q);
    if (wave == 0) {  // the group's new cell: rope(k) and v in f16, written to the caches once
        if (lane < HD / 2) {
            const float2 rk = rope_pair(kp.x, kp.y, cs.x, cs.y);
            const uint16_t k0 = h2u(f2h_rne(rk.x)), k1 = h2u(f2h_rne(rk.y));
            kn[2 * lane] = k0;
            kn[2 * lane + 1] = k1;
            if (!bad) *(uint32_t *)(a.k_cache + (int64_t)pos * kvw + g * HD + 2 * lane) = k0 | ((uint32_t)k1 << 16);
        }
        const uint16_t h0 = h2u(f2h_rne(v0));
        vn[lane] = h0;
        if (!bad) a.v_cache[(int64_t)(g * HD + lane) * n_ctx + pos] = h0;
        if (HD == 128) {
            const uint16_t h1 = h2u(f2h_rne(v1));
            vn[64 + lane] = h1;
            if (!bad) a.v_cache[(int64_t)(g * HD + 64 + lane) * n_ctx + pos] = h1;
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");  // slices landed, kn/vn written

    // ---- B. one head per wave
    for (int i = wave; i < gsz; i += nwaves) {
        const int h = g * gsz + i;
        uint8_t *const slot = base + L.slot + (i % slots) * L.slot_stride;
        uint16_t *const q16 = (uint16_t *)slot;
        float *const w = (float *)(slot + 2 * HD);
        uint16_t *const p16 = (uint16_t *)(w + n_ctx);
        double *const gsum = (double *)(p16 + n_ctx);
        if (i != wave) {  // more heads than waves: this head's q, one more round trip
            uint64_t r = ld8_asm(a.q + (int64_t)h * HD + 2 * lp);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("" : "+v"(r));
            qp = pair_of(r);
        }
        if (lane < HD / 2) {
            const float2 rq = rope_pair(qp.x, qp.y, cs.x, cs.y);
            q16[2 * lane] = h2u(f2h_rne(rq.x));
            q16[2 * lane + 1] = h2u(f2h_rne(rq.y));
        }
        wave_lds_fence();
        // KQ + scale + causal mask, one cell per lane and pass
        float m = -INFINITY;
        for (int c0 = 0; c0 < n_kv; c0 += 64) {
            const int c = c0 + lane;
            float s = -INFINITY;
            if (c < n_kv && c <= pos) {
                s = c == pos ? vec_dot_f16_lds<HD>((const uint4 *)kn, 1, (const uint4 *)q16)
                             : vec_dot_f16_lds<HD>((const uint4 *)Ks + c, n_ctx, (const uint4 *)q16);
                s = s * a.scale;
            }
            if (c < n_kv) w[c] = s;
            m = fmaxf(m, s);
        }
        const float mx = wave_fmax(m);  // order-free
        // exp and the vaddvq group sums (e0 + e1) + (e2 + e3) over lanes 4q .. 4q+3
        for (int c0 = 0; c0 < n_kv; c0 += 64) {
            const int c = c0 + lane;
            const float sv = c < n_kv ? w[c] : -INFINITY;
            const float e = sv == -INFINITY ? 0.0f : v_expf(sv - mx);
            const float s01 = e + dpp_mov_f32<0xB1>(e);
            const float g4 = s01 + dpp_mov_f32<0x4E>(s01);
            if (c < n_kv) {
                w[c] = e;
                if ((lane & 3) == 0) gsum[c >> 2] = (double)g4;
            }
        }
        wave_lds_fence();
        const double sum = softmax_group_sum(gsum, n_kv / 4, lane);  // ggml's in-order sum (a tree where exact)
        const float inv = (float)(1.0 / sum);
        for (int c = lane; c < n_kv; c += 64) p16[c] = h2u(f2h_rne(w[c] * inv));
        wave_lds_fence();
        // KQV: lane d runs the four 8-lane accumulators of output d over its cells
        const int n_it = (pos + 32) / 32;  // iterations holding a cell <= pos
#pragma unroll 1
        for (int d = lane; d < HD; d += 64) {
            h16 acc[4][8];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int l = 0; l < 8; ++l) acc[j][l] = (h16)0.0f;
            for (int it = 0; it < n_it; ++it) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int s = 4 * it + j;
                    const uint4 vv = ((const uint4 *)Vs)[s * HD + d];
                    const uint4 pp = ((const uint4 *)p16)[s];
                    uint32_t vw[4] = {vv.x, vv.y, vv.z, vv.w};
                    const uint32_t pw[4] = {pp.x, pp.y, pp.z, pp.w};
                    if (pos >= 8 * s && pos < 8 * s + 8) {  // the new cell: the group's LDS copy
                        const int l = pos - 8 * s;
                        vw[l >> 1] = (vw[l >> 1] & (0xffff0000u >> (16 * (l & 1)))) | ((uint32_t)vn[d] << (16 * (l & 1)));
                    }
#pragma unroll
                    for (int l = 0; l < 8; ++l)
                        acc[j][l] = hfma(u2h((uint16_t)(vw[l >> 1] >> (16 * (l & 1)))),
                                         u2h((uint16_t)(pw[l >> 1] >> (16 * (l & 1)))), acc[j][l]);
                }
            }
            h16 sv[8];
#pragma unroll
            for (int l = 0; l < 8; ++l) {
                const h16 s0 = acc[0][l] + acc[2][l];
                const h16 s1 = acc[1][l] + acc[3][l];
                sv[l] = s0 + s1;
            }
            const float o = f16x8_reduce(sv);
            a.out[(int64_t)h * HD + d] = bad ? __builtin_nanf("") : o;
        }
    }
}

}  // namespace kq
