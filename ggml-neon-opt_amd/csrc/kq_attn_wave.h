// kq_attn_wave.h — the decode attention block of one query head on ONE wave (64 lanes):
// the kq_attn_wave kernel (one 64-thread workgroup per query head, no workgroup barrier).
//
// The arithmetic is kq_attn_decode's (kq_ops.hip), operation for operation, only mapped
// onto 64 lanes instead of 256 threads: rope of q / k at the position (rope_pair),
// f16 rounding, KQ per cell with ggml_vec_dot_f16's NEON FP16 structure
// (vec_dot_f16_rows), * scale, the causal mask, the order-free max, ggml_v_expf per
// cell, the vaddvq group sums (e0 + e1) + (e2 + e3) over 4 consecutive cells (a DPP quad),
// ggml's in-order double sum (softmax_group_sum), p = f16(e * (float)(1 / sum)), and KQV
// as 4 f16 accumulators of 8 lanes per output (cells 32 it + 8 j + l) with the f16 reduce
// tree (f16x8_reduce_quad). Each of these is a per-cell or per-output computation in a
// fixed order, so the lanes that run it do not change its bits.
// Every cell of the head sits in the wave's registers: n_kv <= ATTW_MAX_CTX (4 per lane).
#pragma once

#include "kq_device.h"
#include "kq_ops_device.h"

namespace kq {

constexpr int ATTW_MAX_CTX = 256;
// LDS of one wave: q16, k16, v16 (HD f16 each) | p16 (256 f16) | 64 group sums (double)
__host__ __device__ constexpr int attw_lds(int hd) { return 6 * hd + 2 * ATTW_MAX_CTX + 8 * (ATTW_MAX_CTX / 4); }

// Head h of the token at `pos` (bad: no cache cell, NaN output, no stores). store: this
// wave writes the head's kv-group cell to the caches (one writer per group and launch).
// scr: the wave's LDS scratch (attw_lds(HD) bytes, 16-B aligned); xatt: the attention
// output, [n_head * HD] f32. Every lane of the wave must be active.
template <int HD>
__device__ __forceinline__ void attn_head_wave(const AttnArgs &a, int h, int pos, bool bad, bool store, uint8_t *scr,
                                               float *xatt, int lane) {
    static_assert(HD == 64 || HD == 128, "head_dim");
    constexpr int KV4 = HD / 8;      // 16-B pieces of one K-cache row
    constexpr int NP = HD / 2 / 64 > 0 ? HD / 2 / 64 : 1;  // rope pairs per lane (lanes < HD/2 for HD 64)
    constexpr int NV = HD / 64;      // v values per lane
    constexpr int ITEMS = HD / 16;   // KQV (d, j) items per lane: HD * 4 / 64
    const int gsz = a.n_head / a.n_head_kv;
    const int g = h / gsz;
    const int kvw = a.n_head_kv * HD;
    uint16_t *q16 = (uint16_t *)scr;
    uint16_t *k16 = q16 + HD;
    uint16_t *v16 = k16 + HD;
    uint16_t *p16 = (uint16_t *)(scr + 6 * HD);
    double *gsum = (double *)(scr + 6 * HD + 2 * ATTW_MAX_CTX);
    int n_kv = (pos + 1 + 31) / 32 * 32;
    n_kv = n_kv < a.n_ctx ? n_kv : a.n_ctx;

    // ---- loads: this token's q (head h) / k / v (group g), the rope row, the first cells' K rows
    float x0[NP], x1[NP], y0[NP], y1[NP], rc[NP], rs[NP];
    const float *tc = a.rope_table + (a.rope_row ? 0 : (int64_t)pos * (HD / 2) * 2);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int pi = lane + 64 * p;
        x0[p] = x1[p] = y0[p] = y1[p] = rc[p] = rs[p] = 0.f;
        if (pi < HD / 2) {
            rc[p] = tc[2 * pi];
            rs[p] = tc[2 * pi + 1];
            const float *qp = a.q + (int64_t)h * HD + 2 * pi;
            const float *kp = a.k + (int64_t)g * HD + 2 * pi;
            x0[p] = qp[0];
            x1[p] = qp[1];
            y0[p] = kp[0];
            y1[p] = kp[1];
        }
    }
    float vv[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) vv[k] = a.v[(int64_t)g * HD + lane + 64 * k];
    // the first VPF 8-cell groups of each KQV item's V row, issued with the loads above (the
    // KQV loop then runs without a memory round trip for positions < 32 * VPF)
    constexpr int VPF = HD == 64 ? 2 : 1;
    uint4 vpre[ITEMS][VPF];
#pragma unroll
    for (int ii = 0; ii < ITEMS; ++ii) {
        const int item = lane + 64 * ii, d = item >> 2, j = item & 3;
        const uint16_t *vr = a.v_cache + (int64_t)(g * HD + d) * a.n_ctx + 8 * j;
#pragma unroll
        for (int it = 0; it < VPF; ++it) {
            vpre[ii][it] = make_uint4(0u, 0u, 0u, 0u);
            if (32 * it < a.n_ctx) vpre[ii][it] = *(const uint4 *)(vr + 32 * it);
        }
    }
    // head_dim 64: the K row of cell `lane` (the first 64 cells) is issued with the loads above
    // (a cell at or after the position is never used: the new cell comes from LDS); at 128 the
    // row's 64 registers would spill inside the GEMV's budget, so it is read where it is used
    constexpr bool KPRE = HD == 64;
    uint4 kpre[KPRE ? KV4 : 1] = {};
    if (KPRE && lane < a.n_ctx) {
        const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)lane * kvw + (int64_t)g * HD);
#pragma unroll
        for (int i = 0; i < KV4; ++i) kpre[i] = kr[i];
    }

    // ---- rope -> f16, the new cell (written to the caches by the group's writer)
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int pi = lane + 64 * p;
        if (pi < HD / 2) {
            const float2 rq = rope_pair(x0[p], x1[p], rc[p], rs[p]);
            q16[2 * pi] = h2u(f2h_rne(rq.x));
            q16[2 * pi + 1] = h2u(f2h_rne(rq.y));
            const float2 rk = rope_pair(y0[p], y1[p], rc[p], rs[p]);
            const uint16_t k0 = h2u(f2h_rne(rk.x)), k1 = h2u(f2h_rne(rk.y));
            k16[2 * pi] = k0;
            k16[2 * pi + 1] = k1;
            if (store)
                *(uint32_t *)(a.k_cache + (int64_t)pos * kvw + (int64_t)g * HD + 2 * pi) = k0 | ((uint32_t)k1 << 16);
        }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int d = lane + 64 * k;
        const uint16_t hv = h2u(f2h_rne(vv[k]));
        v16[d] = hv;
        if (store) a.v_cache[(int64_t)(g * HD + d) * a.n_ctx + pos] = hv;
    }
    wave_lds_fence();

    // ---- KQ + scale + causal mask: cell c = lane + 64 i
    float sc[ATTW_MAX_CTX / 64];
#pragma unroll
    for (int i = 0; i < ATTW_MAX_CTX / 64; ++i) {
        sc[i] = -INFINITY;
        const int c = lane + 64 * i;
        if (64 * i < n_kv && c < n_kv && c <= pos) {
            if (KPRE) {
                uint4 kv[KV4];
                if (c == pos) {
#pragma unroll
                    for (int q = 0; q < KV4; ++q) kv[q] = ((const uint4 *)k16)[q];
                } else if (i == 0) {
#pragma unroll
                    for (int q = 0; q < KV4; ++q) kv[q] = kpre[KPRE ? q : 0];
                } else {
                    const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)c * kvw + (int64_t)g * HD);
#pragma unroll
                    for (int q = 0; q < KV4; ++q) kv[q] = kr[q];
                }
                sc[i] = vec_dot_f16_rows<HD>(kv, (const uint4 *)q16) * a.scale;
            } else {  // the row read inside the dot, piece by piece (same operations)
                const uint4 *kr = c == pos ? (const uint4 *)k16
                                           : (const uint4 *)(a.k_cache + (int64_t)c * kvw + (int64_t)g * HD);
                sc[i] = vec_dot_f16_rows<HD>(kr, (const uint4 *)q16) * a.scale;
            }
        }
    }
    float m = sc[0];
#pragma unroll
    for (int i = 1; i < ATTW_MAX_CTX / 64; ++i) m = fmaxf(m, sc[i]);
    const float mx = wave_fmax(m);  // order-free

    // ---- soft_max: exp, the vaddvq group sums, ggml's in-order double sum, p -> f16
    float e[ATTW_MAX_CTX / 64];
#pragma unroll
    for (int i = 0; i < ATTW_MAX_CTX / 64; ++i) {
        e[i] = 0.f;
        if (64 * i < n_kv) {  // wave-uniform: every lane takes part in the DPP sums
            const int c = lane + 64 * i;
            e[i] = c < n_kv && sc[i] != -INFINITY ? v_expf(sc[i] - mx) : 0.0f;
            const float s01 = e[i] + dpp_mov_f32<0xB1>(e[i]);   // lane 4g: e0 + e1, lane 4g+2: e2 + e3
            const float g4 = s01 + dpp_mov_f32<0x4E>(s01);      // lane 4g: (e0 + e1) + (e2 + e3)
            if ((lane & 3) == 0 && c < n_kv) gsum[c >> 2] = (double)g4;
        }
    }
    wave_lds_fence();
    const double sum = softmax_group_sum(gsum, n_kv / 4, lane);
    const float inv = (float)(1.0 / sum);
#pragma unroll
    for (int i = 0; i < ATTW_MAX_CTX / 64; ++i) {
        const int c = lane + 64 * i;
        if (c < n_kv) p16[c] = h2u(f2h_rne(e[i] * inv));
    }
    wave_lds_fence();

    // ---- KQV: lane (d, j) -> accumulator j of output d over cells 32 it + 8 j + l, VPF
    // iterations per round (every item's V groups of the round loaded before they are used)
    const int n_it = (pos + 32) / 32;  // iterations holding a cell <= pos; later ones add exact zeros
    uint32_t acc[ITEMS][4] = {};
    for (int it0 = 0; it0 < n_it; it0 += VPF) {
        uint4 vq[ITEMS][VPF];
#pragma unroll
        for (int ii = 0; ii < ITEMS; ++ii) {
            const int item = lane + 64 * ii, d = item >> 2, j = item & 3;
            const uint16_t *vr = a.v_cache + (int64_t)(g * HD + d) * a.n_ctx + 8 * j;
#pragma unroll
            for (int k = 0; k < VPF; ++k) {
                if (it0 == 0) vq[ii][k] = vpre[ii][k];
                else vq[ii][k] = it0 + k < n_it ? *(const uint4 *)(vr + 32 * (it0 + k)) : make_uint4(0u, 0u, 0u, 0u);
            }
        }
#pragma unroll
        for (int ii = 0; ii < ITEMS; ++ii) {
            const int item = lane + 64 * ii, d = item >> 2, j = item & 3;
#pragma unroll
            for (int k = 0; k < VPF; ++k) {
                if (it0 + k < n_it) {
                    const int c0 = 32 * (it0 + k) + 8 * j;
                    const uint4 pp = *(const uint4 *)(p16 + c0);
                    uint32_t vw[4] = {vq[ii][k].x, vq[ii][k].y, vq[ii][k].z, vq[ii][k].w};
                    const uint32_t pw[4] = {pp.x, pp.y, pp.z, pp.w};
                    if (pos >= c0 && pos < c0 + 8) {  // the new cell: this wave's LDS copy
                        const int l = pos - c0;
                        vw[l >> 1] = (vw[l >> 1] & (0xffff0000u >> (16 * (l & 1)))) | ((uint32_t)v16[d] << (16 * (l & 1)));
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[ii][q] = pk_fma_w(vw[q], pw[q], acc[ii][q]);
                }
            }
        }
    }
#pragma unroll
    for (int ii = 0; ii < ITEMS; ++ii) {
        const int item = lane + 64 * ii, d = item >> 2, j = item & 3;
        const float o = f16x8_reduce_quad(acc[ii]);  // accumulators j = 0..3 of output d: one quad of lanes
        if (j == 0) xatt[h * HD + d] = bad ? __builtin_nanf("") : o;
    }
}

}  // namespace kq
