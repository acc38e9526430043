// kq_rows_device.h — device helpers of the row-stream decode kernel (kq_rows.hip):
// fused Q8_K quantization into the aligned Q8L layout, the per-type
// quad partials and the counted-wait helpers.
#pragma once

#include "kq_device.h"
#include "kq_ops_device.h"

namespace kq {

// ---------------------------------------------------------------- fused Q8_K quantization
// Reductions over an aligned row of 16 lanes (DPP only): xor 1, xor 2, 8-mirror, 16-mirror.
template <typename Op>
__device__ __forceinline__ int row16_reduce(int v, Op op) {
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false));
    return v;
}

__device__ __forceinline__ uint32_t qbyte(float iscale, float x) {
    int q = nearest_int_fused(iscale, x);
    q = q < 127 ? q : 127;  // MIN(127, v); the int8 store truncates
    return (uint32_t)q & 0xffu;
}

// One superblock per 16-lane row; lane l of the row owns x[16l .. 16l+15] (v[0..3]).
// quantize_row_q8_K_ref semantics exactly as quant_values_wave (kq_device.h):
// amax ignores NaN, max = first x with |x| == amax, iscale = -127/max (correctly
// rounded), qs = MIN(127, nearest_int(fmaf(iscale, x, 1.5*2^23))) as int8,
// bsums over the stored int8, d = 1/iscale; all-zero block -> zeros.
// Writes the Q8L block (d @0, qs @16, bsums @272) at `qb`. AM (the prefill GEMMs' blocks,
// "Q8L/mmq"): bytes 272..303 hold the f16 operand of kq_mmq's mins MFMA instead of the
// bsums: bs_j = bsums[2j] + bsums[2j+1] = 64*hi + lo (lo in 0..63) as [lo_0..7 | hi_0..7],
// integers exact in f16.
template <bool AM = false>
__device__ __forceinline__ void quant16_store(const u32x4 v[4], int l, uint8_t *qb) {
    float x[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        x[4 * k + 0] = __uint_as_float(v[k].x);
        x[4 * k + 1] = __uint_as_float(v[k].y);
        x[4 * k + 2] = __uint_as_float(v[k].z);
        x[4 * k + 3] = __uint_as_float(v[k].w);
    }
    // amax and the sign of the first x with |x| == amax: the largest positive and
    // the largest negated value (both >= 0, NaN dropped by fmaxf); only a tie
    // (+amax and -amax both present) needs the first-index scan.
    float mp = 0.f, mn = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        mp = fmaxf(mp, x[k]);
        mn = fmaxf(mn, -x[k]);
    }
    const int mpb = row16_reduce(__float_as_int(mp), [](int a, int c) { return a > c ? a : c; });
    const int mnb = row16_reduce(__float_as_int(mn), [](int a, int c) { return a > c ? a : c; });
    const float m = __int_as_float(mpb > mnb ? mpb : mnb);
    bool neg = mnb > mpb;
    if (mpb == mnb && mpb != 0) {  // tie: serial `if (ax > amax)` keeps the first index
        uint32_t key = 0xffffffffu;
#pragma unroll
        for (int k = 15; k >= 0; --k)
            if (fabsf(x[k]) == m) key = 2u * (uint32_t)(16 * l + k) + (x[k] < 0.f ? 1u : 0u);
        key = (uint32_t)row16_reduce((int)key, [](int a, int c) { return (uint32_t)a < (uint32_t)c ? a : c; });
        neg = (key & 1u) != 0;
    }
    const float maxv = neg ? -m : m;
    const float iscale = -127.f / maxv;
    u32x4 q;
    q.x = qbyte(iscale, x[0]) | (qbyte(iscale, x[1]) << 8) | (qbyte(iscale, x[2]) << 16) | (qbyte(iscale, x[3]) << 24);
    q.y = qbyte(iscale, x[4]) | (qbyte(iscale, x[5]) << 8) | (qbyte(iscale, x[6]) << 16) | (qbyte(iscale, x[7]) << 24);
    q.z = qbyte(iscale, x[8]) | (qbyte(iscale, x[9]) << 8) | (qbyte(iscale, x[10]) << 16) |
          (qbyte(iscale, x[11]) << 24);
    q.w = qbyte(iscale, x[12]) | (qbyte(iscale, x[13]) << 8) | (qbyte(iscale, x[14]) << 16) |
          (qbyte(iscale, x[15]) << 24);
    int bsum = sdot4(q.x, 0x01010101u, 0);
    bsum = sdot4(q.y, 0x01010101u, bsum);
    bsum = sdot4(q.z, 0x01010101u, bsum);
    bsum = sdot4(q.w, 0x01010101u, bsum);
    float d = 1.f / iscale;
    if (m == 0.f) {  // `if (!amax)`: d = 0, qs = 0 (bsums then 0)
        q = u32x4{0u, 0u, 0u, 0u};
        bsum = 0;
        d = 0.f;
    }
    *(u32x4 *)(qb + 16 + 16 * l) = q;
    if (AM) {
        const int bs = bsum + __builtin_amdgcn_update_dpp(bsum, bsum, 0xB1, 0xF, 0xF, false);  // lanes 2j, 2j+1
        if (!(l & 1)) {
            *(_Float16 *)(qb + 272 + l) = (_Float16)(bs & 63);
            *(_Float16 *)(qb + 288 + l) = (_Float16)(bs >> 6);
        }
    } else {
        *(int16_t *)(qb + 272 + 2 * l) = (int16_t)bsum;
    }
    if (l == 0) *(float *)qb = d;
}

__device__ __forceinline__ uint32_t gload4_asm(const float *p) {
    uint32_t r;
    asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}

// Fused-prologue transforms of 4 activation values held as f32 bits (kq_ops_device.h):
// ggml_vec_swiglu_f32 (silu(g) * u) and rms_norm + MUL ((x * scale) * w).
__device__ __forceinline__ u32x4 swiglu4(u32x4 g, u32x4 u) {
    u32x4 r;
    r.x = __float_as_uint(v_silu(__uint_as_float(g.x)) * __uint_as_float(u.x));
    r.y = __float_as_uint(v_silu(__uint_as_float(g.y)) * __uint_as_float(u.y));
    r.z = __float_as_uint(v_silu(__uint_as_float(g.z)) * __uint_as_float(u.z));
    r.w = __float_as_uint(v_silu(__uint_as_float(g.w)) * __uint_as_float(u.w));
    return r;
}

__device__ __forceinline__ u32x4 normmul4(u32x4 x, u32x4 w, float scale) {
    u32x4 r;
    r.x = __float_as_uint((__uint_as_float(x.x) * scale) * __uint_as_float(w.x));
    r.y = __float_as_uint((__uint_as_float(x.y) * scale) * __uint_as_float(w.y));
    r.z = __float_as_uint((__uint_as_float(x.z) * scale) * __uint_as_float(w.z));
    r.w = __float_as_uint((__uint_as_float(x.w) * scale) * __uint_as_float(w.w));
    return r;
}

__device__ __forceinline__ u32x4 gload16_asm(const float *p) {
    u32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}

// ---------------------------------------------------------------- per-type quad partials
// Lane s (0..3) of a quad covers 64 quants of the superblock at `blk` (LDS) against
// the Q8L activation block `ab`. Every sum is an exact int32; the pairings below
// only re-associate integer additions of lane_q4K/q5K/q6K (kq_device.h).
__device__ __forceinline__ int dotacc(u32x4 q, u32x4 a, int acc) {
    acc = sdot4(q.x, a.x, acc);
    acc = sdot4(q.y, a.y, acc);
    acc = sdot4(q.z, a.z, acc);
    return sdot4(q.w, a.w, acc);
}

struct QuadOut {
    int isum, imin;
    uint32_t dh;  // Q4_K/Q5_K: d | dmin << 16 ; Q6_K: d
};

// Q4_K: s <-> sub-blocks 2s (low nibbles) / 2s+1 (high), qs[32s, 32s+32).
__device__ __forceinline__ QuadOut quad_q4K(const uint8_t *blk, const uint8_t *ab, int s) {
    const u32x4 hdr = *(const u32x4 *)blk;
    const u32x4 q0 = *(const u32x4 *)(blk + 16 + 32 * s);
    const u32x4 q1 = *(const u32x4 *)(blk + 32 + 32 * s);
    const uint8_t *aq = ab + 16 + 64 * s;
    const u32x4 a0 = *(const u32x4 *)(aq), a1 = *(const u32x4 *)(aq + 16);
    const u32x4 a2 = *(const u32x4 *)(aq + 32), a3 = *(const u32x4 *)(aq + 48);
    const ScMn s0 = scales_k4(hdr, 2 * s), s1 = scales_k4(hdr, 2 * s + 1);
    const int dlo = dotacc(q1 & 0x0f0f0f0fu, a1, dotacc(q0 & 0x0f0f0f0fu, a0, 0));
    const int dhi = dotacc((q1 >> 4) & 0x0f0f0f0fu, a3, dotacc((q0 >> 4) & 0x0f0f0f0fu, a2, 0));
    const uint2 bs = *(const uint2 *)(ab + 272 + 8 * s);
    QuadOut r;
    r.isum = __mul24(dlo, s0.sc_lo) + __mul24(dhi, s0.sc_hi);  // |dot| < 2^17: full-rate i24
    r.imin = ((int)(int16_t)(bs.x & 0xffffu) + (int)(int16_t)(bs.x >> 16)) * s0.mn +
             ((int)(int16_t)(bs.y & 0xffffu) + (int)(int16_t)(bs.y >> 16)) * s1.mn;
    r.dh = hdr.x;
    return r;
}

// Q5_K: as Q4_K plus the 5th bit from qh (bit 2s for low nibbles, 2s+1 for high).
__device__ __forceinline__ QuadOut quad_q5K(const uint8_t *blk, const uint8_t *ab, int s) {
    const u32x4 hdr = *(const u32x4 *)blk;
    const u32x4 h0 = *(const u32x4 *)(blk + 16), h1 = *(const u32x4 *)(blk + 32);
    const u32x4 q0 = *(const u32x4 *)(blk + 48 + 32 * s);
    const u32x4 q1 = *(const u32x4 *)(blk + 64 + 32 * s);
    const uint8_t *aq = ab + 16 + 64 * s;
    const u32x4 a0 = *(const u32x4 *)(aq), a1 = *(const u32x4 *)(aq + 16);
    const u32x4 a2 = *(const u32x4 *)(aq + 32), a3 = *(const u32x4 *)(aq + 48);
    const ScMn s0 = scales_k4(hdr, 2 * s), s1 = scales_k4(hdr, 2 * s + 1);
    const uint32_t sl = (uint32_t)(2 * s), shh = (uint32_t)(2 * s + 1);
    const u32x4 lo0 = (q0 & 0x0f0f0f0fu) | (((h0 >> sl) & 0x01010101u) << 4);
    const u32x4 hi0 = ((q0 >> 4) & 0x0f0f0f0fu) | (((h0 >> shh) & 0x01010101u) << 4);
    const u32x4 lo1 = (q1 & 0x0f0f0f0fu) | (((h1 >> sl) & 0x01010101u) << 4);
    const u32x4 hi1 = ((q1 >> 4) & 0x0f0f0f0fu) | (((h1 >> shh) & 0x01010101u) << 4);
    const int dlo = dotacc(lo1, a1, dotacc(lo0, a0, 0));
    const int dhi = dotacc(hi1, a3, dotacc(hi0, a2, 0));
    const uint2 bs = *(const uint2 *)(ab + 272 + 8 * s);
    QuadOut r;
    r.isum = __mul24(dlo, s0.sc_lo) + __mul24(dhi, s0.sc_hi);  // |dot| < 2^17: full-rate i24
    r.imin = ((int)(int16_t)(bs.x & 0xffffu) + (int)(int16_t)(bs.x >> 16)) * s0.mn +
             ((int)(int16_t)(bs.y & 0xffffu) + (int)(int16_t)(bs.y >> 16)) * s1.mn;
    r.dh = hdr.x;
    return r;
}

// Q6_K (210 B, any byte alignment in LDS: 4-aligned dword reads + alignbyte):
// s <-> ql[32s, 32s+32), qh[128 + 32(s>>1), +32), qh bit pair 2(s&1) / +4.
__device__ __forceinline__ QuadOut quad_q6K(const uint8_t *blk, const uint8_t *ab, int s) {
    const uint32_t s4 = (uint32_t)((uintptr_t)blk & 3u);
    const uint8_t *b = blk - s4;
    const int n = s >> 1, part2 = s & 1;
    const u32x4 L0 = realign(*(const u32x4a *)(b + 32 * s), *(const uint32_t *)(b + 32 * s + 16), s4);
    const u32x4 L1 = realign(*(const u32x4a *)(b + 32 * s + 16), *(const uint32_t *)(b + 32 * s + 32), s4);
    const u32x4 H0 = realign(*(const u32x4a *)(b + 128 + 32 * n), *(const uint32_t *)(b + 144 + 32 * n), s4);
    const u32x4 H1 = realign(*(const u32x4a *)(b + 144 + 32 * n), *(const uint32_t *)(b + 160 + 32 * n), s4);
    const uint32_t w208 = *(const uint32_t *)(b + 208);
    const u32x4 SC = realign(*(const u32x4a *)(b + 192), w208, s4);
    const uint32_t shl = (uint32_t)part2 * 2u;
    const u32x4 ql0 = (L0 & 0x0f0f0f0fu) | (((H0 >> shl) & 0x03030303u) << 4);
    const u32x4 qh0 = ((L0 >> 4) & 0x0f0f0f0fu) | (((H0 >> (shl + 4u)) & 0x03030303u) << 4);
    const u32x4 ql1 = (L1 & 0x0f0f0f0fu) | (((H1 >> shl) & 0x03030303u) << 4);
    const u32x4 qh1 = ((L1 >> 4) & 0x0f0f0f0fu) | (((H1 >> (shl + 4u)) & 0x03030303u) << 4);
    const int elo = 128 * n + 32 * part2;  // elements of ql0's low nibbles; ql1: +16
    const uint8_t *aq = ab + 16 + elo;
    const int sb = elo >> 4;
    const int d00 = dotacc(ql0, *(const u32x4 *)(aq), 0);
    const int d01 = dotacc(qh0, *(const u32x4 *)(aq + 64), 0);
    const int d10 = dotacc(ql1, *(const u32x4 *)(aq + 16), 0);
    const int d11 = dotacc(qh1, *(const u32x4 *)(aq + 80), 0);
    QuadOut r;
    r.isum = __mul24(d00, sbyte(SC, sb)) + __mul24(d01, sbyte(SC, sb + 4)) + __mul24(d10, sbyte(SC, sb + 1)) +
             __mul24(d11, sbyte(SC, sb + 5));  // |dot| < 2^17: full-rate i24
    const uint2 bs = *(const uint2 *)(ab + 272 + 8 * s);
    r.imin = (int)(int16_t)(bs.x & 0xffffu) * sbyte(SC, 4 * s) + (int)(int16_t)(bs.x >> 16) * sbyte(SC, 4 * s + 1) +
             (int)(int16_t)(bs.y & 0xffffu) * sbyte(SC, 4 * s + 2) + (int)(int16_t)(bs.y >> 16) * sbyte(SC, 4 * s + 3);
    r.dh = (w208 >> (8u * s4)) & 0xffffu;
    return r;
}

__device__ __forceinline__ int quad_sum(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    return v;
}

// ---------------------------------------------------------------- the row stream of one wave
struct WaveWork {
    int m, r0, nrows;
};

// s_waitcnt vmcnt(N * k) for runtime k in [0, 3] (tail of the stream).
template <int N>
__device__ __forceinline__ void vm_wait_k(int k) {
    if (k >= 3) vm_wait<3 * N>();
    else if (k == 2) vm_wait<2 * N>();
    else if (k == 1) vm_wait<N>();
    else vm_wait<0>();
}
// s_waitcnt vmcnt(N * k + P): the same with P younger L2-prefetch loads still counted.
template <int N, int P>
__device__ __forceinline__ void vm_wait_kp(int k) {
    if (k >= 3) vm_wait<3 * N + P>();
    else if (k == 2) vm_wait<2 * N + P>();
    else if (k == 1) vm_wait<N + P>();
    else vm_wait<P>();
}

// s_waitcnt vmcnt(n) for a run-time, wave-uniform n (a scalar branch per case); above
// the table's range it waits for the table's largest count, a stronger wait.
__device__ __forceinline__ void vm_wait_dyn(int n) {
#define KQ_VMW_CASE(N) \
    case N: vm_wait<N>(); break;
    switch (n < 0 ? 0 : n) {
        KQ_VMW_CASE(0) KQ_VMW_CASE(1) KQ_VMW_CASE(2) KQ_VMW_CASE(3) KQ_VMW_CASE(4) KQ_VMW_CASE(5) KQ_VMW_CASE(6)
        KQ_VMW_CASE(7) KQ_VMW_CASE(8) KQ_VMW_CASE(9) KQ_VMW_CASE(10) KQ_VMW_CASE(11) KQ_VMW_CASE(12)
        KQ_VMW_CASE(13) KQ_VMW_CASE(14) KQ_VMW_CASE(15) KQ_VMW_CASE(16) KQ_VMW_CASE(17) KQ_VMW_CASE(18)
        KQ_VMW_CASE(19) KQ_VMW_CASE(20) KQ_VMW_CASE(21) KQ_VMW_CASE(22) KQ_VMW_CASE(23) KQ_VMW_CASE(24)
        KQ_VMW_CASE(25) KQ_VMW_CASE(26) KQ_VMW_CASE(27) KQ_VMW_CASE(28) KQ_VMW_CASE(29) KQ_VMW_CASE(30)
        KQ_VMW_CASE(31) KQ_VMW_CASE(32) KQ_VMW_CASE(33) KQ_VMW_CASE(34) KQ_VMW_CASE(35) KQ_VMW_CASE(36)
        KQ_VMW_CASE(37) KQ_VMW_CASE(38) KQ_VMW_CASE(39) KQ_VMW_CASE(40)
        default: vm_wait<40>(); break;
    }
#undef KQ_VMW_CASE
}

// One L2 prefetch touch: a dword load per lane into a register reserved for it
// (tied in/out, so every touch reuses it and nothing else is allocated there while
// the loads are in flight); the caller consumes `sink` after its covering wait.
__device__ __forceinline__ void l2_touch(const void *p, uint32_t &sink) {
    asm volatile("global_load_dword %0, %1, off" : "+v"(sink) : "v"(p) : "memory");
}

}  // namespace kq
