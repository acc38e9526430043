// kq_rows.hip — decode GEMV (one activation column) over contiguous row streams.
//
// Same numerics as kq_gemv (kq_kernels.hip): integer partials bit-exact, the
// reference's fp32 update in superblock order per row (README.md:551/:614 for
// Q4_K), so outputs are bit-identical to ggml_vec_dot_q4_K_q8_K (and the Q5_K /
// Q6_K siblings) called row by row from ggml_compute_forward_mul_mat
// (ggml-cpu.c:1389, README.md:137).
//
// Decomposition (HBM-bound, so everything serves the weight stream):
//  * a wave owns `rpw` consecutive rows of one matrix; with GGUF's contiguous
//    rows that is ONE contiguous byte stream, fetched in steps of 16 superblocks
//    (2.3-3.4 KB, 3-4 LDS-DMA instructions of 1 KB, non-temporal) into a
//    per-wave ring, completion by counted s_waitcnt vmcnt (a constant in steady
//    state); no workgroup barrier after the prologue;
//  * lane quad q computes superblock 16t+q of the stream (4 lanes x 64 quants,
//    v_dot4_i32_i8, 2 DPP adds) and its leader stores the exact fp32 operands of
//    the reference's update as a 16-B record, block-major per row batch;
//  * when a batch of bR rows is complete, lane r replays row r's records in
//    superblock order (the serial fp32 chain, 64 rows per instruction);
//  * the activation is quantized to Q8_K once per workgroup into LDS (aligned
//    304-B "Q8L" blocks: d @0, qs @16, bsums @272): 16 lanes per superblock, x
//    loaded by inline-asm global loads issued before the weight DMAs (K <= 8192);
//    above that kq_quantize_q8L writes Q8L blocks to a workspace, copied by DMA.
#include "kq_device.h"

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
// Writes the Q8L block (d @0, qs @16, bsums @272) at `qb`.
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
    *(int16_t *)(qb + 272 + 2 * l) = (int16_t)bsum;
    if (l == 0) *(float *)qb = d;
}

__device__ __forceinline__ u32x4 gload16_asm(const float *p) {
    u32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}

// Q8L quantization of whole rows (K > 8192 path): 16 superblocks per workgroup.
__global__ void __launch_bounds__(WG_THREADS) kq_quantize_q8L(const float *__restrict__ x, int64_t x_stride,
                                                              uint8_t *__restrict__ y, int nb, int64_t nblocks) {
    const int lane = threadIdx.x & 63;
    const int64_t bi = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
    if (bi >= nblocks) return;  // whole 16-lane rows drop out together
    const int64_t row = bi / nb;
    const int b = (int)(bi - row * nb);
    const float *xb = x + row * x_stride + (int64_t)b * QK + 16 * (lane & 15);
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = *(const u32x4 *)(xb + 4 * k);
    quant16_store(v, lane & 15, y + bi * Q8L_STRIDE);
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
    r.isum = dlo * s0.sc_lo + dhi * s0.sc_hi;
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
    r.isum = dlo * s0.sc_lo + dhi * s0.sc_hi;
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
    r.isum = d00 * sbyte(SC, sb) + d01 * sbyte(SC, sb + 4) + d10 * sbyte(SC, sb + 1) + d11 * sbyte(SC, sb + 5);
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

template <int TYPE, bool FUSEDQ>
__device__ __forceinline__ void rows_body(const RowsArgs &a, const WaveWork &ww, uint8_t *smem, const RowsLayout &L,
                                          int wave, int lane, uint64_t st0) {
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int GRAN = rows_gran(TYPE);
    constexpr int NI = rows_ni(TYPE);
    constexpr int SLOT = rows_slot(TYPE);
    constexpr int D = rows_depth(TYPE);
    static_assert(D >= 2 && D <= 4, "vm_wait_k covers 3 steps in flight");
    const int nb = a.nb, bR = a.bR;
    const int q = lane >> 2, s = lane & 3;
    uint8_t *const ring = smem + L.ring + wave * L.ring_stride;
    uint8_t *const ring_end = ring + D * SLOT;
    Rec *const recs = (Rec *)(smem + L.recs + wave * L.recs_stride);
    float *const outs = (float *)(smem + L.outs + wave * L.outs_stride);
    const uint8_t *const actq = smem + L.act;

    // weight stream of this wave
    const int G = ww.nrows * nb;               // superblocks
    const int T = (G + ROWS_SB - 1) / ROWS_SB;  // steps
    const uint8_t *src = a.w[ww.m] + (int64_t)ww.r0 * nb * BSZ;
    const uint32_t mis = (uint32_t)((uintptr_t)src & 15u);
    const uint8_t *s16 = src - mis;
    const uint8_t *last16 =
        G > 0 ? (const uint8_t *)((uintptr_t)(src + (int64_t)G * BSZ - 1) & ~(uintptr_t)15) : s16;

    uint8_t *islot = ring;
    int it_ = 0;  // next step to issue
    auto issue = [&]() {
        const uint8_t *base = s16 + (int64_t)it_ * (ROWS_SB * BSZ) + 16 * lane;
        if (it_ + 1 < T) {  // interior step: every granule inside the stream
#pragma unroll
            for (int i = 0; i < NI; ++i)
                if (i + 1 < NI || lane < GRAN - 64 * (NI - 1)) dma16_nt(base + 1024 * i, (LDS void *)(islot + 1024 * i));
        } else {            // last step: clamp to the stream's last granule
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const uint8_t *p = base + 1024 * i;
                if (i + 1 < NI || lane < GRAN - 64 * (NI - 1))
                    dma16_nt(p < last16 ? p : last16, (LDS void *)(islot + 1024 * i));
            }
        }
        islot = islot + SLOT == ring_end ? ring : islot + SLOT;
        ++it_;
    };

    // ---- prologue: activation loads, pre0 weight steps, quantize, then the rest of the ring
    const int pre_cap = a.pre0 < D ? a.pre0 : D;  // never more than the ring holds
    const int pre0 = T < pre_cap ? T : pre_cap;     // 0..3
    uint64_t sx = 0, sq = 0, sf = 0;  // diagnostics: x landed, quantized, first step computed
    if (FUSEDQ) {
        constexpr int PASS = 4 * ROWS_WAVES;  // superblocks per workgroup pass
        u32x4 xv[ROWS_QPASS][4] = {};
        const int qiters = (nb + PASS - 1) / PASS;
#pragma unroll
        for (int i = 0; i < ROWS_QPASS; ++i) {
            if (i < qiters && PASS * i + 4 * wave < nb) {  // waves past the row load nothing
                int b = PASS * i + 4 * wave + (lane >> 4);
                b = b < nb ? b : nb - 1;
                const float *xp = a.x + (int64_t)b * QK + 16 * (lane & 15);
#pragma unroll
                for (int k = 0; k < 4; ++k) xv[i][k] = gload16_asm(xp + 4 * k);
            }
        }
        for (int j = 0; j < pre0; ++j) issue();
        vm_wait_k<NI>(pre0);  // the activation loads are older than pre0 weight steps
        // the loads above are invisible to the compiler: pin their registers past the wait
        asm volatile("" : "+v"(xv[0][0]), "+v"(xv[0][1]), "+v"(xv[0][2]), "+v"(xv[0][3]), "+v"(xv[1][0]),
                     "+v"(xv[1][1]), "+v"(xv[1][2]), "+v"(xv[1][3]), "+v"(xv[2][0]), "+v"(xv[2][1]), "+v"(xv[2][2]),
                     "+v"(xv[2][3]));
        if (a.stamps) sx = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
        for (int i = 0; i < qiters; ++i) {  // one copy of the quantizer; pick the pass's registers
            u32x4 cur[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) cur[k] = i == 0 ? xv[0][k] : i == 1 ? xv[1][k] : xv[2][k];
            const int b = PASS * i + 4 * wave + (lane >> 4);
            if (b < nb) quant16_store(cur, lane & 15, smem + L.act + Q8L_STRIDE * b);
        }
        if (a.stamps) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            sq = __builtin_amdgcn_s_memrealtime();
        }
    } else {
        const int ng = nb * (Q8L_STRIDE / 16);
        for (int j = wave; 64 * j < ng; j += ROWS_WAVES) {
            const int k = 64 * j + lane;
            if (k < ng) dma16(a.xq + 16 * k, (LDS void *)(smem + L.act + 1024 * j));
        }
        for (int j = 0; j < pre0; ++j) issue();
        vm_wait_k<NI>(pre0);
    }
    while (it_ < D && it_ < T) issue();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // Q8_K row complete (no vmcnt drain)
    const uint64_t st1 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;

    // ---- main loop
    int io = q, rr = 0;  // quad's (block, row-in-batch) of superblock 16t+q
    while (io >= nb) {
        io -= nb;
        ++rr;
    }
    int bend = bR * nb < G ? bR * nb : G;  // superblock index ending the current batch
    int brow = 0;
    const uint8_t *cslot = ring;
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
        if (T - t >= D) vm_wait<NI * (D - 1)>();  // steady state: D-1 younger steps in flight
        else vm_wait_k<NI>(T - t - 1);
        if (!(a.diag & 8) && ROWS_SB * t + q < G) {
            const uint8_t *blk = cslot + mis + q * BSZ;
            const uint8_t *ab = actq + io * Q8L_STRIDE;
            QuadOut r = TYPE == Q4_K ? quad_q4K(blk, ab, s) : TYPE == Q5_K ? quad_q5K(blk, ab, s) : quad_q6K(blk, ab, s);
            const int isum = quad_sum(r.isum);
            const int imin = quad_sum(r.imin);
            if (s == 0) {
                const float yd = *(const float *)ab;
                Rec rec;
                if (TYPE == Q6_K) {
                    rec.a = isum - 32 * imin;
                    rec.b = 0;
                    rec.c = h2f(r.dh) * yd;  // d_all * y.d
                    rec.e = 0.f;
                } else {
                    rec.a = isum;
                    rec.b = imin;
                    rec.c = yd * h2f(r.dh & 0xffffu);  // y.d * fp16(x.d)
                    rec.e = yd * h2f(r.dh >> 16);      // y.d * fp16(x.dmin)
                }
                recs[io * bR + rr] = rec;
            }
        }
        cslot = cslot + SLOT == ring_end ? ring : cslot + SLOT;
        io += ROWS_SB;
        if (nb >= ROWS_SB) {
            if (io >= nb) {
                io -= nb;
                ++rr;
            }
        } else {
            while (io >= nb) {
                io -= nb;
                ++rr;
            }
        }
        if (it_ < T) issue();
        if (a.stamps && t == 0) sf = __builtin_amdgcn_s_memrealtime();
        if (ROWS_SB * (t + 1) >= bend) {  // batch complete: replay its rows' chains, lane r <-> row r
            wave_lds_fence();
            const int nr = bR < ww.nrows - brow ? bR : ww.nrows - brow;
            if (lane < nr) {
                float v = 0.f;
                const Rec *rc = recs + lane;
#pragma unroll 4
                for (int i = 0; i < nb; ++i) v = chain_step(TYPE, rc[i * bR], v);
                outs[brow + lane] = v;
            }
            brow += bR;
            rr -= bR;
            bend = bend + bR * nb < G ? bend + bR * nb : G;
            wave_lds_fence();
        }
    }
    const uint64_t st2 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;

    // ---- flush staged results (coalesced)
    if (ww.nrows > 0) {
        wave_lds_fence();
        float *y = a.y[ww.m] + ww.r0;
        for (int k = 0; k < ww.nrows; k += 64)
            if (k + lane < ww.nrows) y[k + lane] = outs[k + lane];
    }
    if (a.stamps) {
        const int64_t o = ((int64_t)blockIdx.x * ROWS_WAVES + wave) * 8;
        if (lane == 0 && o + 7 < a.stamps_cap) {
            a.stamps[o] = st0;
            a.stamps[o + 1] = st1;
            a.stamps[o + 2] = st2;
            a.stamps[o + 3] = __builtin_amdgcn_s_memrealtime();
            a.stamps[o + 4] = sx;
            a.stamps[o + 5] = sq;
            a.stamps[o + 6] = sf;
        }
    }
}

template <int TMASK, bool FUSEDQ>
__global__ void __launch_bounds__(ROWS_WAVES * 64) kq_rows(const RowsArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint64_t st0 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const RowsLayout L = rows_layout(a.nb, TMASK, a.bR, a.rpw);

    const int gw = wave * gridDim.x + blockIdx.x;  // active waves spread over every CU
    WaveWork ww;
    int m = 0;
#pragma unroll
    for (int i = 1; i < MI355X_MAX_FUSED; ++i)
        if (i < a.n_desc && gw >= a.wave_prefix[i]) m = i;
    ww.m = m;
    const int j = gw - a.wave_prefix[m];
    const int base = a.rbase[m], rem = a.rrem[m];
    ww.r0 = j * base + (j < rem ? j : rem);
    ww.nrows = gw < a.waves_total ? base + (j < rem ? 1 : 0) : 0;

    if (TMASK == 1) {
        rows_body<Q4_K, FUSEDQ>(a, ww, smem, L, wave, lane, st0);
    } else if (TMASK == 2) {
        rows_body<Q5_K, FUSEDQ>(a, ww, smem, L, wave, lane, st0);
    } else if (TMASK == 4) {
        rows_body<Q6_K, FUSEDQ>(a, ww, smem, L, wave, lane, st0);
    } else {
        const int type = a.type[m];
        if (type == Q6_K) rows_body<Q6_K, FUSEDQ>(a, ww, smem, L, wave, lane, st0);
        else if (type == Q5_K) rows_body<Q5_K, FUSEDQ>(a, ww, smem, L, wave, lane, st0);
        else rows_body<Q4_K, FUSEDQ>(a, ww, smem, L, wave, lane, st0);
    }
}

#define KQ_ROWS_INST(TM, FQ) template __global__ void kq_rows<TM, FQ>(const RowsArgs a);
KQ_ROWS_INST(1, true)
KQ_ROWS_INST(2, true)
KQ_ROWS_INST(4, true)
KQ_ROWS_INST(7, true)
KQ_ROWS_INST(1, false)
KQ_ROWS_INST(2, false)
KQ_ROWS_INST(4, false)
KQ_ROWS_INST(7, false)

}  // namespace kq
