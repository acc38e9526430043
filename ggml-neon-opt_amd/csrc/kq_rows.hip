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
//    rows that is ONE contiguous byte stream, fetched in steps of 8 superblocks
//    (1152 / 1408 / 1680 B) by two LDS-DMA instructions (global_load_lds_dwordx4,
//    16-B granules) into a per-wave ring of D slots, completion by counted
//    s_waitcnt vmcnt; no workgroup barrier after the prologue;
//  * lane octet o computes superblock 8t+o of the stream (8 lanes x 32 quants,
//    v_dot4_i32_i8, 3 DPP adds) and its leader stores the exact fp32 operands of
//    the reference's update as a 16-B record, block-major per row batch;
//  * when a batch of bR rows is complete, lane r replays row r's records in
//    superblock order (the serial fp32 chain, 64 rows per instruction);
//  * the activation is quantized to Q8_K once per workgroup into LDS: 16 lanes
//    per superblock, x loaded by inline-asm global loads issued before the
//    weight DMAs (K <= 8192), or its raw Q8_K row copied by LDS-DMA.
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
// Writes the block's 292 bytes at `qb` (LDS).
__device__ __forceinline__ void quant16_store(const u32x4 v[4], int l, uint8_t *qb) {
    float x[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        x[4 * k + 0] = __uint_as_float(v[k].x);
        x[4 * k + 1] = __uint_as_float(v[k].y);
        x[4 * k + 2] = __uint_as_float(v[k].z);
        x[4 * k + 3] = __uint_as_float(v[k].w);
    }
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) m = fmaxf(m, fabsf(x[k]));  // fmaxf drops NaN
    int mb = (m == m) ? __float_as_int(m) : 0;
    mb = row16_reduce(mb, [](int a, int c) { return a > c ? a : c; });
    m = __int_as_float(mb);
    uint32_t key = 0xffffffffu;
#pragma unroll
    for (int k = 15; k >= 0; --k)
        if (fabsf(x[k]) == m) key = 2u * (uint32_t)(16 * l + k) + (x[k] < 0.f ? 1u : 0u);
    key = (uint32_t)row16_reduce((int)key, [](int a, int c) { return (uint32_t)a < (uint32_t)c ? a : c; });
    const float maxv = (key & 1u) ? -m : m;
    const float iscale = -127.f / maxv;
    u32x4 q;
    uint32_t *qw = (uint32_t *)&q;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        qw[k] = qbyte(iscale, x[4 * k]) | (qbyte(iscale, x[4 * k + 1]) << 8) | (qbyte(iscale, x[4 * k + 2]) << 16) |
                (qbyte(iscale, x[4 * k + 3]) << 24);
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
    *(u32x4a *)(qb + 4 + 16 * l) = q;
    *(int16_t *)(qb + 260 + 2 * l) = (int16_t)bsum;
    if (l == 0) *(float *)qb = d;
}

__device__ __forceinline__ u32x4 gload16_asm(const float *p) {
    u32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}

// ---------------------------------------------------------------- the row stream of one wave
struct WaveWork {
    int m, r0, nrows;
};

template <int TYPE, bool FUSEDQ>
__device__ __forceinline__ void rows_body(const RowsArgs &a, const WaveWork &ww, uint8_t *smem, const RowsLayout &L,
                                          int slot_bytes, int wave, int lane, uint64_t st0) {
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int GRAN = rows_gran(TYPE);
    constexpr int TM = TYPE == Q4_K ? 1 : TYPE == Q5_K ? 2 : 4;
    const int nb = a.nb, D = a.ring, bR = a.bR;
    const int o = lane >> 3, p = lane & 7;
    uint8_t *const ring = smem + L.ring + wave * L.ring_stride;
    uint8_t *const ring_end = ring + D * slot_bytes;
    Rec *const recs = (Rec *)(smem + L.recs + wave * L.recs_stride);
    float *const outs = (float *)(smem + L.outs + wave * L.outs_stride);

    // weight stream of this wave
    const int G = ww.nrows * nb;  // superblocks
    const int T = (G + 7) >> 3;   // steps
    const uint8_t *src = a.w[ww.m] + (int64_t)ww.r0 * nb * BSZ;
    const uint32_t mis = (uint32_t)((uintptr_t)src & 15u);
    const uint8_t *s16 = src - mis;
    const uint8_t *last16 =
        G > 0 ? (const uint8_t *)((uintptr_t)(src + (int64_t)G * BSZ - 1) & ~(uintptr_t)15) : s16;

    uint8_t *islot = ring;
    int it_ = 0;  // next step to issue
    auto issue = [&]() {
        const uint8_t *base = s16 + (int64_t)it_ * (8 * BSZ);
        const uint8_t *p0 = base + 16 * lane;
        dma16(p0 < last16 ? p0 : last16, (LDS void *)islot);
        if (lane < GRAN - 64) {
            const uint8_t *p1 = base + 1024 + 16 * lane;
            dma16(p1 < last16 ? p1 : last16, (LDS void *)(islot + 1024));
        }
        islot = islot + slot_bytes == ring_end ? ring : islot + slot_bytes;
        ++it_;
    };

    // ---- prologue: activation loads first, then the first D weight steps, then quantize
    u32x4 xv[2][4] = {};
    const int qiters = (nb + 15) >> 4;  // 16 superblocks per workgroup pass
    uint8_t *actq = smem + L.act;
    if (FUSEDQ) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i < qiters) {
                int b = 16 * i + 4 * wave + (lane >> 4);
                b = b < nb ? b : nb - 1;
                const float *xp = a.x + (int64_t)b * QK + 16 * (lane & 15);
#pragma unroll
                for (int k = 0; k < 4; ++k) xv[i][k] = gload16_asm(xp + 4 * k);
            }
        }
    } else {
        const uintptr_t q0 = (uintptr_t)a.xq;
        const uint8_t *q16 = (const uint8_t *)(q0 & ~(uintptr_t)15);
        actq = smem + L.act + (q0 & 15u);
        const int ng = (int)(((q0 & 15u) + (uintptr_t)nb * 292 + 15) / 16);
        for (int j = wave; 64 * j < ng; j += WAVES_PER_WG) {
            const int k = 64 * j + lane;
            if (k < ng) dma16(q16 + 16 * k, (LDS void *)(smem + L.act + 1024 * j));
        }
    }
    const int pre = T < D ? T : D;
    for (int j = 0; j < pre; ++j) issue();
    vm_wait_steps(pre);  // activation loads are older than the 2*pre weight DMAs
    if (FUSEDQ) {
        asm volatile("" : "+v"(xv[0][0]), "+v"(xv[0][1]), "+v"(xv[0][2]), "+v"(xv[0][3]), "+v"(xv[1][0]),
                     "+v"(xv[1][1]), "+v"(xv[1][2]), "+v"(xv[1][3]));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i < qiters) {
                const int b = 16 * i + 4 * wave + (lane >> 4);
                if (b < nb) quant16_store(xv[i], lane & 15, actq + 292 * b);
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // Q8_K row complete (no vmcnt drain)
    const uint64_t st1 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;

    // ---- main loop
    int io = o, rr = 0;  // octet's (block, row-in-batch) of superblock 8t+o
    while (io >= nb) {
        io -= nb;
        ++rr;
    }
    int bend = bR * nb < G ? bR * nb : G;  // superblock index ending the current batch
    int brow = 0;
    const uint8_t *cslot = ring;
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
        vm_wait_steps((T - t < D ? T - t : D) - 1);
        if (!(a.diag & 8) && 8 * t + o < G) {
            const uint32_t off = mis + (uint32_t)(o * BSZ);
            Regs rg;
            lds_block<TM>(rg, cslot + (off & ~15u), off & 15u, TYPE, p);
            const uint8_t *ab = actq + io * 292;
            int isum = 0, imin = 0;
            uint32_t dh = rg.dh;
            lane_partials<TM>(rg, ab + 4, (const int16_t *)(ab + 260), TYPE, p, isum, imin, dh);
            isum = octet_sum(isum);
            imin = octet_sum(imin);
            const Rec rec = make_rec<TM>(TYPE, isum, imin, rg, dh, *(const float *)ab);
            if (p == 0) recs[io * bR + rr] = rec;
        }
        cslot = cslot + slot_bytes == ring_end ? ring : cslot + slot_bytes;
        io += 8;
        while (io >= nb) {
            io -= nb;
            ++rr;
        }
        if (it_ < T) issue();
        if (8 * t + 8 >= bend) {  // batch complete: replay its rows' chains, lane r <-> row r
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
        const int64_t s = ((int64_t)blockIdx.x * WAVES_PER_WG + wave) * 8;
        if (lane == 0 && s + 7 < a.stamps_cap) {
            a.stamps[s] = st0;
            a.stamps[s + 1] = st1;
            a.stamps[s + 2] = st2;
            a.stamps[s + 3] = __builtin_amdgcn_s_memrealtime();
            a.stamps[s + 4] = st0;
            a.stamps[s + 5] = st0;
            a.stamps[s + 6] = st1;
        }
    }
}

template <int TMASK, bool FUSEDQ>
__global__ void __launch_bounds__(WG_THREADS) kq_rows(const RowsArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint64_t st0 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int SLOT = rows_slot(TMASK);
    const RowsLayout L = rows_layout(a.nb, SLOT, a.ring, a.bR, a.rpw);

    const int gw = blockIdx.x * WAVES_PER_WG + wave;
    WaveWork ww;
    int m = 0;
#pragma unroll
    for (int i = 1; i < MI355X_MAX_FUSED; ++i)
        if (i < a.n_desc && gw >= a.wave_prefix[i]) m = i;
    ww.m = m;
    ww.r0 = (gw - a.wave_prefix[m]) * a.rpw;
    const int left = a.n_rows[m] - ww.r0;
    ww.nrows = gw < a.waves_total ? (left < a.rpw ? left : a.rpw) : 0;
    if (ww.nrows < 0) ww.nrows = 0;

    if (TMASK == 1) {
        rows_body<Q4_K, FUSEDQ>(a, ww, smem, L, SLOT, wave, lane, st0);
    } else if (TMASK == 2) {
        rows_body<Q5_K, FUSEDQ>(a, ww, smem, L, SLOT, wave, lane, st0);
    } else if (TMASK == 4) {
        rows_body<Q6_K, FUSEDQ>(a, ww, smem, L, SLOT, wave, lane, st0);
    } else {
        const int type = a.type[m];
        if (type == Q6_K) rows_body<Q6_K, FUSEDQ>(a, ww, smem, L, SLOT, wave, lane, st0);
        else if (type == Q5_K) rows_body<Q5_K, FUSEDQ>(a, ww, smem, L, SLOT, wave, lane, st0);
        else rows_body<Q4_K, FUSEDQ>(a, ww, smem, L, SLOT, wave, lane, st0);
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
