// kq_mmq.hip — batched (prefill) K-quant x Q8_K matmul on MFMA, bit-exact.
//
// Replaces, for ne11 = M > 1 activation columns, the per-(row, column) vec_dot
// calls of ggml_compute_forward_mul_mat_one_chunk (ggml-cpu.c:1194,
// README.md:136) with int8 matrix cores while keeping the reference's numerics:
//  * per 32-element sub-block j, v_mfma_i32_32x32x32_i8 gives exact int32 dots of
//    32 weight rows x 32 activation columns (K = 32 = one Q4_K sub-block). Q4_K:
//    the 6-bit scale is split into 3-bit halves folded into the weight operand
//    (nibble*half <= 105 fits int8), so sumi = 8*S8 + S1 accumulates across all
//    sub-blocks inside the matrix core; Q5_K: sumi += sc_j(row) * dot_j on VALU.
//    Exact int32 either way (README.md:754-771);
//  * summins = sum_j mn_j(row) * (bsums[2j] + bsums[2j+1]) on one f16 MFMA 32x32x16
//    (bs = 64*hi + lo split, below): integers below 2^24, so exact (README.md:741-744);
//  * the fp32 chain per output element runs superblock by superblock in order,
//    sumf = fmaf(-(float)summins, dmin, sumf); sumf = fmaf((float)sumi, d, sumf)
//    (fmsub/fmadd, README.md:551/:614) -- the same ops as the GEMV kernels, so
//    the result equals the oracle's mul_mat (and ggml's vec_dot loop) bit for bit.
// Tiles: a workgroup of 4 waves owns 64 activation columns x 64 weight rows (2x2
// waves of 32x32); each superblock's Q8L activation blocks (64 x 304 B) and weight
// blocks (64 x 144/176 B) are double-buffered in LDS by LDS-DMA, a fixed number of
// DMA instructions per wave and superblock so the wait is a constant vmcnt.
// MFMA operand maps (verified with exact integer data, tools/mfma_layout_check.hip):
//   i8 32x32x32: lane l (r = l&31, h = l>>5) holds A[r][16h+j], B[16h+j][r], j<16;
//   f16 32x32x16: A[r][8h+j], B[8h+j][r], j<8; C/D (every dtype): col = r,
//   row = (reg&3) + 8(reg>>2) + 4h.
#include "kq_device.h"
#include "kq_ops_device.h"

// Timing-only ablations of kq_mmq<Q4_K>, compile time so the product kernel carries none of
// them (as run-time branches they cost 40 VGPRs and a wave per SIMD): 1 no chain epilogue,
// 2 no scale split, 4 no integer MFMA, 8 no mins MFMA, 16 launch-order tiles.
// Experiment build: make variant-mmq NAME=d13 VFLAGS=-DKQ_MMQ_DIAG=13 (tools/mmq_diag.sh).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

#ifndef KQ_MMQ_DIAG
#define KQ_MMQ_DIAG 0
#endif
// Experiment build: Q4_K with unsplit operands (one int8 MFMA per sub-block, the scale
// applied on VALU as for Q5_K) instead of the scale split (two MFMAs per sub-block).
// Q6_K chunk loop unrolled by 2 and kq_mmq held to 2 waves per SIMD: fully unrolled, the
// compiler kept every chunk's MFMA results live (376 VGPRs, one wave per SIMD); now 146
// and Q6_K prefill 23-29 % faster, Q5_K 4 % (profiles/r02_prefill_ablation.md).
#ifndef KQ_MMQ_Q6_UNROLL
#define KQ_MMQ_Q6_UNROLL 2
#endif
#ifndef KQ_MMQ_WPE
#define KQ_MMQ_WPE 2
#endif
#if KQ_MMQ_WPE > 0
#define KQ_MMQ_WPE_ATTR __attribute__((amdgpu_waves_per_eu(KQ_MMQ_WPE)))
#else
#define KQ_MMQ_WPE_ATTR
#endif
#ifndef KQ_MMQ_Q4_VALU
#define KQ_MMQ_Q4_VALU 0
#endif
// One barrier per superblock (the next superblock's DMA issued right after it, into the
// buffer every wave has finished reading) instead of a landing and a release barrier:
// 2-12 % faster on every prefill shape (profiles/r03_mmq_onebar_tile128.txt). 0: the
// round-2 loop (experiment build).
#ifndef KQ_MMQ_ONEBAR
#define KQ_MMQ_ONEBAR 1
#endif
#ifndef KQ_MMQ_PKCHAIN
// The fp32 chain on packed f32 (v_pk_mul_f32 / v_pk_fma_f32, two elements per instruction,
// each lane an IEEE op: the same bits). Bits: 1 Q4_K (product: 8B ffn_down 3-8 % faster, the
// rest equal), 2 Q5_K, 4 Q6_K (no gain; experiment builds), profiles/r04_mmq_pkchain_ab.txt.
#define KQ_MMQ_PKCHAIN 1
#endif
// Experiment build: static issue priority 1 for the second half of the workgroup's waves (the
// arbitration losers of every two-waves-per-SIMD pair, MI355X_MICROARCH.md item 4).
#ifndef KQ_MMQ_PRIO
#define KQ_MMQ_PRIO 0
#endif
#ifndef KQ_MMQ_Q5_VALU
#define KQ_MMQ_Q5_VALU 0  // experiment build: Q5_K sub-block scales on VALU (the round-2 kernel)
#endif

namespace kq {

typedef int i32x4m __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) {
    u16x2 r;
    __builtin_memcpy(&r, &v, 4);
    return r;
}
__device__ __forceinline__ uint32_t as_u32(u16x2 v) {
    uint32_t r;
    __builtin_memcpy(&r, &v, 4);
    return r;
}


// Weight rows per workgroup: RT = 64 (4 waves, 2 x 2 of 32 x 32) or 128 (8 waves, 2 x 4):
// the activation tile is fetched once per RT rows, so RT = 128 halves its LDS-DMA traffic.

// Weight bytes per row in the LDS tile: the superblock itself (Q4_K 144, Q5_K 176,
// 16-B aligned rows), or for Q6_K (210 B, any alignment) the 14 granules from the
// 16-B boundary below it.
__host__ __device__ constexpr int mmq_row_bytes(int type) { return type == Q6_K ? KQ_MMQ_Q6_STRIDE : block_bytes(type); }
__host__ __device__ constexpr int mmq_b_instr(int type, int rt) { return rt * mmq_row_bytes(type) / 1024; }  // 9 / 11 / 15 per 64 rows
static_assert(64 * KQ_MMQ_Q6_STRIDE % 1024 == 0, "whole DMA instructions per 64 rows");


// Scale-split multipliers of sub-blocks 2jp (lo nibbles) and 2jp+1 (hi nibbles) as 16-bit
// pairs: sc = 8*sh + sl; sh / sl bytes of all four sub-blocks of a word split with two
// masks, then one byte-broadcast permute per multiplier.
struct SplitScales {
    uint32_t sh03, sl03, sh47, sl47;
};
__device__ __forceinline__ SplitScales split_scales(uint32_t s03, uint32_t s47) {
    return {(s03 >> 3) & 0x07070707u, s03 & 0x07070707u, (s47 >> 3) & 0x07070707u, s47 & 0x07070707u};
}
__device__ __forceinline__ uint32_t bcast16(uint32_t w, int k) {  // byte k of w in both 16-bit lanes
    return __builtin_amdgcn_perm(0u, w, 0x0c000c00u + 0x00010001u * (uint32_t)k);
}

// B operand of the mins MFMA: [mn_0..7 | 64*mn_0..7] of the lane's row (h selects the half),
// from the 6-bit mins bytes m03 / m47. Each byte pair becomes a 16-bit pair with a magic f16
// exponent (v_perm with a constant byte): 0x64 -> 1024 + mn (ulp 1), 0x54 -> 64 + mn/16
// (ulp 1/16); subtracting the magic and scaling by 1 or 1024 gives mn or 64*mn exactly.
__device__ __forceinline__ f16x8 mins_operand(uint32_t m03, uint32_t m47, int h) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const uint32_t magic = h ? 0x54545454u : 0x64646464u;
    const _Float16 base = h ? (_Float16)64.0f : (_Float16)1024.0f, mul = h ? (_Float16)1024.0f : (_Float16)1.0f;
    const h2 nb2 = {(_Float16)-base, (_Float16)-base}, m2 = {mul, mul};
    const uint32_t w[4] = {__builtin_amdgcn_perm(magic, m03, 0x04010400u), __builtin_amdgcn_perm(magic, m03, 0x04030402u),
                           __builtin_amdgcn_perm(magic, m47, 0x04010400u), __builtin_amdgcn_perm(magic, m47, 0x04030402u)};
    f16x8 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        h2 v;
        __builtin_memcpy(&v, &w[k], 4);
        v = (v + nb2) * m2;
        r[2 * k] = v[0];
        r[2 * k + 1] = v[1];
    }
    return r;
}

// Q6_K superblock of one 32x32 tile: 8 chunks of 32 elements; a lane's 16 values of a
// chunk are one 16-element scale group g (int8 scale sc). The scaled weight
// W = sc * (q - 32) (|W| <= 4096) rides in the MFMA operands as two int8 bytes,
// W = 256 * hi + lo with lo in [-128, 127] and hi = (W + 128) >> 8 in [-16, 16]: one
// packed 16-bit multiply-add per two values gives T = W + 128 = q*sc + (128 - 32 sc),
// whose high byte is hi and whose low byte xor 0x80 is lo. Both sums accumulate over
// the whole superblock in the matrix core, sumi = 256 * S_hi + S_lo exactly -- the
// reference's isum - 32*isum_mins with its scales (README.md:369-394 / lane_q6K) --
// instead of two half-empty MFMAs and 32 VALU multiplies per chunk.
// With CW column tiles per wave the weight operands of a chunk are built once and feed
// CW MFMA pairs (the activation operands differ per tile).
template <int CW>
__device__ __forceinline__ void q6_superblock(const MmqArgs &a, const uint8_t *Bbase, const uint8_t *const *At,
                                              const float *yd, int n, int b, int h, f32x16 *sumf) {
    const int nrow = n < a.n_rows ? n : a.n_rows - 1;  // the DMA clamped the same way
    const uint32_t mis = (uint32_t)((uintptr_t)(a.w + (int64_t)nrow * a.row_stride + (int64_t)b * 210) & 15u);
    const uint8_t *region = Bbase + mis;
    const uint32_t s4 = (uint32_t)((uintptr_t)region & 3u);
    const uint8_t *bb = region - s4;
    const u32x4 SC = realign(*(const u32x4a *)(bb + 192), *(const uint32_t *)(bb + 208), s4);
    const uint32_t dh = (*(const uint32_t *)(bb + 208) >> (8u * s4)) & 0xffffu;
    i32x16 shi[CW], slo[CW];
#pragma unroll
    for (int ct = 0; ct < CW; ++ct) shi[ct] = slo[ct] = i32x16{};
#pragma unroll
    for (int nh = 0; nh < 2; ++nh) {
        const u32x4 L0 = realign(*(const u32x4a *)(bb + 64 * nh + 16 * h), *(const uint32_t *)(bb + 64 * nh + 16 * h + 16), s4);
        const u32x4 L1 = realign(*(const u32x4a *)(bb + 64 * nh + 32 + 16 * h),
                                 *(const uint32_t *)(bb + 64 * nh + 48 + 16 * h), s4);
        const u32x4 H = realign(*(const u32x4a *)(bb + 128 + 32 * nh + 16 * h),
                                *(const uint32_t *)(bb + 144 + 32 * nh + 16 * h), s4);
#pragma unroll KQ_MMQ_Q6_UNROLL
        for (int cc = 0; cc < 4; ++cc) {
            const int c = 4 * nh + cc;  // chunk: elements 32c .. 32c+31
            const u32x4 L = (cc & 1) ? L1 : L0;
            const uint32_t sh = (uint32_t)(cc >> 1) * 4u;
            const int sc = h ? sbyte(SC, 2 * c + 1) : sbyte(SC, 2 * c);
            const uint32_t scw = (uint32_t)sc & 0xffffu, cw = (uint32_t)(128 - 32 * sc) & 0xffffu;
            const u16x2 scp = {(uint16_t)scw, (uint16_t)scw}, cp = {(uint16_t)cw, (uint16_t)cw};
            u32x4 blo, bhi;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t x = ((L[k] >> sh) & 0x0f0f0f0fu) | (((H[k] >> (2u * cc)) & 0x03030303u) << 4);  // q, 0..63
                const uint32_t t0 = as_u32(as_u16x2(__builtin_amdgcn_perm(0u, x, 0x0c010c00u)) * scp + cp);  // values 0, 1
                const uint32_t t1 = as_u32(as_u16x2(__builtin_amdgcn_perm(0u, x, 0x0c030c02u)) * scp + cp);  // values 2, 3
                blo[k] = __builtin_amdgcn_perm(t1, t0, 0x06040200u) ^ 0x80808080u;
                bhi[k] = __builtin_amdgcn_perm(t1, t0, 0x07050301u);
            }
#pragma unroll
            for (int ct = 0; ct < CW; ++ct) {
                const u32x4 act = *(const u32x4 *)(At[ct] + 16 + 32 * c + 16 * h);
                shi[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&act, *(const i32x4m *)&bhi, shi[ct], 0, 0, 0);
                slo[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&act, *(const i32x4m *)&blo, slo[ct], 0, 0, 0);
            }
        }
    }
    const float xd = h2f(dh);
    if (KQ_MMQ_PKCHAIN & 4) {  // experiment build: two elements per packed f32 instruction
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 xd2 = {xd, xd};
#pragma unroll
        for (int ct = 0; ct < CW; ++ct)
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                const f32x2 y2 = {yd[16 * ct + i], yd[16 * ct + i + 1]};
                const f32x2 s2 = {(float)(256 * shi[ct][i] + slo[ct][i]), (float)(256 * shi[ct][i + 1] + slo[ct][i + 1])};
                f32x2 acc = {sumf[ct][i], sumf[ct][i + 1]};
                acc = __builtin_elementwise_fma(xd2 * y2, s2, acc);
                sumf[ct][i] = acc.x;
                sumf[ct][i + 1] = acc.y;
            }
        return;
    }
#pragma unroll
    for (int ct = 0; ct < CW; ++ct)
#pragma unroll
        for (int i = 0; i < 16; ++i)  // sum += d_all*y.d*(isum - 32*isum_mins)
            sumf[ct][i] = fmaf(xd * yd[16 * ct + i], (float)(256 * shi[ct][i] + slo[ct][i]), sumf[ct][i]);
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (speed only,
// MI355X_MICROARCH.md), so the column tiles of one row tile go to blocks L, L + 8,
// L + 16, ... (one XCD): the weight tile is fetched into that XCD's L2 once and
// served from it to the others; the activation tiles fit every XCD's L2. With several
// matrices on one activation, a gets this row tile's matrix d (returned).
__device__ __forceinline__ int mmq_tile_of(const MmqArgs &a0, MmqArgs &a, int &tx, int &ty) {
    tx = blockIdx.x;
    ty = blockIdx.y;
    if (!(KQ_MMQ_DIAG & 16)) {
        const int gx = gridDim.x, L = blockIdx.y * gx + blockIdx.x;
        const int span = 8 * gx;                  // blocks per group of 8 row tiles
        const int grp = L / span, in = L - grp * span;
        const int rows_here = gridDim.y - 8 * grp < 8 ? gridDim.y - 8 * grp : 8;
        if (rows_here == 8) {
            ty = 8 * grp + in % 8;
            tx = in / 8;
        }
    }
    int d = 0;
    if (a0.n_mat > 1) {  // several matrices on one activation: this row tile's matrix
#pragma unroll
        for (int k = 1; k < 4; ++k)
            if (k < a0.n_mat && ty >= a0.tile0[k]) d = k;
        a.w = a0.mw[d];
        a.row_stride = a0.mrow_stride[d];
        a.n_rows = a0.mn_rows[d];
        a.y = a0.my[d];
        a.y_col_stride = a0.my_col_stride[d];
        a.kv_cur = a0.kv_kind[d];
        ty -= a0.tile0[d];
    }
    return d;
}

// One (64 * CW)-column x RT-row output tile over the whole K: RT / 16 waves, each 32 weight
// rows x 32 * CW columns (CW MFMA tiles sharing the wave's weight operands).
template <int TYPE, int RT, int CW>
__device__ __forceinline__ void mmq_tile(const MmqArgs &a, int tx, int ty) {
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int NWV = mmq_waves(RT, CW);  // waves
    constexpr int CG = mmq_cgroups(CW);     // column groups of waves
    constexpr int COLS = mmq_cols(CW);
    constexpr int A_BYTES = COLS * Q8L_STRIDE;
    constexpr int A_INSTR = A_BYTES / 1024;  // 19 per 64 columns (exact)
    constexpr int NB_I = mmq_b_instr(TYPE, RT);
    constexpr int NW = (A_INSTR + NB_I + NWV - 1) / NWV;
    constexpr int BUF = A_BYTES + RT * mmq_row_bytes(TYPE);
    constexpr int NBUF = mmq_nbuf(TYPE, RT, CW);
    static_assert(BUF == mmq_buf_bytes(TYPE, RT, CW), "host and kernel agree on the buffer size");
    static_assert(!KQ_MMQ_PF || (RT == 64 && CW == 1), "the L2 warm-up assumes the 4-wave 64 x 64 tile");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = CG == 2 ? wave & 1 : 0, wn = CG == 2 ? wave >> 1 : wave;
    const int r = lane & 31, h = lane >> 5;
    const int col0 = tx * COLS, row0 = ty * RT;
    const int nb = a.nb;

    // ---- DMA plan: the superblock's A_INSTR activation + NB_I weight instructions, NW per wave
    auto issue = [&](int b) {
        uint8_t *buf = smem + (NBUF == 2 ? (b & 1) : b % NBUF) * BUF;
#pragma unroll
        for (int s = 0; s < NW; ++s) {
            int t = wave + NWV * s;
            if (t >= A_INSTR + NB_I) t = A_INSTR + NB_I - 1;  // pad: repeat the last one
            const int g = 64 * (t < A_INSTR ? t : t - A_INSTR) + lane;  // granule in its tile
            const uint8_t *src;
            if (t < A_INSTR) {
                int c = g / (Q8L_STRIDE / 16);
                const int piece = g - c * (Q8L_STRIDE / 16);
                c = col0 + c < a.m_cols ? col0 + c : a.m_cols - 1;
                src = a.xq + (int64_t)c * a.xq_col_stride + (int64_t)b * Q8L_STRIDE + 16 * piece;
                dma16(src, (LDS void *)(buf + 1024 * t));
            } else {
                constexpr int RG = mmq_row_bytes(TYPE) / 16;
                int rw = g / RG;
                int piece = g - rw * RG;
                if (TYPE == Q6_K && piece > 13) piece = 13;  // padding granules: the row's last one again
                rw = row0 + rw < a.n_rows ? row0 + rw : a.n_rows - 1;
                const uintptr_t blk = (uintptr_t)(a.w + (int64_t)rw * a.row_stride + (int64_t)b * BSZ);
                src = (const uint8_t *)(blk & ~(uintptr_t)15) + 16 * piece;
                dma16(src, (LDS void *)(buf + A_BYTES + 1024 * (t - A_INSTR)));
            }
        }
        if (KQ_MMQ_PF) {  // L2 warm-up of superblock b + KQ_MMQ_PF's weight tile: one dword per
                          // 64-B piece of every row (LDS-DMA into a scratch area nobody reads)
            int bp = b + KQ_MMQ_PF - 1;
            bp = bp < nb ? bp : nb - 1;  // always one instruction: the vmcnt waits count it
            const int t = threadIdx.x, part = t & 3;
            int rw = row0 + (t >> 2);
            rw = rw < a.n_rows ? rw : a.n_rows - 1;
            const int off = part < 3 ? 64 * part : BSZ - 4;
            dma4((const void *)((uintptr_t)(a.w + (int64_t)rw * a.row_stride + (int64_t)bp * BSZ + off) & ~(uintptr_t)3),
                 (LDS void *)(smem + NBUF * BUF + 16 + 256 * wave));
        }
    };
    constexpr int NWP = NW + (KQ_MMQ_PF ? 1 : 0);  // vm instructions per issue()

    f32x16 sumf[CW];
#pragma unroll
    for (int ct = 0; ct < CW; ++ct)
#pragma unroll
        for (int i = 0; i < 16; ++i) sumf[ct][i] = 0.f;

    if (KQ_MMQ_PRIO && NWV >= 8 && wave >= NWV / 2) __builtin_amdgcn_s_setprio(1);
    if (NBUF > 1) issue(0);
    if (NBUF == 3 && nb > 1) issue(1);
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {
        if (NBUF == 1) {
            // one buffer (experiment: occupancy instead of double buffering): every wave
            // finished reading b - 1 at the trailing barrier of the previous iteration
            issue(b);
            vm_wait<0>();
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        } else if (NBUF == 3) {
            // superblock b landed (b + 1's DMAs, younger, may be in flight); after the barrier
            // every wave has finished reading b - 1's buffer, where b + 2 goes
            if (b + 1 < nb) vm_wait<NWP>();
            else vm_wait<0>();
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            if (b + 2 < nb) issue(b + 2);
        } else if (KQ_MMQ_ONEBAR) {
            // superblock b (the only DMA in flight) landed; after the barrier every wave's part
            // of b is in LDS and every wave has finished reading b - 1's buffer (lgkmcnt(0)
            // before it), so b + 1 goes into that buffer while b is computed
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            if (b + 1 < nb) issue(b + 1);
        } else {
            if (b + 1 < nb) {
                issue(b + 1);
                vm_wait<NWP>();  // superblock b's DMAs (older than b+1's NW) have landed
            } else {
                vm_wait<0>();
            }
            asm volatile("s_barrier" ::: "memory");  // every wave's part of superblock b
        }
        const uint8_t *buf = smem + (NBUF == 2 ? (b & 1) : b % NBUF) * BUF;
        const uint8_t *At[CW];  // this lane's activation column of each tile
#pragma unroll
        for (int ct = 0; ct < CW; ++ct) At[ct] = buf + (32 * CW * wm + 32 * ct + r) * Q8L_STRIDE;
        // y.d of the column accumulator element i of tile ct belongs to (read where it is used)
        auto yd_of = [&](int ct, int i) {
            return *(const float *)(buf + (32 * CW * wm + 32 * ct + (i & 3) + 8 * (i >> 2) + 4 * h) * Q8L_STRIDE);
        };
        const uint8_t *Bt = buf + A_BYTES + (32 * wn + r) * mmq_row_bytes(TYPE);  // this lane's weight row
        if (TYPE == Q6_K) {
            float yd[16 * CW];
#pragma unroll
            for (int ct = 0; ct < CW; ++ct)
#pragma unroll
                for (int i = 0; i < 16; ++i) yd[16 * ct + i] = yd_of(ct, i);
            q6_superblock<CW>(a, Bt, At, yd, row0 + 32 * wn + r, b, h, sumf);
            if (!KQ_MMQ_ONEBAR || NBUF == 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            continue;
        }
        const u32x4 hdr = *(const u32x4 *)Bt;
        // 6-bit scales / mins of the lane's row (get_scale_min_k4, README.md:732-739)
        const uint32_t s03 = hdr.y & 0x3f3f3f3fu;
        const uint32_t m03 = hdr.z & 0x3f3f3f3fu;
        const uint32_t s47 = (hdr.w & 0x0f0f0f0fu) | ((hdr.y >> 2) & 0x30303030u);
        const SplitScales ss = split_scales(s03, s47);
        const uint32_t m47 = ((hdr.w >> 4) & 0x0f0f0f0fu) | ((hdr.z >> 2) & 0x30303030u);
        // Q4_K / Q5_K: sumi = 8*s8 + s1 (scale split into 3-bit halves; Q5_K's fifth bit in s8)
        i32x16 sumi[CW], s8[CW], s1[CW];
#pragma unroll
        for (int ct = 0; ct < CW; ++ct) sumi[ct] = s8[ct] = s1[ct] = i32x16{};
        u32x4 qh = {0u, 0u, 0u, 0u};
        if (TYPE == Q5_K) qh = *(const u32x4 *)(Bt + 16 + 16 * h);
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
            const u32x4 qv = *(const u32x4 *)(Bt + (TYPE == Q5_K ? 48 : 16) + 32 * jp + 16 * h);
            u32x4 lo = qv & 0x0f0f0f0fu, hi = (qv >> 4) & 0x0f0f0f0fu;
            if (TYPE == Q5_K && KQ_MMQ_Q5_VALU) {  // the whole 5-bit quant (the VALU-scaled experiment)
                lo = lo | (((qh >> (uint32_t)(2 * jp)) & 0x01010101u) << 4);
                hi = hi | (((qh >> (uint32_t)(2 * jp + 1)) & 0x01010101u) << 4);
            }
            u32x4 alo[CW], ahi[CW];
#pragma unroll
            for (int ct = 0; ct < CW; ++ct) {
                alo[ct] = *(const u32x4 *)(At[ct] + 16 + 64 * jp + 16 * h);
                ahi[ct] = *(const u32x4 *)(At[ct] + 48 + 64 * jp + 16 * h);
            }
            const uint32_t sw = jp < 2 ? s03 : s47;
            const int sc_lo = (int)((sw >> (16u * (uint32_t)(jp & 1))) & 0xffu);
            const int sc_hi = (int)((sw >> (16u * (uint32_t)(jp & 1) + 8u)) & 0xffu);
            if (TYPE == Q4_K && (KQ_MMQ_DIAG & 6)) {  // diagnostics (timing only)
#pragma unroll
                for (int ct = 0; ct < CW; ++ct) {
                    if (!(KQ_MMQ_DIAG & 4)) {
                        s8[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&alo[ct], *(const i32x4m *)&lo, s8[ct], 0, 0, 0);
                        s1[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&ahi[ct], *(const i32x4m *)&hi, s1[ct], 0, 0, 0);
                    } else {
                        s8[ct][jp] += (int)(lo.x ^ alo[ct].y ^ (uint32_t)sc_lo);
                        s1[ct][jp] += (int)(hi.y ^ ahi[ct].x ^ (uint32_t)sc_hi);
                    }
                }
            } else if (TYPE == Q4_K && !KQ_MMQ_Q4_VALU) {
                // sc = 8*sh + sl (3-bit halves): nibble*sh and nibble*sl <= 105 stay int8, and a
                // packed 16-bit multiply scales two bytes per half without carries, so the
                // per-sub-block scale rides in the MFMA operand and both sums accumulate
                // across sub-blocks in the matrix core (exact int32).
                const int kb = 2 * (jp & 1);  // bytes of sub-blocks 2jp, 2jp+1 in their word
                const u16x2 lh = as_u16x2(bcast16(jp < 2 ? ss.sh03 : ss.sh47, kb));
                const u16x2 ll = as_u16x2(bcast16(jp < 2 ? ss.sl03 : ss.sl47, kb));
                const u16x2 hh = as_u16x2(bcast16(jp < 2 ? ss.sh03 : ss.sh47, kb + 1));
                const u16x2 hl = as_u16x2(bcast16(jp < 2 ? ss.sl03 : ss.sl47, kb + 1));
                u32x4 b8lo, b1lo, b8hi, b1hi;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    b8lo[k] = as_u32(as_u16x2(lo[k]) * lh);
                    b1lo[k] = as_u32(as_u16x2(lo[k]) * ll);
                    b8hi[k] = as_u32(as_u16x2(hi[k]) * hh);
                    b1hi[k] = as_u32(as_u16x2(hi[k]) * hl);
                }
#pragma unroll
                for (int ct = 0; ct < CW; ++ct) {
                    s8[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&alo[ct], *(const i32x4m *)&b8lo, s8[ct], 0, 0, 0);
                    s1[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&alo[ct], *(const i32x4m *)&b1lo, s1[ct], 0, 0, 0);
                    s8[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&ahi[ct], *(const i32x4m *)&b8hi, s8[ct], 0, 0, 0);
                    s1[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&ahi[ct], *(const i32x4m *)&b1hi, s1[ct], 0, 0, 0);
                }
            } else if (TYPE == Q5_K && !KQ_MMQ_Q5_VALU) {
                // Q5_K: q = ql + 16 qh (ql the nibble, qh the fifth bit) and, as for Q4_K,
                // sc = 8 sh + sl (3-bit halves): W = sc q = 8 (sh ql + 2 sc qh) + sl ql with
                // sh ql, sl ql <= 105 and 2 sc qh <= 126 all int8, so three MFMAs per sub-block,
                // two of them into the x8 sum, accumulate over the superblock in the matrix core:
                // sumi = 8 S8 + S1 (exact int32). The packed 16-bit multiplies scale two bytes
                // per lane half without carries, as in the Q4_K split.
                const int kb = 2 * (jp & 1);  // bytes of sub-blocks 2jp, 2jp+1 in their word
                const u16x2 lh = as_u16x2(bcast16(jp < 2 ? ss.sh03 : ss.sh47, kb));
                const u16x2 ll = as_u16x2(bcast16(jp < 2 ? ss.sl03 : ss.sl47, kb));
                const u16x2 hh = as_u16x2(bcast16(jp < 2 ? ss.sh03 : ss.sh47, kb + 1));
                const u16x2 hl = as_u16x2(bcast16(jp < 2 ? ss.sl03 : ss.sl47, kb + 1));
                const u16x2 scl = {(uint16_t)(2 * sc_lo), (uint16_t)(2 * sc_lo)};
                const u16x2 sch = {(uint16_t)(2 * sc_hi), (uint16_t)(2 * sc_hi)};
#pragma unroll
                for (int half = 0; half < 2; ++half) {  // sub-block 2jp (lo nibbles), then 2jp+1
                    const u32x4 &qn = half ? hi : lo;
                    const u16x2 m8 = half ? hh : lh, m1 = half ? hl : ll, mq = half ? sch : scl;
                    u32x4 b8, b1, bq;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        b8[k] = as_u32(as_u16x2(qn[k]) * m8);
                        b1[k] = as_u32(as_u16x2(qn[k]) * m1);
                        bq[k] = as_u32(as_u16x2((qh[k] >> (uint32_t)(2 * jp + half)) & 0x01010101u) * mq);
                    }
#pragma unroll
                    for (int ct = 0; ct < CW; ++ct) {
                        const u32x4 &av = half ? ahi[ct] : alo[ct];
                        s8[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&av, *(const i32x4m *)&b8, s8[ct], 0, 0, 0);
                        s1[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&av, *(const i32x4m *)&b1, s1[ct], 0, 0, 0);
                        s8[ct] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&av, *(const i32x4m *)&bq, s8[ct], 0, 0, 0);
                    }
                }
            } else {  // Q5_K in the KQ_MMQ_Q5_VALU experiment build (and Q4_K in KQ_MMQ_Q4_VALU):
                      // per-sub-block dots scaled on VALU
                const i32x16 zero = {};
#pragma unroll
                for (int ct = 0; ct < CW; ++ct) {
                    i32x16 c = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&alo[ct], *(const i32x4m *)&lo, zero, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 16; ++i) sumi[ct][i] += __mul24(sc_lo, c[i]);  // |c| < 2^17: full-rate i24
                    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const i32x4m *)&ahi[ct], *(const i32x4m *)&hi, zero, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 16; ++i) sumi[ct][i] += __mul24(sc_hi, c[i]);
                }
            }
        }
#pragma unroll
        for (int ct = 0; ct < CW; ++ct) {
            if (TYPE == Q4_K && !KQ_MMQ_Q4_VALU) {
#pragma unroll
                for (int i = 0; i < 16; ++i) sumi[ct][i] = 8 * s8[ct][i] + s1[ct][i];
            }
            if (TYPE == Q5_K && !KQ_MMQ_Q5_VALU) {
#pragma unroll
                for (int i = 0; i < 16; ++i) sumi[ct][i] = 8 * s8[ct][i] + s1[ct][i];
            }
        }
        // summins = sum_j mn_j * bs_j exactly on one f16 MFMA 32x32x16 per tile (bs_j =
        // bsums[2j] + bsums[2j+1] = 64*hi + lo, lo in 0..63): A = [lo_0..7 | hi_0..7] of the
        // lane's activation column (stored so by the quantizer: the Q8L/mmq layout), B = [mn_0..7 |
        // 64*mn_0..7] of its weight row; every product and partial sum is an integer below 2^24.
        // (Four dependent f32 MFMAs 32x32x2 cost 256 cycles per superblock against 32 for this one.)
        const f16x8 bm = mins_operand(m03, m47, h);
        // the reference's fp32 update per element, superblock order
        const float xd = h2f(hdr.x & 0xffffu), xdm = h2f(hdr.x >> 16), nxdm = -xdm;
#pragma unroll
        for (int ct = 0; ct < CW; ++ct) {
            const f16x8 am = *(const f16x8 *)(At[ct] + 272 + 16 * h);  // [lo | hi] of bs_j (Q8L/mmq)
            const f32x16 zero = {};
            const f32x16 mins = (KQ_MMQ_DIAG & 8) ? zero : __builtin_amdgcn_mfma_f32_32x32x16_f16(am, bm, zero, 0, 0, 0);
            if ((KQ_MMQ_PKCHAIN & 1) && TYPE == Q4_K && !(KQ_MMQ_DIAG & 1)) {
                // two elements per packed f32 instruction (each lane an IEEE mul / fma: the
                // scalar chain's bits)
                typedef float f32x2 __attribute__((ext_vector_type(2)));
                const f32x2 nxdm2 = {nxdm, nxdm}, xd2 = {xd, xd};
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    const f32x2 y2 = {yd_of(ct, i), yd_of(ct, i + 1)};
                    const f32x2 m2 = {mins[i], mins[i + 1]};
                    const f32x2 s2 = {(float)sumi[ct][i], (float)sumi[ct][i + 1]};
                    f32x2 acc = {sumf[ct][i], sumf[ct][i + 1]};
                    acc = __builtin_elementwise_fma(m2, y2 * nxdm2, acc);
                    acc = __builtin_elementwise_fma(s2, y2 * xd2, acc);
                    sumf[ct][i] = acc.x;
                    sumf[ct][i + 1] = acc.y;
                }
                continue;
            }
            if ((KQ_MMQ_PKCHAIN & 2) && TYPE == Q5_K && !(KQ_MMQ_DIAG & 1)) {
                typedef float f32x2 __attribute__((ext_vector_type(2)));
                const f32x2 xd2 = {xd, xd}, xdm2 = {xdm, xdm};
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    const f32x2 y2 = {yd_of(ct, i), yd_of(ct, i + 1)};
                    const f32x2 m2 = {mins[i], mins[i + 1]};
                    const f32x2 s2 = {(float)sumi[ct][i], (float)sumi[ct][i + 1]};
                    const f32x2 t = __builtin_elementwise_fma(y2 * xd2, s2, -((y2 * xdm2) * m2));
                    f32x2 acc = {sumf[ct][i], sumf[ct][i + 1]};
                    acc = acc + t;
                    sumf[ct][i] = acc.x;
                    sumf[ct][i + 1] = acc.y;
                }
                continue;
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float y = yd_of(ct, i);
                if (KQ_MMQ_DIAG & 1) {  // diagnostics (timing only)
                    sumf[ct][i] += (float)sumi[ct][i] + mins[i] + y;
                } else if (TYPE == Q5_K) {
                    const float t = fmaf(y * xd, (float)sumi[ct][i], -((y * xdm) * mins[i]));
                    sumf[ct][i] = sumf[ct][i] + t;
                } else {
                    sumf[ct][i] = fmaf(mins[i], y * nxdm, sumf[ct][i]);  // = fmaf(-mins, yd*xdm, .) exactly
                    sumf[ct][i] = fmaf((float)sumi[ct][i], y * xd, sumf[ct][i]);
                }
            }
        }
        if (!KQ_MMQ_ONEBAR || NBUF == 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // buffer b&1 free for b+2
    }

    // ---- store: lane's weight row n, 16 activation columns per tile
    const int n = row0 + 32 * wn + r;
#pragma unroll
    for (int ct = 0; ct < CW; ++ct) {
        const int cb = col0 + 32 * CW * wm + 32 * ct;
        if (n < a.n_rows) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int m = cb + (i & 3) + 8 * (i >> 2) + 4 * h;
                if (m < a.m_cols)
                    a.y[(int64_t)m * a.y_col_stride + n] =
                        a.res ? sumf[ct][i] + a.res[(int64_t)m * a.res_col_stride + n] : sumf[ct][i];
            }
        }
        if (a.kv_cur) {  // the prompt's KV-cache cells, as kq_kv_store computes them (kq_ops.hip)
            const int hd = a.kv_hd;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int m = cb + (i & 3) + 8 * (i >> 2) + 4 * h;
                const float other = __shfl_xor(sumf[ct][i], 1, 64);  // row n ^ 1: the rope partner
                const int pos = m < a.m_cols ? a.kv_pos[m] : -1;
                if (n >= a.n_rows || pos < 0 || pos >= a.kv_n_ctx) continue;  // no cell (its output is NaN)
                if (a.kv_cur == 1) {
                    const int pr = (n % hd) >> 1;
                    const float *tc = a.kv_rope + (int64_t)pos * (hd / 2) * 2;
                    const bool odd = n & 1;
                    const float2 rk = rope_pair(odd ? other : sumf[ct][i], odd ? sumf[ct][i] : other, tc[2 * pr], tc[2 * pr + 1]);
                    a.kv_k_cache[(int64_t)pos * a.n_rows + n] = h2u(f2h_rne(odd ? rk.y : rk.x));
                } else {
                    a.kv_v_cache[(int64_t)n * a.kv_n_ctx + pos] = h2u(f2h_rne(sumf[ct][i]));
                }
            }
        }
    }
}

// (64 x 128: one 4-wave workgroup per CU by LDS, so one wave per SIMD and every register)
#define KQ_MMQ_WPE_OF(RT, CW) __attribute__((amdgpu_waves_per_eu(((RT) == 64 && (CW) == 2) || (CW) == 4 ? 1 : (RT) == 192 ? 3 : KQ_MMQ_WPE)))
template <int TYPE, int RT, int CW>
__global__ void __launch_bounds__(mmq_waves(RT, CW) * 64) KQ_MMQ_WPE_OF(RT, CW) kq_mmq(const MmqArgs a0) {
    MmqArgs a = a0;
    int tx, ty;
    mmq_tile_of(a0, a, tx, ty);
    mmq_tile<TYPE, RT, CW>(a, tx, ty);
}

// Q4_K / Q5_K and Q6_K matrices on one activation in one launch (a prompt batch's q/k with a
// Q6_K attn_v): each row tile runs its matrix's kernel body (a0.mtype), LDS sized for Q6_K.
template <int RT, int CW>
__global__ void __launch_bounds__(mmq_waves(RT, CW) * 64) KQ_MMQ_WPE_OF(RT, CW) kq_mmq_mixed(const MmqArgs a0) {
    MmqArgs a = a0;
    int tx, ty;
    const int d = mmq_tile_of(a0, a, tx, ty);
    if (a0.mtype[d] == Q6_K) {
        mmq_tile<Q6_K, RT, CW>(a, tx, ty);
    } else if (a0.mtype[d] == Q5_K) {
        // (the host never launches a Q5_K matrix on the mixed 128 x 128 tiles: beside the
        // Q6_K body its registers would spill; launch_mmq_multi takes 128 x 64 there)
        if constexpr (!(RT == 128 && CW == 2)) mmq_tile<Q5_K, RT, CW>(a, tx, ty);
    } else {
        mmq_tile<Q4_K, RT, CW>(a, tx, ty);
    }
}

#define KQ_MMQ_INST(RT, CW)                                         \
    template __global__ void kq_mmq<Q4_K, RT, CW>(const MmqArgs a); \
    template __global__ void kq_mmq<Q5_K, RT, CW>(const MmqArgs a); \
    template __global__ void kq_mmq<Q6_K, RT, CW>(const MmqArgs a); \
    template __global__ void kq_mmq_mixed<RT, CW>(const MmqArgs a);
KQ_MMQ_INST(64, 1)
KQ_MMQ_INST(128, 1)
KQ_MMQ_INST(128, 2)
KQ_MMQ_INST(64, 2)
template __global__ void kq_mmq<Q4_K, 128, 4>(const MmqArgs a);
template __global__ void kq_mmq<Q4_K, 192, 1>(const MmqArgs a);
template __global__ void kq_mmq<Q5_K, 192, 1>(const MmqArgs a);
template __global__ void kq_mmq<Q5_K, 128, 4>(const MmqArgs a);

}  // namespace kq
