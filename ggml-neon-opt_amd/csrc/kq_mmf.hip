// kq_mmf.hip — batched (prefill, M >= 16) K-quant matmul on the f16 matrix core: the
// stated-tolerance path beside the bit-exact kq_mmq (mi355x_prefill_precision).
//
// north_star: "bit-exact on the integer dequant/index arithmetic and within a stated
// fp32 tolerance on the accumulated dot". This path keeps the reference's integer side
// exactly -- the activation is quantized by quantize_row_q8_K_ref semantics
// (kq_device.h quant_values_wave), the 4/5/6-bit quants and the 6-bit / int8 scales are
// unpacked as ggml does (README.md:732-739 get_scale_min_k4; dequantize_row_q6_K) -- and
// moves the accumulation onto v_mfma_f32_32x32x16_f16 over the whole K:
//   y[c][r] = sum_k f16(dsc_g(k) * q_k) * f16(yd * q8_k)                      (main)
//           + sum_g A'_g(r) * f16(yd * bsum16_g)                               (per group)
// with dsc_g = f16(d * sc_g), A' = -f16(dmin * m_j) (Q4_K/Q5_K mins, one per 16-element
// half of sub-block j) or -32 * dsc_g (Q6_K's q - 32 offset). Every weight operand is one
// rounding of an exact product (v_pk_fma_f16 of the magic-exponent quant 1024 + q with
// dsc and the exact -1024 * dsc), every activation operand one rounding of the reference's
// own d * q. Tolerance (tests/test_gpu_mmf.py): |y - y_ref| <= 2^-8 * sum_k |w_k| |x^_k|
// + 2^-24 * K * max|w| max|x^| (w, x^ the dequantized operands; mmf_bound of the tests' numpy checker), y_ref the oracle's
// bit-exact mul_mat.
//
// Tiles: a workgroup of 4 waves owns 128 weight rows (32 per wave: the MFMA's columns)
// x 128 activation columns (4 MFMA tiles of 32 per wave, fed by ONE dequantized weight
// fragment). K runs in half-superblock steps: the activation image half (128 x 256 B)
// and the d*bsum16 block (128 x 32 B) arrive by LDS-DMA into one of two 36-KB buffers
// (two workgroups per CU), one barrier per step; the weight bytes of superblock b+1 are
// loaded into registers while b is computed. Weight fragments are built in registers
// (each weight byte is read by one wave only), so only the activation goes through LDS.
#include "kq_device.h"

// Pin the one-step-ahead activation reads with a scheduling barrier (hipcc otherwise
// moves each read next to its MFMA).
// Timing-only ablations (experiment builds, make variant-mmf NAME=d1 VFLAGS=-DKQ_MMF_DIAG=1):
// 1 no activation refill after the first step, 8 no workgroup barrier (round 3, RR = 1:
// the 8B ffn_up 79 -> 69 us without the refill, 66 us without both).
#ifndef KQ_MMF_DIAG
#define KQ_MMF_DIAG 0
#endif
#ifndef KQ_MMF_PIN
#define KQ_MMF_PIN 1
#endif

namespace kq {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

__device__ __forceinline__ h2v as_h2(uint32_t v) {
    h2v r;
    __builtin_memcpy(&r, &v, 4);
    return r;
}

constexpr uint32_t MAGIC = 0x64646464u;  // f16 exponent byte of 1024: 0x64xx = 1024 + xx

// (1024 + byte k of w) in both f16 lanes
__device__ __forceinline__ h2v magic_bcast(uint32_t w, int k) {
    return as_h2(__builtin_amdgcn_perm(MAGIC, w, 0x04000400u + 0x00010001u * (uint32_t)k));
}

// f16(v) in both lanes of a pair
__device__ __forceinline__ h2v h2_bcast(_Float16 v) { return h2v{v, v}; }

// Per-superblock register image of a lane's weight bytes (lane half h). Q4_K: v0 header,
// v1..v4 qs bytes [32p + 16h, +16); Q5_K: v0 header, v1 qh bytes [16h, +16), v2..v5 qs;
// Q6_K: v0..v3 ql bytes [64n + 32g + 16h, +16) (index 2n + g), v4/v5 qh bytes
// [32n + 16h, +16), v6 the 16 int8 scales, e the f16 d.
struct MmfW {
    u32x4 v[7];
    uint32_t e;
};

template <int TYPE>
__device__ __forceinline__ void mmf_load(MmfW &w, const uint8_t *blk, int h) {
    if (TYPE == Q4_K) {
        w.v[0] = *(const u32x4 *)blk;
#pragma unroll
        for (int p = 0; p < 4; ++p) w.v[1 + p] = *(const u32x4 *)(blk + 16 + 32 * p + 16 * h);
    } else if (TYPE == Q5_K) {
        w.v[0] = *(const u32x4 *)blk;
        w.v[1] = *(const u32x4 *)(blk + 16 + 16 * h);
#pragma unroll
        for (int p = 0; p < 4; ++p) w.v[2 + p] = *(const u32x4 *)(blk + 48 + 32 * p + 16 * h);
    } else {  // Q6_K: 210-B blocks, any alignment (unaligned vector loads)
#pragma unroll
        for (int i = 0; i < 4; ++i) __builtin_memcpy(&w.v[i], blk + 64 * (i >> 1) + 32 * (i & 1) + 16 * h, 16);
#pragma unroll
        for (int n = 0; n < 2; ++n) __builtin_memcpy(&w.v[4 + n], blk + 128 + 32 * n + 16 * h, 16);
        __builtin_memcpy(&w.v[6], blk + 192, 16);
        uint16_t d;
        __builtin_memcpy(&d, blk + 208, 2);
        w.e = d;
    }
}

// Per-superblock scale operands: DSC/NB pairs of the two 32-element halves each step
// uses (Q4_K/Q5_K: sub-blocks 2p, 2p+1; Q6_K: groups 4p+h, 4p+2+h), and the group
// operand of the per-group MFMA (k' = 8h + j <-> group 8h + j).
struct MmfS {
    h2v dlo[4], dhi[4], nlo[4], nhi[4];
    f16x8 wg;
};

template <int TYPE>
__device__ __forceinline__ MmfS mmf_setup(const MmfW &w, int h) {
    MmfS s;
    if (TYPE == Q4_K || TYPE == Q5_K) {
        const u32x4 hdr = w.v[0];
        const uint32_t s03 = hdr.y & 0x3f3f3f3fu;
        const uint32_t m03 = hdr.z & 0x3f3f3f3fu;
        const uint32_t s47 = (hdr.w & 0x0f0f0f0fu) | ((hdr.y >> 2) & 0x30303030u);
        const uint32_t m47 = ((hdr.w >> 4) & 0x0f0f0f0fu) | ((hdr.z >> 2) & 0x30303030u);
        const h2v d2 = as_h2((hdr.x & 0xffffu) * 0x00010001u);
        const h2v dm2 = as_h2((hdr.x >> 16) * 0x00010001u);
        const h2v k1024 = {(_Float16)1024.0f, (_Float16)1024.0f}, km1024 = {(_Float16)-1024.0f, (_Float16)-1024.0f};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t sw = p < 2 ? s03 : s47;
            // f16(d * sc): the magic pair minus 1024 is sc exactly, one rounding in the multiply
            s.dlo[p] = (magic_bcast(sw, 2 * (p & 1)) - k1024) * d2;
            s.dhi[p] = (magic_bcast(sw, 2 * (p & 1) + 1) - k1024) * d2;
            s.nlo[p] = s.dlo[p] * km1024;  // exact
            s.nhi[p] = s.dhi[p] * km1024;
        }
        const uint32_t mw = h ? m47 : m03;  // sub-blocks 4h .. 4h+3
        const h2v ndm2 = -dm2;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const h2v m = (magic_bcast(mw, k) - k1024) * ndm2;  // -f16(dmin * m), both halves of sub-block 4h+k
            s.wg[2 * k] = m[0];
            s.wg[2 * k + 1] = m[1];
        }
    } else {
        const float d = h2f(w.e);
        const u32x4 sc = w.v[6];
        auto dsc = [&](int g) {  // f16(d * sc_g): exact f32 product, one rounding
            const int sv = (int)(int8_t)((sc[g >> 2] >> (8u * (uint32_t)(g & 3))) & 0xffu);
            return (_Float16)(d * (float)sv);
        };
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const _Float16 a = dsc(4 * p + h), b = dsc(4 * p + 2 + h);
            s.dlo[p] = h2_bcast(a);
            s.dhi[p] = h2_bcast(b);
            s.nlo[p] = h2_bcast(a * (_Float16)-1024.0f);
            s.nhi[p] = h2_bcast(b * (_Float16)-1024.0f);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s.wg[j] = dsc(8 * h + j) * (_Float16)-32.0f;  // exact
    }
    return s;
}

// Weight fragment of step (p, t): k-slot j of lane half h is element
// 64p + 32(j>>2) + 16h + 4t + (j&3) of the superblock.
template <int TYPE>
__device__ __forceinline__ f16x8 mmf_frag(const MmfW &w, const MmfS &s, int p, int t) {
    uint32_t lo, hi;
    if (TYPE == Q4_K) {
        const uint32_t q = w.v[1 + p][t];
        lo = q & 0x0f0f0f0fu;
        hi = (q >> 4) & 0x0f0f0f0fu;
    } else if (TYPE == Q5_K) {
        const uint32_t q = w.v[2 + p][t], qh = w.v[1][t];
        lo = (q & 0x0f0f0f0fu) | (((qh >> (uint32_t)(2 * p)) & 0x01010101u) << 4);
        hi = ((q >> 4) & 0x0f0f0f0fu) | (((qh >> (uint32_t)(2 * p + 1)) & 0x01010101u) << 4);
    } else {
        const int n = p >> 1;
        const uint32_t sh = 4u * (uint32_t)(p & 1);
        const uint32_t l0 = w.v[2 * n][t], l1 = w.v[2 * n + 1][t], qh = w.v[4 + n][t];
        lo = ((l0 >> sh) & 0x0f0f0f0fu) | (((qh >> sh) & 0x03030303u) << 4);
        hi = ((l1 >> sh) & 0x0f0f0f0fu) | (((qh >> (sh + 2u)) & 0x03030303u) << 4);
    }
    const h2v a0 = __builtin_elementwise_fma(as_h2(__builtin_amdgcn_perm(MAGIC, lo, 0x04010400u)), s.dlo[p], s.nlo[p]);
    const h2v a1 = __builtin_elementwise_fma(as_h2(__builtin_amdgcn_perm(MAGIC, lo, 0x04030402u)), s.dlo[p], s.nlo[p]);
    const h2v a2 = __builtin_elementwise_fma(as_h2(__builtin_amdgcn_perm(MAGIC, hi, 0x04010400u)), s.dhi[p], s.nhi[p]);
    const h2v a3 = __builtin_elementwise_fma(as_h2(__builtin_amdgcn_perm(MAGIC, hi, 0x04030402u)), s.dhi[p], s.nhi[p]);
    return f16x8{a0[0], a0[1], a1[0], a1[1], a2[0], a2[1], a3[0], a3[1]};
}

}  // namespace

// ------------------------------------------------------------------ activation image
// One wave per superblock: quantize_row_q8_K_ref (the exact values of kq_quantize_q8K),
// then f16(d * q) of lane l's elements 4l .. 4l+3 at k-slots 4*jhi .. 4*jhi+3 of chunk
// 2*(4p + t) + h (l = 16p + 8jhi + 4h + t), and f16(d * bsum16_g) of group g = l/4.
__global__ void __launch_bounds__(WG_THREADS) kq_quantize_f16img(const float *__restrict__ x, int64_t x_stride,
                                                                 uint8_t *__restrict__ img, uint8_t *__restrict__ bs,
                                                                 int nb, int64_t nblocks) {
    const int lane = threadIdx.x & 63;
    const int64_t bi = (int64_t)blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6);
    if (bi >= nblocks) return;
    const int64_t row = bi / nb;
    const int b = (int)(bi - row * nb);
    const Q8Lane q = quant_block_wave(x + row * x_stride + (int64_t)b * QK, lane);
    h2v v01, v23;
    v01[0] = (_Float16)(q.d * (float)(int8_t)(q.qs4 & 0xffu));
    v01[1] = (_Float16)(q.d * (float)(int8_t)((q.qs4 >> 8) & 0xffu));
    v23[0] = (_Float16)(q.d * (float)(int8_t)((q.qs4 >> 16) & 0xffu));
    v23[1] = (_Float16)(q.d * (float)(int8_t)(q.qs4 >> 24));
    const int p = lane >> 4, jhi = (lane >> 3) & 1, h = (lane >> 2) & 1, t = lane & 3;
    uint2 o;
    __builtin_memcpy(&o.x, &v01, 4);
    __builtin_memcpy(&o.y, &v23, 4);
    *(uint2 *)(img + bi * MMF_IMG + (2 * (4 * p + t) + h) * 16 + 8 * jhi) = o;
    if ((lane & 3) == 0) {
        const _Float16 s = (_Float16)(q.d * (float)q.bsum);
        *(_Float16 *)(bs + bi * MMF_BSB + 2 * (lane >> 2)) = s;
    }
}

// ------------------------------------------------------------------ GEMM
// NW waves of 32 weight rows each: NW = 4 (128 rows per workgroup, two workgroups per CU)
// or NW = 8 (256 rows, one workgroup per CU: the activation tile's LDS-DMA shared by twice
// the rows). Round 3 also measured two row tiles per wave (256 rows on 4 waves, one wave
// per SIMD, accumulators in AGPRs): equal on 8B ffn_down, 3-18 % slower elsewhere
// (profiles/r03_mmf_rr_ab.txt); removed.
template <int TYPE, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) kq_mmf(const MmfArgs a) {
    constexpr int RR = 1;
    constexpr int HALF = MMF_COLS * MMF_IMG / 2;  // 32 KB of image per step
    constexpr int RT = 32 * NW;                   // weight rows per workgroup
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, h = lane >> 5;

    // XCD-aware order (speed only): blocks L, L+8, ... share an XCD and get consecutive
    // tiles T (bijective for any grid size). order 0: the row tiles of one column tile
    // and K split are consecutive, so an XCD's L2 holds ~one column tile's activation
    // image (K x 128 x 2 B) and the weights stream past it; order 1: the column tiles of
    // one row tile (the weight bytes shared in L2). Measured equal (round 3).
    const int G = gridDim.x, L = blockIdx.x;
    const int q8 = G >> 3, r8 = G & 7, xcd = L & 7;
    const int T = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
    int tx, ty, kz;
    if (a.order == 0) {
        ty = T % a.n_rt;
        const int rest = T / a.n_rt;
        kz = rest % a.n_split;
        tx = rest / a.n_split;
    } else {
        tx = T % a.n_ct;
        const int rest = T / a.n_ct;
        kz = rest % a.n_split;
        ty = rest / a.n_split;
    }
    // several matrices on one activation: this row tile's matrix (slab columns from roff)
    const uint8_t *wmat = a.w;
    int64_t wstride = a.row_stride;
    int n_rows = a.n_rows, roff = 0;
    float *y = a.y;
    int64_t ycs = a.y_col_stride;
    if (a.n_mat > 1) {
        int t0 = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)  // selects, no dynamic index into the kernel arguments (scratch)
            if (k < a.n_mat && ty >= a.tile0[k]) {
                wmat = a.mw[k];
                wstride = a.mrow_stride[k];
                n_rows = a.mn_rows[k];
                roff = a.roff[k];
                y = a.my[k];
                ycs = a.my_col_stride[k];
                t0 = a.tile0[k];
            }
        ty -= t0;
    }
    const int col0 = tx * MMF_COLS, row0 = ty * RT;
    const int b0 = kz * a.nbs;
    const int b1 = b0 + a.nbs < a.nb ? b0 + a.nbs : a.nb;
    const int nst = 2 * (b1 - b0);
    const int64_t icol = (int64_t)a.nb * MMF_IMG, bcol = (int64_t)a.nb * MMF_BSB;

    // DMA of step st (superblock b0 + st/2, half st&1): 32 image instructions (4 columns
    // x 16 chunks each, chunk q of column c at slot q ^ (c & 15): conflict-free
    // ds_read_b128) and, on the first half, 4 of d*bsum16 (waves 0-3) -- 32/NW (+1) per wave.
    auto issue = [&](int st) {
        uint8_t *buf = smem + (st & 1) * MMF_BUF;
        const int b = b0 + (st >> 1), hf = st & 1;
#pragma unroll
        for (int i = 0; i < 32 / NW; ++i) {
            const int inst = (32 / NW) * wave + i;
            const int c = 4 * inst + (lane >> 4), slot = lane & 15;
            const int cc = col0 + c < a.m_cols ? col0 + c : a.m_cols - 1;
            const uint8_t *src = a.img + cc * icol + (int64_t)b * MMF_IMG + hf * (MMF_IMG / 2) + 16 * (slot ^ (c & 15));
            dma16(src, (LDS void *)(buf + 1024 * inst));
        }
        if (!hf && wave < 4) {
            const int c = 32 * wave + (lane >> 1);
            const int cc = col0 + c < a.m_cols ? col0 + c : a.m_cols - 1;
            dma16(a.bs + cc * bcol + (int64_t)b * MMF_BSB + 16 * (lane & 1), (LDS void *)(buf + HALF + 1024 * wave));
        }
    };

    const uint8_t *wp[RR];
#pragma unroll
    for (int rr = 0; rr < RR; ++rr) {
        int wrow = row0 + 32 * (RR * wave + rr) + r;
        wrow = wrow < n_rows ? wrow : n_rows - 1;
        wp[rr] = wmat + (int64_t)wrow * wstride;
    }
    constexpr int BSZ = block_bytes(TYPE);

    f32x16 acc[RR][4];
#pragma unroll
    for (int rr = 0; rr < RR; ++rr)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[rr][ct][i] = 0.f;

    MmfW wc[RR], wn[RR];
#pragma unroll
    for (int rr = 0; rr < RR; ++rr) mmf_load<TYPE>(wc[rr], wp[rr] + (int64_t)b0 * BSZ, h);
    issue(0);
#pragma unroll 1
    for (int b = b0; b < b1; ++b) {
        MmfS s[RR];
#pragma unroll
        for (int rr = 0; rr < RR; ++rr) s[rr] = mmf_setup<TYPE>(wc[rr], h);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int st = 2 * (b - b0) + hf;
            // step st landed (the only DMA in flight); after the barrier every wave has
            // finished reading the other buffer (lgkmcnt(0) before it), which st+1 refills
            // (the builtin wait, not inline asm: hipcc's waitcnt pass then knows the weight
            // loads of the previous superblock have landed and inserts no counted wait of
            // its own -- one that, blind to the LDS-DMA, would stall on the refill below)
            __builtin_amdgcn_s_waitcnt(0);
            if (!(KQ_MMF_DIAG & 8)) asm volatile("s_barrier" ::: "memory");
            if (st + 1 < nst && !((KQ_MMF_DIAG & 1) && st > 0)) issue(st + 1);
            if (hf == 0 && b + 1 < b1)
#pragma unroll
                for (int rr = 0; rr < RR; ++rr) mmf_load<TYPE>(wn[rr], wp[rr] + (int64_t)(b + 1) * BSZ, h);
            const uint8_t *buf = smem + (st & 1) * MMF_BUF;
            if (hf == 0) {  // per-group term: mins (Q4_K/Q5_K) or the -32 offset (Q6_K)
#pragma unroll
                for (int ct = 0; ct < 4; ++ct) {
                    const f16x8 ab = *(const f16x8 *)(buf + HALF + (32 * ct + r) * MMF_BSB + 16 * h);
#pragma unroll
                    for (int rr = 0; rr < RR; ++rr)
                        acc[rr][ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab, s[rr].wg, acc[rr][ct], 0, 0, 0);
                }
            }
            // activation fragments one step ahead of their MFMAs (the LDS latency of step
            // sl+1's four reads runs under step sl's MFMAs)
            auto act = [&](f16x8 *av, int sl) {
                const int slot = (2 * sl + h) ^ (r & 15);
#pragma unroll
                for (int ct = 0; ct < 4; ++ct) av[ct] = *(const f16x8 *)(buf + (32 * ct + r) * (MMF_IMG / 2) + 16 * slot);
            };
            f16x8 av[2][4];
            act(av[0], 0);
#pragma unroll
            for (int sl = 0; sl < 8; ++sl) {
                if (sl < 7) act(av[(sl + 1) & 1], sl + 1);
                if (KQ_MMF_PIN) __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead
#pragma unroll
                for (int rr = 0; rr < RR; ++rr) {
                    const f16x8 wf = mmf_frag<TYPE>(wc[rr], s[rr], 2 * hf + (sl >> 2), sl & 3);
#pragma unroll
                    for (int ct = 0; ct < 4; ++ct)
                        acc[rr][ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[sl & 1][ct], wf, acc[rr][ct], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int rr = 0; rr < RR; ++rr) wc[rr] = wn[rr];
    }

    // ---- store: lane's weight row, accumulator element i = column (i&3) + 8(i>>2) + 4h
    float *dst = a.n_split > 1 ? a.slab + (int64_t)kz * a.m_cols * a.n_rows + roff : y;
    const int64_t cs = a.n_split > 1 ? (int64_t)a.n_rows : ycs;
#pragma unroll
    for (int rr = 0; rr < RR; ++rr) {
        const int n = row0 + 32 * (RR * wave + rr) + r;
        if (n >= n_rows) continue;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int c = col0 + 32 * ct + (i & 3) + 8 * (i >> 2) + 4 * h;
                if (c < a.m_cols)
                    dst[(int64_t)c * cs + n] = a.res && a.n_split == 1
                                                   ? acc[rr][ct][i] + a.res[(int64_t)c * a.res_col_stride + n]
                                                   : acc[rr][ct][i];
            }
    }
}

// Split-K combine: y = sum of the n_split partial slabs, in split order (+ res). The slab
// holds n_split planes of m_cols x slab_rows; this matrix is its columns [0, n_rows) from
// `slab` on.
__global__ void __launch_bounds__(256) kq_mmf_reduce(const float *__restrict__ slab, int n_split, int m_cols,
                                                     int n_rows, int slab_rows, float *__restrict__ y,
                                                     int64_t y_col_stride, const float *__restrict__ res,
                                                     int64_t res_col_stride) {
    const int64_t total = (int64_t)m_cols * n_rows, plane = (int64_t)m_cols * slab_rows;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int64_t c = i / n_rows, n = i - c * n_rows;
    const float *p = slab + c * slab_rows + n;
    float s = p[0];
    for (int k = 1; k < n_split; ++k) s += p[(int64_t)k * plane];
    y[c * y_col_stride + n] = res ? s + res[c * res_col_stride + n] : s;
}

template __global__ void kq_mmf<Q4_K, 4>(const MmfArgs a);
template __global__ void kq_mmf<Q5_K, 4>(const MmfArgs a);
template __global__ void kq_mmf<Q6_K, 4>(const MmfArgs a);
template __global__ void kq_mmf<Q4_K, 8>(const MmfArgs a);
template __global__ void kq_mmf<Q5_K, 8>(const MmfArgs a);
template __global__ void kq_mmf<Q6_K, 8>(const MmfArgs a);

}  // namespace kq
