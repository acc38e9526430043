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
#include <hip/hip_ext.h>

#include "kq_internal.h"
#include "kq_ops_device.h"
#include "kq_rows_device.h"

// Diagnostics (timing only: MI355X_GEMV_DIAG bits, per-wave s_memrealtime stamps) exist
// only in experiment builds: make variant NAME=rdiag VFLAGS=-DKQ_ROWS_DIAG=1. In the
// product build RDIAG / RSTAMPS are constants and every diagnostic branch compiles out
// (run-time diag branches cost kq_mmq 40 VGPRs).
#ifndef KQ_ROWS_DIAG
#define KQ_ROWS_DIAG 0
#endif
#if KQ_ROWS_DIAG
#define RDIAG(a) ((a).diag)
#define RSTAMPS(a) ((a).stamps)
#else
#define RDIAG(a) 0
#define RSTAMPS(a) ((uint64_t *)nullptr)
#endif

#ifndef KQ_ROWS_XMODE
#define KQ_ROWS_XMODE 0  // fused-quantization prologue (ROWS_X_* bits); -1: a.xmode at run time
#endif
// Weight steps issued before the activation wait, and the L2 prefetch touches past the
// ring: compile-time (-1: from RowsArgs at run time, the experiment knobs
// MI355X_GEMV_PRE0 / MI355X_GEMV_PF). Constants make every s_waitcnt that covers an
// inline-asm activation load a constant on each path, which tools/vmem_lint.py checks.
#ifndef KQ_ROWS_PRE0
#define KQ_ROWS_PRE0 1
#endif
#ifndef KQ_ROWS_L2PF
#define KQ_ROWS_L2PF 0
#endif
// Prologue DMA and activation wait (profiles/r03_masked_ab.txt): 2 (product) issues the
// step's partial last DMA instruction with its lane mask inside the asm, so it is issued on
// every path, and the activation wait then leaves the residual load (younger than x, a
// gather from memory the previous launches did not touch) in flight: TinyLlama token +4.8 %,
// Llama-3-8B +3.1 %. 1: the masked DMA with the old wait; 0: both as before (experiments).
#ifndef KQ_ROWS_MASKED
#define KQ_ROWS_MASKED 2
#endif
#ifndef KQ_ROWS_LINT_BREAK
#define KQ_ROWS_LINT_BREAK 0  // 1: drop the activation wait (a lint self-test build, never run)
#endif

// The GEMV's outputs (and the SWIGLU epilogue's) are stored write-through (sc1), so the next
// launch's activation is in the memory-side caches before the kernel boundary
// (tools/xfresh.hip: the consumer's fresh-read price 0.15 -> 0.03 us per edge).
// Issue priority by remaining work (MI355X_MICROARCH.md "Two waves per SIMD": VALU and memory
// issue go by priority, then age, so with three waves per SIMD the older ones stream faster
// and the middle one ends last, r05 stamps): every few steps a wave sets s_setprio from the
// weight bytes it still has to stream, relative to the most any wave streams, so the waves
// behind catch up.
#ifndef KQ_ROWS_PRIO
#define KQ_ROWS_PRIO 0
#endif

#ifndef KQ_ROWS_YSC1
#define KQ_ROWS_YSC1 1  // TinyLlama token +0.5-1.4 %, Llama-3-8B +0.7 % (profiles/r04_store_flavour_ab.txt)
#endif

namespace kq {

__device__ __forceinline__ void store_y(float *p, float v) {
    if (KQ_ROWS_YSC1) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else *p = v;
}

// Q8L quantization of whole rows (K > 8192 path): 16 superblocks per workgroup.
// AM: the prefill GEMMs' layout (quant16_store<true>: the mins operand in place of bsums).
template <bool AM>
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
    quant16_store<AM>(v, lane & 15, y + bi * Q8L_STRIDE);
}
template __global__ void kq_quantize_q8L<false>(const float *, int64_t, uint8_t *, int, int64_t);
template __global__ void kq_quantize_q8L<true>(const float *, int64_t, uint8_t *, int, int64_t);

// ------------------------------------------------------------ prefill prologues
// The prompt graph's RMS_NORM -> MUL(norm weight) -> MUL_MATs and SWIGLU -> MUL_MAT:
// the op's arithmetic exactly as kq_rms_norm / kq_swiglu compute it (same sum order and
// exactness guard, (x*scale)*w; silu(g)*u on the NEON path), quantized straight into the
// GEMMs' Q8L blocks (row r's superblock b at (r*nb + b)*304); the f32 intermediate is
// never written.
__global__ void __launch_bounds__(256) kq_rms_norm_q8L(const float *__restrict__ x, const float *__restrict__ w,
                                                       uint8_t *__restrict__ yq, int64_t n, float eps) {
    extern __shared__ __attribute__((aligned(16))) double sb_sum[];
    const int64_t row = blockIdx.x;
    const float *xr = x + row * n;
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
    if (rms_mean_ambiguous(div_by_count(total, n), n)) {  // ggml's sequential order (block-uniform)
        __syncthreads();
        if (threadIdx.x < 64) {
            const double s = seq_sumsq_wave(xr, n, threadIdx.x);
            if (threadIdx.x == 0) sb_sum[0] = s;
        }
        __syncthreads();
        total = sb_sum[0];
    }
    const float mean = (float)div_by_count(total, n);
    const float scale = 1.0f / sqrtf(mean + eps);
    for (int b0 = 0; b0 < nb; b0 += 16) {
        const int b = b0 + rid;  // uniform over the 16-lane row: quant16_store's DPP row
        if (b >= nb) continue;
        const float4 *p = (const float4 *)(xr + (int64_t)b * QK + 16 * l);
        const float4 *q = (const float4 *)(w + (int64_t)b * QK + 16 * l);
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 t = p[k], m = q[k];
            v[k].x = __float_as_uint((t.x * scale) * m.x);
            v[k].y = __float_as_uint((t.y * scale) * m.y);
            v[k].z = __float_as_uint((t.z * scale) * m.z);
            v[k].w = __float_as_uint((t.w * scale) * m.w);
        }
        quant16_store<true>(v, l, yq + (row * nb + b) * Q8L_STRIDE);  // (prefill only: Q8L/mmq)
    }
}

__global__ void __launch_bounds__(256) kq_swiglu_q8L(const float *__restrict__ g, const float *__restrict__ u,
                                                     uint8_t *__restrict__ yq, int nb, int64_t nblocks) {
    const int64_t bi = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);  // superblock (row * nb + b)
    if (bi >= nblocks) return;  // whole 16-lane rows drop out together
    const int l = threadIdx.x & 15;
    const int64_t e0 = bi * QK + 16 * l;  // rows are contiguous: element index = superblock * 256 + ...
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 gv = *(const float4 *)(g + e0 + 4 * k), uv = *(const float4 *)(u + e0 + 4 * k);
        v[k].x = __float_as_uint(v_silu(gv.x) * uv.x);
        v[k].y = __float_as_uint(v_silu(gv.y) * uv.y);
        v[k].z = __float_as_uint(v_silu(gv.z) * uv.z);
        v[k].w = __float_as_uint(v_silu(gv.w) * uv.w);
    }
    (void)nb;
    quant16_store<true>(v, l, yq + bi * Q8L_STRIDE);  // (prefill only: Q8L/mmq)
}

int launch_rms_norm_q8L(const float *x, const float *w, void *yq, int64_t n, int64_t nrows, float eps, hipStream_t s) {
    if (nrows == 0) return MI355X_OK;
    hipEvent_t e0, e1;
    const size_t lds = (size_t)(n / QK) * 8 + 8;
    if (timing_slot(s, e0, e1)) {
        hipExtLaunchKernelGGL(kq_rms_norm_q8L, dim3((unsigned)nrows), dim3(256), (uint32_t)lds, s, e0, e1, 0, x, w,
                              (uint8_t *)yq, n, eps);
        timing_log("kq::kq_rms_norm_q8L", (double)nrows * (n * 4.0 + (n / QK) * (double)Q8L_STRIDE) + n * 4.0, e0, e1);
    } else {
        hipLaunchKernelGGL(kq_rms_norm_q8L, dim3((unsigned)nrows), dim3(256), lds, s, x, w, (uint8_t *)yq, n, eps);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

int launch_swiglu_q8L(const float *g, const float *u, void *yq, int64_t n, int64_t nrows, hipStream_t s) {
    const int64_t nb = n / QK, nblocks = nb * nrows;
    if (nblocks == 0) return MI355X_OK;
    const int64_t wgs = (nblocks + 15) / 16;
    hipEvent_t e0, e1;
    if (timing_slot(s, e0, e1)) {
        hipExtLaunchKernelGGL(kq_swiglu_q8L, dim3((unsigned)wgs), dim3(256), 0, s, e0, e1, 0, g, u, (uint8_t *)yq,
                              (int)nb, nblocks);
        timing_log("kq::kq_swiglu_q8L", (double)nblocks * (QK * 8.0 + Q8L_STRIDE), e0, e1);
    } else {
        hipLaunchKernelGGL(kq_swiglu_q8L, dim3((unsigned)wgs), dim3(256), 0, s, g, u, (uint8_t *)yq, (int)nb, nblocks);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

template <int TYPE, bool FUSEDQ, int PRO>
__device__ __forceinline__ void rows_body(const RowsArgs &a, const WaveWork &ww, uint8_t *smem, const RowsLayout &L,
                                          int wave, int lane, uint64_t st0) {
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int GRAN = rows_gran(TYPE);
    constexpr int NI = rows_ni(TYPE);
    constexpr int SLOT = rows_slot(TYPE);
    constexpr int D = rows_depth(TYPE);
    static_assert(D >= 2 && D <= 4, "vm_wait_k covers 3 steps in flight");
    const int nb = a.nb, bR = a.bR;
    const int nwv = __builtin_amdgcn_readfirstlane((int)(blockDim.x >> 6));  // waves in this workgroup
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

    // L2 prefetch (uniform per wave): only streams longer than the ring, fused path
    const bool pf_on = FUSEDQ && (KQ_ROWS_L2PF < 0 ? a.pf != 0 : KQ_ROWS_L2PF != 0) && T > D + 1;
    uint32_t pf_sink = 0;
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

    const float *const res_p = a.res[ww.m];
    uint32_t rv = 0;  // residual of the fused ADD for row r0 + lane (first 64 rows)

    // ---- prologue: activation loads, pre0 weight steps, quantize, then the rest of the ring
    const int pre_req = KQ_ROWS_PRE0 < 0 ? a.pre0 : KQ_ROWS_PRE0;
    const int pre_cap = pre_req < D ? pre_req : D;  // never more than the ring holds
    // min(T, pre_cap) written so that the compiler sees 0 <= pre0 <= pre_cap (T >= 0)
    const int pre0 = T >= pre_cap ? pre_cap : (T > 0 ? T : 0);
    uint64_t sx = 0, sq = 0, sf = 0;  // diagnostics: x landed, quantized, first step computed
    if (FUSEDQ) {
        const int PASS = 4 * nwv;  // superblocks per workgroup pass
        // KQ_ROWS_XMODE >= 0: the prologue fixed at compile time (experiment builds)
        const int xm = KQ_ROWS_XMODE >= 0 ? KQ_ROWS_XMODE : a.xmode;
        u32x4 xv[ROWS_QPASS][4] = {};
        u32x4 x2v[ROWS_QPASS][4] = {};  // norm weight / up, same elements as xv
        const int qiters = (nb + PASS - 1) / PASS;
        // passes this wave loads (wave-uniform): pass i while slot 4*wave of it lies in the row
        int qw = 0;
#pragma unroll
        for (int i = 0; i < ROWS_QPASS; ++i) qw += (i < qiters && PASS * i + 4 * wave < nb) ? 1 : 0;
        // slot j of the passes -> superblock: rotated by the workgroup (ROWS_X_ROT) so the
        // grid does not read the activation's lines in one order; slots past the row read
        // superblock nb-1's place and store nothing
        const int rot = (xm & ROWS_X_ROT) ? (int)(blockIdx.x % (unsigned)nb) : 0;
        auto sbk = [&](int j) {
            int b = (j < nb ? j : nb - 1) + rot;
            return b >= nb ? b - nb : b;
        };
        constexpr int pro = PRO;
        constexpr int PL = PRO != ROWS_PRO_NONE ? 8 : 4;  // loads per pass
#pragma unroll
        for (int i = 0; i < ROWS_QPASS; ++i) {
            if (i < qw) {  // waves past the row load nothing
                const int b = sbk(PASS * i + 4 * wave + (lane >> 4));
                const float *xp = a.x + (int64_t)b * QK + 16 * (lane & 15);
#pragma unroll
                for (int k = 0; k < 4; ++k) xv[i][k] = gload16_asm(xp + 4 * k);
                if (PRO != ROWS_PRO_NONE) {  // (diag bit 4: read x again instead of x2, timing only)
                    const float *x2p = ((RDIAG(a) & 16) ? a.x : a.x2) + (int64_t)b * QK + 16 * (lane & 15);
#pragma unroll
                    for (int k = 0; k < 4; ++k) x2v[i][k] = gload16_asm(x2p + 4 * k);
                }
            }
        }
        // residual of the fused ADD: one row per lane, fetched with the activation. Issued
        // on every path (a dummy read of x without a residual) so that no branch joins a
        // register whose asm load is still in flight; rv stays live until the flush waits
        // for it (the res_p branch is a run-time condition). An asm load whose register the
        // compiler sees dead is reused while the load is in flight: a build with that branch
        // compiled out faulted (profiles/r02_attn_epilogue_rejected.md).
        rv = gload4_asm(res_p && ww.nrows > 0 ? res_p + ww.r0 + (lane < ww.nrows ? lane : 0) : a.x);
        // ROWS_X_BAR: every wave's activation requests are queued before any weight DMA of
        // the workgroup (uniform: every wave of the workgroup runs the prologue)
        if (xm & ROWS_X_BAR) asm volatile("s_barrier" ::: "memory");
        // The product build (one step ahead, no prefetch touches) issues exactly one step's
        // DMA instructions on every path: a wave without rows (T == 0) issues them from the
        // activation (valid memory, into a ring slot it never reads), so the one constant
        // wait below covers the activation loads on every path (tools/vmem_lint.py).
        constexpr bool kConstPre = KQ_ROWS_PRE0 == 1 && KQ_ROWS_L2PF == 0;
        if (kConstPre && T == 0) {
            const uint8_t *xb = (const uint8_t *)a.x + 16 * lane;
#pragma unroll
            for (int i = 0; i < NI; ++i)
                if (KQ_ROWS_MASKED && i + 1 == NI) dma16_nt_lanes(xb, (LDS void *)(islot + 1024 * i), lane, GRAN - 64 * (NI - 1));
                else if (i + 1 < NI || lane < GRAN - 64 * (NI - 1)) dma16_nt(xb, (LDS void *)(islot + 1024 * i));
        }
        if (KQ_ROWS_MASKED && kConstPre && T > 0) {  // the one step, its partial DMA masked in asm
            const uint8_t *base = s16 + 16 * lane;
            const uint8_t *lim = T > 1 ? base + 1024 * (NI - 1) : base + 1024 * (NI - 1) < last16 ? base + 1024 * (NI - 1) : last16;
#pragma unroll
            for (int i = 0; i + 1 < NI; ++i) {
                const uint8_t *p = base + 1024 * i;
                dma16_nt(T > 1 || p < last16 ? p : last16, (LDS void *)(islot + 1024 * i));
            }
            dma16_nt_lanes(lim, (LDS void *)(islot + 1024 * (NI - 1)), lane, GRAN - 64 * (NI - 1));
            islot = islot + SLOT == ring_end ? ring : islot + SLOT;
            ++it_;
        } else {
            for (int j = 0; j < pre0; ++j) issue();
        }
        if (pf_on) {  // L2 prefetch of the stream just past the ring (younger than the pre0 steps)
            const uint8_t *p = s16 + (int64_t)D * (ROWS_SB * BSZ) + 64 * lane;
#pragma unroll
            for (int i = 0; i < ROWS_PF; ++i) l2_touch(p + 4096 * i < last16 ? p + 4096 * i : last16, pf_sink);
        }
        // vector-memory operations younger than the last pass's activation loads
        const int tail = 1 + NI * pre0 + (pf_on ? ROWS_PF : 0);
        // the asm loads are invisible to the compiler: pin their registers past each wait
        auto pin = [&]() {
            asm volatile("" : "+v"(xv[0][0]), "+v"(xv[0][1]), "+v"(xv[0][2]), "+v"(xv[0][3]), "+v"(xv[1][0]),
                         "+v"(xv[1][1]), "+v"(xv[1][2]), "+v"(xv[1][3]), "+v"(xv[2][0]), "+v"(xv[2][1]),
                         "+v"(xv[2][2]), "+v"(xv[2][3]));
            if (pro != ROWS_PRO_NONE) {
#pragma unroll
                for (int i = 0; i < ROWS_QPASS; ++i)
#pragma unroll
                    for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(x2v[i][k]));
            }
        };
        if (pro != ROWS_PRO_NORM && (xm & ROWS_X_PIPE)) {
            // pass by pass: pass i's transform + quantization overlap the later passes' loads
#pragma unroll
            for (int i = 0; i < ROWS_QPASS; ++i) {
                if (i < qw) {
                    vm_wait_dyn((qw - 1 - i) * PL + tail);
                    pin();
                    if (pro == ROWS_PRO_SWIGLU && !(RDIAG(a) & 32)) {  // ggml_vec_swiglu_f32: silu(gate) * up
#pragma unroll
                        for (int k = 0; k < 4; ++k) xv[i][k] = swiglu4(xv[i][k], x2v[i][k]);
                    }
                    const int j = PASS * i + 4 * wave + (lane >> 4);
                    if (j < nb && !(RDIAG(a) & 64)) quant16_store(xv[i], lane & 15, smem + L.act + Q8L_STRIDE * sbk(j));
                }
            }
            if (RSTAMPS(a)) sx = sq = __builtin_amdgcn_s_memrealtime();
        } else {
            // every pass landed: all but the pre0 weight steps (and prefetch touches); with
            // compile-time pre0 / prefetch a constant per path
            if (KQ_ROWS_LINT_BREAK) {
                // deliberately broken build (tests/test_abi.py: the ISA lint must flag it): no wait
            } else if (kConstPre && KQ_ROWS_MASKED == 2) {
                // x landed: the residual load (rv, younger than x) and the step's NI DMA
                // instructions (all issued on every path) may still be in flight
                vm_wait<NI + 1>();
            } else if (kConstPre) {
                vm_wait<NI>();  // all but the one step's DMA instructions (fewer if predicated off: a stronger wait)
            } else {
                vm_wait_dyn(tail);
            }
            pin();
            if (RDIAG(a) & 32) {  // diagnostics (timing only): skip the transform
            } else if (pro == ROWS_PRO_SWIGLU) {  // ggml_vec_swiglu_f32: silu(gate) * up
#pragma unroll
                for (int i = 0; i < ROWS_QPASS; ++i)
                    if (i < qw)
#pragma unroll
                        for (int k = 0; k < 4; ++k) xv[i][k] = swiglu4(xv[i][k], x2v[i][k]);
            } else if (pro == ROWS_PRO_NORM) {  // rms_norm then MUL by the norm weight
                double *sums = (double *)(smem + L.sums);
#pragma unroll
                for (int i = 0; i < ROWS_QPASS; ++i) {
                    if (i < qw) {  // wave-uniform: this wave holds x of the pass
                        const int j = PASS * i + 4 * wave + (lane >> 4);
                        double sq = 0.0;
                        if (j < nb) {
                            float v[16];
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                v[4 * k] = __uint_as_float(xv[i][k].x), v[4 * k + 1] = __uint_as_float(xv[i][k].y);
                                v[4 * k + 2] = __uint_as_float(xv[i][k].z), v[4 * k + 3] = __uint_as_float(xv[i][k].w);
                            }
                            sq = sumsq16(v);
                        }
                        sq = row16_sum(sq);  // DPP, every lane of the wave active
                        if (j < nb && (lane & 15) == 0) sums[sbk(j)] = sq;
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                double tot = seq_sum_lanes(sums, nb, lane);  // superblocks in order
                // workgroup-uniform (every wave sums the same LDS values): the rare rows whose
                // float mean could depend on the order are summed in ggml's order (each wave)
                if (rms_mean_ambiguous(div_by_count(tot, (int64_t)nb * QK), (int64_t)nb * QK))
                    tot = seq_sumsq_wave(a.x, (int64_t)nb * QK, lane);
                const float mean = (float)div_by_count(tot, (int64_t)nb * QK);
                const float scale = 1.0f / sqrtf(mean + a.eps);
#pragma unroll
                for (int i = 0; i < ROWS_QPASS; ++i)
                    if (i < qw)
#pragma unroll
                        for (int k = 0; k < 4; ++k) xv[i][k] = normmul4(xv[i][k], x2v[i][k], scale);
            }
            if (RSTAMPS(a)) sx = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
            for (int i = 0; i < qw; ++i) {  // one copy of the quantizer; pick the pass's registers
                u32x4 cur[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = i == 0 ? xv[0][k] : i == 1 ? xv[1][k] : xv[2][k];
                const int j = PASS * i + 4 * wave + (lane >> 4);
                if (j < nb && !(RDIAG(a) & 64)) quant16_store(cur, lane & 15, smem + L.act + Q8L_STRIDE * sbk(j));  // (diag 64: timing only)
            }
            if (RSTAMPS(a)) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                sq = __builtin_amdgcn_s_memrealtime();
            }
        }
    } else {
        const int ng = nb * (Q8L_STRIDE / 16);
        for (int j = wave; 64 * j < ng; j += nwv) {
            const int k = 64 * j + lane;
            if (k < ng) dma16(a.xq + 16 * k, (LDS void *)(smem + L.act + 1024 * j));
        }
        for (int j = 0; j < pre0; ++j) issue();
        vm_wait_k<NI>(pre0);
    }
    while (it_ < D && it_ < T) issue();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // Q8_K row complete (no vmcnt drain)
    const uint64_t st1 = RSTAMPS(a) ? __builtin_amdgcn_s_memrealtime() : 0;

    // ---- main loop
    int io = q, rr = 0;  // quad's (block, row-in-batch) of superblock 16t+q
    while (io >= nb) {
        io -= nb;
        ++rr;
    }
    int bend = bR * nb < G ? bR * nb : G;  // superblock index ending the current batch
    int brow = 0;
    const uint8_t *cslot = ring;
    int prio = -1;
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
        if (KQ_ROWS_PRIO && (t & 3) == 0) {
            const int64_t rem = (int64_t)(T - t) * (ROWS_SB * BSZ);
            int p = (int)(rem * 4 / (a.prio_bytes + 1));
            p = __builtin_amdgcn_readfirstlane(p > 3 ? 3 : p);
            if (p != prio) {
                prio = p;
                if (p == 3) __builtin_amdgcn_s_setprio(3);
                else if (p == 2) __builtin_amdgcn_s_setprio(2);
                else if (p == 1) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }
        }
        if (pf_on && t < pre0) {  // the prefetch touches sit between steps pre0-1 and pre0
            if (T - t >= D) vm_wait<NI * (D - 1) + ROWS_PF>();
            else vm_wait_kp<NI, ROWS_PF>(T - t - 1);
        } else if (T - t >= D) {
            vm_wait<NI * (D - 1)>();  // steady state: D-1 younger steps in flight
        } else {
            vm_wait_k<NI>(T - t - 1);
        }
        if (!(RDIAG(a) & 8) && ROWS_SB * t + q < G) {
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
        if (RSTAMPS(a) && t == 0) sf = __builtin_amdgcn_s_memrealtime();
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
    if (KQ_ROWS_PRIO) __builtin_amdgcn_s_setprio(0);
    const uint64_t st2 = RSTAMPS(a) ? __builtin_amdgcn_s_memrealtime() : 0;
    if (pf_on) {  // every touch has landed (they are older than step pre0): release the register
        asm volatile("" ::"v"(pf_sink));
    }

    // ---- flush staged results (coalesced)
    if (ww.nrows > 0) {
        wave_lds_fence();
        float *y = a.y[ww.m] + ww.r0;
        if (res_p) {  // ggml_add(mul_mat, residual): the same single f32 add per element
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("" : "+v"(rv));
            for (int k = 0; k < ww.nrows; k += 64)
                if (k + lane < ww.nrows)
                    store_y(y + k + lane, outs[k + lane] + (k == 0 ? __uint_as_float(rv) : res_p[ww.r0 + k + lane]));
        } else {
            for (int k = 0; k < ww.nrows; k += 64)
                if (k + lane < ww.nrows) store_y(y + k + lane, outs[k + lane]);
        }
    }
    // ---- SWIGLU epilogue (the GLU node after the gate/up MUL_MATs): up wave and its
    // gate partner own the same rows in this workgroup; both results are staged in LDS.
    // Same arithmetic as kq_swiglu (ggml_vec_swiglu_f32: NEON body, libm tail).
    if (a.epi && !(RDIAG(a) & 128)) {  // uniform over the grid: every wave of the workgroup reaches the barrier (diag 128: timing only)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (ww.m == 1 && ww.nrows > 0) {
            const float *gouts = (const float *)(smem + L.outs + (wave - a.epi_wave_off) * L.outs_stride);
            const int n4 = a.epi_n & ~3;
            for (int k = 0; k < ww.nrows; k += 64)
                if (k + lane < ww.nrows) {
                    const int r = ww.r0 + k + lane;
                    const float gv = gouts[k + lane], uv = outs[k + lane];
                    store_y(a.epi_y + r, r < n4 ? v_silu(gv) * uv : (gv / (1.0f + expf(-gv))) * uv);
                }
        }
    }
    if (RSTAMPS(a)) {
        const int64_t o = ((int64_t)blockIdx.x * ROWS_WAVES + wave) * 8;  // stamp slots sized for the most waves
        if (lane == 0 && o + 7 < a.stamps_cap) {
            RSTAMPS(a)[o] = st0;
            RSTAMPS(a)[o + 1] = st1;
            RSTAMPS(a)[o + 2] = st2;
            RSTAMPS(a)[o + 3] = __builtin_amdgcn_s_memrealtime();
            RSTAMPS(a)[o + 4] = sx;
            RSTAMPS(a)[o + 5] = sq;
            RSTAMPS(a)[o + 6] = sf;
        }
    }
}

template <int TMASK, bool FUSEDQ, int PRO>
__global__ void __launch_bounds__(ROWS_WAVES * 64) kq_rows(const RowsArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (RDIAG(a) & 256) return;  // diagnostics (timing only): empty launch
    const uint64_t st0 = RSTAMPS(a) ? __builtin_amdgcn_s_memrealtime() : 0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const RowsLayout L = rows_layout(a.nb, TMASK, a.bR, a.rpw, __builtin_amdgcn_readfirstlane((int)(blockDim.x >> 6)));

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
        rows_body<Q4_K, FUSEDQ, PRO>(a, ww, smem, L, wave, lane, st0);
    } else if (TMASK == 2) {
        rows_body<Q5_K, FUSEDQ, PRO>(a, ww, smem, L, wave, lane, st0);
    } else if (TMASK == 4) {
        rows_body<Q6_K, FUSEDQ, PRO>(a, ww, smem, L, wave, lane, st0);
    } else {
        const int type = a.type[m];
        if (type == Q6_K) rows_body<Q6_K, FUSEDQ, PRO>(a, ww, smem, L, wave, lane, st0);
        else if (type == Q5_K) rows_body<Q5_K, FUSEDQ, PRO>(a, ww, smem, L, wave, lane, st0);
        else rows_body<Q4_K, FUSEDQ, PRO>(a, ww, smem, L, wave, lane, st0);
    }
}

#define KQ_ROWS_INST(TM, FQ, PR) template __global__ void kq_rows<TM, FQ, PR>(const RowsArgs a);
#define KQ_ROWS_INST_T(TM)        \
    KQ_ROWS_INST(TM, true, 0)     \
    KQ_ROWS_INST(TM, true, 1)     \
    KQ_ROWS_INST(TM, true, 2)     \
    KQ_ROWS_INST(TM, false, 0)
KQ_ROWS_INST_T(1)
KQ_ROWS_INST_T(2)
KQ_ROWS_INST_T(4)
KQ_ROWS_INST_T(7)

// ---------------------------------------------------------------- claimed rows (kq_rows_dyn)
// The static split above gives every wave a fixed share of whole rows; in the large GEMVs the
// last wave to finish sets the launch time, and which one that is follows the wave's age on
// its SIMD (issue goes by priority, then age: profiles/r05_rows_agew.txt), not its row count.
// Here workgroup b owns the rows [b*N/G, (b+1)*N/G) of every matrix and its waves CLAIM units
// of U rows from an LDS counter (MI355X_MICROARCH.md **dequeue**, kept inside the CU: one
// ds_add per unit), a ring depth ahead of their compute: the first P units of each wave are
// assigned statically (the ring fill before the prologue's barrier claims nothing), every
// later one is taken when the wave has issued its previous unit's last step. A unit's rows
// stay whole in one wave, so each row's fp32 chain is still replayed in superblock order by
// one lane (bit-identical to the static split and to ggml_vec_dot_q4_K_q8_K row by row,
// README.md:137). Results go to the workgroup's LDS rows and are stored coalesced, with the
// residual ADD and the SWIGLU epilogue, after one workgroup barrier.
#ifndef KQ_ROWS_DYN_RR
#define KQ_ROWS_DYN_RR 0
#endif
namespace {
static_assert(MI355X_MAX_FUSED == 4, "four matrices at most");
struct DynUnit {
    const uint8_t *src;
    int rows, flat, G, T;
};
}  // namespace

// Every matrix of a kq_rows_dyn launch has the same rows and type (plan_rows), so one
// workgroup row range [r0, r0 + nr) serves them all: unit u is matrix u / nu's rows
// [r0 + (u % nu) U, ...), flat output index m * nr + local row. Records of consecutive
// units go into one batch of bR rows, replayed together (lane r <-> batch row r).
template <int TYPE, bool FUSEDQ, int PRO>
__device__ __forceinline__ void rows_dyn_body(const RowsArgs &a, uint8_t *smem, const RowsDynLayout &L, int wave,
                                              int lane, uint64_t st0) {
    uint64_t sx = 0, sq = 0, sf = 0;  // diagnostics (KQ_ROWS_DIAG builds): x landed, quantized, first step
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int GRAN = rows_gran(TYPE);
    constexpr int NI = rows_ni(TYPE);
    constexpr int SLOT = rows_slot(TYPE);
    constexpr int D = rows_depth(TYPE);
    static_assert(D >= 2 && D <= 4, "vm_wait_k covers 3 steps in flight");
    const int nb = a.nb, U = a.dyn_u, P = a.dyn_p, bR = a.bR;
    const int nwv = __builtin_amdgcn_readfirstlane((int)(blockDim.x >> 6));
    const int b = (int)blockIdx.x;
    const int q = lane >> 2, s = lane & 3;
    uint8_t *const ring = smem + L.ring + wave * L.ring_stride;
    uint8_t *const ring_end = ring + D * SLOT;
    Rec *const recs = (Rec *)(smem + L.recs + wave * L.recs_stride);
    float *const outs = (float *)(smem + L.outs);
    uint32_t *const cnt = (uint32_t *)(smem + L.cnt);
    const uint8_t *const actq = smem + L.act;

    // ---- the workgroup's rows and units: rows [r0, r0 + nr) of every matrix (the host's
    // N / G split, a.rbase[0] / a.rrem[0]); unit u = matrix u / nu, rows r0 + (u % nu) U ..
    const int N = a.n_rows[0];
    const int ush = a.dyn_ush;  // U = 1 << ush
    const int rbase = a.rbase[0], rrem = a.rrem[0];
    const int r0 = b * rbase + (b < rrem ? b : rrem);
    const int nr = rbase + (b < rrem ? 1 : 0);
    const int nu = (nr + U - 1) >> ush;
    const int units = a.n_desc * nu, nflat = a.n_desc * nr;
    const int64_t rowb = (int64_t)nb * BSZ;
    auto row_of = [&](int f) { return r0 + f; };
    // unit u's stream (its first byte), rows and flat output index: computed once, when the
    // unit is taken, and kept for its consumption in lane (k & 7) of four registers
    auto unit_of = [&](int u) {
        DynUnit d;
        const int m = (u >= nu ? 1 : 0) + (u >= 2 * nu ? 1 : 0) + (u >= 3 * nu ? 1 : 0);
        const int lr = (u - m * nu) << ush;
        d.rows = nr - lr < U ? nr - lr : U;
        d.flat = m * nr + lr;
        const uint8_t *w = m == 0 ? a.w[0] : m == 1 ? a.w[1] : m == 2 ? a.w[2] : a.w[3];
        d.src = w + (int64_t)(r0 + lr) * rowb;
        d.G = d.rows * nb;
        d.T = (d.G + ROWS_SB - 1) / ROWS_SB;
        return d;
    };
    const int nstat = nwv * P < units ? nwv * P : units;  // statically assigned unit ids [0, nstat)

    // ---- issue side: the unit being issued, its next step, the claimed-unit list
    uint32_t ul = 0, uh = 0, ug = 0, uf = 0;  // lane k & 7: the k-th unit's src (lo, hi), G | rows << 16, flat
    int ki = -1, is = 0, iT = 0, issued = 0;
    bool idone = false, iwait = false;
    const uint8_t *is16 = nullptr, *il16 = nullptr;
    uint8_t *islot = ring;
    auto take = [&](int u) {
        ++ki;
        const DynUnit d = unit_of(u);
        const bool mine = lane == (ki & 7);
        ul = mine ? (uint32_t)(uintptr_t)d.src : ul;
        uh = mine ? (uint32_t)((uintptr_t)d.src >> 32) : uh;
        ug = mine ? (uint32_t)(d.G | (d.rows << 16)) : ug;
        uf = mine ? (uint32_t)d.flat : uf;
        is16 = (const uint8_t *)((uintptr_t)d.src & ~(uintptr_t)15);
        il16 = (const uint8_t *)((uintptr_t)(d.src + (int64_t)d.G * BSZ - 1) & ~(uintptr_t)15);
        iT = d.T;
        is = 0;
    };
    // the next unit: static ones first; a claim only once the counter is set (claim_ok)
    auto next_unit = [&](bool claim_ok) {
        const int k = ki + 1;
        if (k < P) {
            const int u = wave * P + k;
            if (u < nstat) take(u);
            else idone = true;
            return;
        }
        if (!claim_ok) {
            iwait = true;
            return;
        }
        iwait = false;
#if KQ_ROWS_DYN_RR  // experiment builds: the same units dealt round-robin, no claim (cost isolation)
        const int uu = nwv * P + (k - P) * nwv + wave;
#else
        uint32_t u = 0;
        if (lane == 0) u = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const int uu = __builtin_amdgcn_readfirstlane((int)u);
#endif
        if (uu < units) take(uu);
        else idone = true;
    };
    auto issue = [&](bool claim_ok) {  // one step (NI DMA instructions), then the next unit if this one is done
        const uint8_t *base = is16 + (int64_t)is * (ROWS_SB * BSZ) + 16 * lane;
        if (is + 1 < iT) {
#pragma unroll
            for (int i = 0; i < NI; ++i)
                if (i + 1 < NI || lane < GRAN - 64 * (NI - 1)) dma16_nt(base + 1024 * i, (LDS void *)(islot + 1024 * i));
        } else {
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const uint8_t *p = base + 1024 * i;
                if (i + 1 < NI || lane < GRAN - 64 * (NI - 1))
                    dma16_nt(p < il16 ? p : il16, (LDS void *)(islot + 1024 * i));
            }
        }
        islot = islot + SLOT == ring_end ? ring : islot + SLOT;
        ++is;
        ++issued;
        if (is == iT) next_unit(claim_ok);
    };
    next_unit(false);  // the first static unit (or none)

    // residual of the fused ADD for flat row 64 * wave + lane, fetched with the activation
    // (issued on every path: a dummy read of x without one; kept live until the flush waits)
    const int f0 = 64 * wave + lane;
    const int fm = (f0 >= nr ? 1 : 0) + (f0 >= 2 * nr ? 1 : 0) + (f0 >= 3 * nr ? 1 : 0);
    const float *fres = fm == 0 ? a.res[0] : fm == 1 ? a.res[1] : fm == 2 ? a.res[2] : a.res[3];
    const int frow = row_of(f0 - fm * nr);
    uint32_t rv = 0;

    // ---- prologue (the product kq_rows prologue: one step before the activation wait)
    if (FUSEDQ) {
        const int PASS = 4 * nwv;
        u32x4 xv[ROWS_QPASS][4] = {};
        u32x4 x2v[ROWS_QPASS][4] = {};
        const int qiters = (nb + PASS - 1) / PASS;
        int qw = 0;
#pragma unroll
        for (int i = 0; i < ROWS_QPASS; ++i) qw += (i < qiters && PASS * i + 4 * wave < nb) ? 1 : 0;
#pragma unroll
        for (int i = 0; i < ROWS_QPASS; ++i) {
            if (i < qw) {
                const int j = PASS * i + 4 * wave + (lane >> 4);
                const int bb = j < nb ? j : nb - 1;
                const float *xp = a.x + (int64_t)bb * QK + 16 * (lane & 15);
#pragma unroll
                for (int k = 0; k < 4; ++k) xv[i][k] = gload16_asm(xp + 4 * k);
                if (PRO != ROWS_PRO_NONE) {
                    const float *x2p = a.x2 + (int64_t)bb * QK + 16 * (lane & 15);
#pragma unroll
                    for (int k = 0; k < 4; ++k) x2v[i][k] = gload16_asm(x2p + 4 * k);
                }
            }
        }
        rv = gload4_asm(fres && f0 < nflat && frow < N ? fres + frow : a.x);
        // exactly one step's NI DMA instructions on every path (the constant wait below)
        if (ki < 0) {  // no unit: from the activation, into a slot never read
            const uint8_t *xb = (const uint8_t *)a.x + 16 * lane;
#pragma unroll
            for (int i = 0; i < NI; ++i)
                if (i + 1 == NI) dma16_nt_lanes(xb, (LDS void *)(islot + 1024 * i), lane, GRAN - 64 * (NI - 1));
                else dma16_nt(xb, (LDS void *)(islot + 1024 * i));
        } else {  // the first unit's first step, its partial DMA masked in asm
            const uint8_t *base = is16 + 16 * lane;
            const uint8_t *lim = iT > 1 ? base + 1024 * (NI - 1) : base + 1024 * (NI - 1) < il16 ? base + 1024 * (NI - 1) : il16;
#pragma unroll
            for (int i = 0; i + 1 < NI; ++i) {
                const uint8_t *p = base + 1024 * i;
                dma16_nt(iT > 1 || p < il16 ? p : il16, (LDS void *)(islot + 1024 * i));
            }
            dma16_nt_lanes(lim, (LDS void *)(islot + 1024 * (NI - 1)), lane, GRAN - 64 * (NI - 1));
            islot = islot + SLOT == ring_end ? ring : islot + SLOT;
            ++is;
            ++issued;
            if (is == iT) next_unit(false);
        }
        vm_wait<NI + 1>();  // x landed; the residual load and the step's DMAs may be in flight
        if (RSTAMPS(a)) sx = __builtin_amdgcn_s_memrealtime();
        asm volatile("" : "+v"(xv[0][0]), "+v"(xv[0][1]), "+v"(xv[0][2]), "+v"(xv[0][3]), "+v"(xv[1][0]),
                     "+v"(xv[1][1]), "+v"(xv[1][2]), "+v"(xv[1][3]), "+v"(xv[2][0]), "+v"(xv[2][1]),
                     "+v"(xv[2][2]), "+v"(xv[2][3]));
        if (PRO != ROWS_PRO_NONE) {
#pragma unroll
            for (int i = 0; i < ROWS_QPASS; ++i)
#pragma unroll
                for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(x2v[i][k]));
        }
        if (PRO == ROWS_PRO_SWIGLU) {
#pragma unroll
            for (int i = 0; i < ROWS_QPASS; ++i)
                if (i < qw)
#pragma unroll
                    for (int k = 0; k < 4; ++k) xv[i][k] = swiglu4(xv[i][k], x2v[i][k]);
        } else if (PRO == ROWS_PRO_NORM) {
            double *sums = (double *)(smem + L.sums);
#pragma unroll
            for (int i = 0; i < ROWS_QPASS; ++i) {
                if (i < qw) {
                    const int j = PASS * i + 4 * wave + (lane >> 4);
                    double sq = 0.0;
                    if (j < nb) {
                        float v[16];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            v[4 * k] = __uint_as_float(xv[i][k].x), v[4 * k + 1] = __uint_as_float(xv[i][k].y);
                            v[4 * k + 2] = __uint_as_float(xv[i][k].z), v[4 * k + 3] = __uint_as_float(xv[i][k].w);
                        }
                        sq = sumsq16(v);
                    }
                    sq = row16_sum(sq);
                    if (j < nb && (lane & 15) == 0) sums[j] = sq;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            double tot = seq_sum_lanes(sums, nb, lane);
            if (rms_mean_ambiguous(div_by_count(tot, (int64_t)nb * QK), (int64_t)nb * QK))
                tot = seq_sumsq_wave(a.x, (int64_t)nb * QK, lane);
            const float mean = (float)div_by_count(tot, (int64_t)nb * QK);
            const float scale = 1.0f / sqrtf(mean + a.eps);
#pragma unroll
            for (int i = 0; i < ROWS_QPASS; ++i)
                if (i < qw)
#pragma unroll
                    for (int k = 0; k < 4; ++k) xv[i][k] = normmul4(xv[i][k], x2v[i][k], scale);
        }
#pragma unroll 1
        for (int i = 0; i < qw; ++i) {
            u32x4 cur[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) cur[k] = i == 0 ? xv[0][k] : i == 1 ? xv[1][k] : xv[2][k];
            const int j = PASS * i + 4 * wave + (lane >> 4);
            if (j < nb) quant16_store(cur, lane & 15, smem + L.act + Q8L_STRIDE * j);
        }
        if (RSTAMPS(a)) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            sq = __builtin_amdgcn_s_memrealtime();
        }
    } else {
        const int ng = nb * (Q8L_STRIDE / 16);
        for (int j = wave; 64 * j < ng; j += nwv) {
            const int k = 64 * j + lane;
            if (k < ng) dma16(a.xq + 16 * k, (LDS void *)(smem + L.act + 1024 * j));
        }
        rv = gload4_asm(fres && f0 < nflat && frow < N ? fres + frow : (const float *)a.xq);
        if (!idone && !iwait && ki >= 0) issue(false);
        vm_wait_k<NI>(issued);
    }
    while (!idone && !iwait && ki >= 0 && issued < D) issue(false);  // the rest of the ring: static units only
    if (wave == 0 && lane == 0) *cnt = (uint32_t)(nwv * P);            // claims start after the static ids
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // Q8_K row complete, counter set
    if (iwait) next_unit(true);
    while (!idone && ki >= 0 && issued < D) issue(true);
    const uint64_t st1 = RSTAMPS(a) ? __builtin_amdgcn_s_memrealtime() : 0;

    // ---- main loop: the oldest step in flight, then one more issued
    int kc = 0, cs = 0, cT = 0, cG = 0, cmis = 0, crows = 0, io = 0, rr = 0;
    int bro = 0;        // batch rows before the current unit
    uint32_t bfl = 0;   // lane r: flat output index of batch row r
    auto consume_unit = [&](int k) {
        const uint32_t gr = (uint32_t)__builtin_amdgcn_readlane((int)ug, k & 7);
        const int flat = __builtin_amdgcn_readlane((int)uf, k & 7);
        cG = (int)(gr & 0xffffu);
        crows = (int)(gr >> 16);
        cT = (cG + ROWS_SB - 1) / ROWS_SB;
        cmis = (int)((uint32_t)__builtin_amdgcn_readlane((int)ul, k & 7) & 15u);
        bfl = lane >= bro && lane < bro + crows ? (uint32_t)(flat + lane - bro) : bfl;
        cs = 0;
        io = q;
        rr = bro;
        while (io >= nb) {
            io -= nb;
            ++rr;
        }
    };
    auto replay = [&]() {  // the batch's rows: lane r <-> batch row r, records in superblock order
        wave_lds_fence();
        if (lane < bro) {
            float v = 0.f;
            const Rec *rc = recs + lane;
#pragma unroll 4
            for (int i = 0; i < nb; ++i) v = chain_step(TYPE, rc[i * bR], v);
            outs[bfl] = v;
        }
        wave_lds_fence();
        bro = 0;
    };
    int consumed = 0;
    if (issued > 0) consume_unit(0);
    const uint8_t *cslot = ring;
#pragma unroll 1
    while (consumed < issued) {
        vm_wait_k<NI>(issued - consumed - 1);
        if (ROWS_SB * cs + q < cG) {
            const uint8_t *blk = cslot + cmis + q * BSZ;
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
        ++consumed;
        ++cs;
        if (!idone) issue(true);
        if (RSTAMPS(a) && consumed == 1) sf = __builtin_amdgcn_s_memrealtime();
        if (cs == cT) {  // the unit's last step: into the batch; replay when the next unit may not fit
            bro += crows;
            if (bro + U > bR || consumed == issued) replay();
            ++kc;
            if (consumed < issued) consume_unit(kc);
        } else {
            io += ROWS_SB;
            while (io >= nb) {
                io -= nb;
                ++rr;
            }
        }
    }

    const uint64_t st2 = RSTAMPS(a) ? __builtin_amdgcn_s_memrealtime() : 0;
    // ---- flush: the workgroup's rows, coalesced, with the residual ADD / SWIGLU epilogue
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(rv));
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int f = f0; f < nflat; f += 64 * nwv) {
        const int m = (f >= nr ? 1 : 0) + (f >= 2 * nr ? 1 : 0) + (f >= 3 * nr ? 1 : 0);
        const int row = f == f0 ? frow : row_of(f - m * nr);
        if (row >= N) continue;  // the short last unit's unused slots
        const float *res = m == 0 ? a.res[0] : m == 1 ? a.res[1] : m == 2 ? a.res[2] : a.res[3];
        float *y = m == 0 ? a.y[0] : m == 1 ? a.y[1] : m == 2 ? a.y[2] : a.y[3];
        float v = outs[f];
        if (res) v = v + (f == f0 ? __uint_as_float(rv) : res[row]);  // ggml_add(mul_mat, residual)
        store_y(y + row, v);
    }
    if (a.epi) {  // y[0] = gate, y[1] = up: the same rows of both in this workgroup
        const int n4 = a.epi_n & ~3;
        for (int f = f0; f < nr; f += 64 * nwv) {
            const int r = row_of(f);
            if (r >= N) continue;
            const float gv = outs[f], uv = outs[nr + f];
            store_y(a.epi_y + r, r < n4 ? v_silu(gv) * uv : (gv / (1.0f + expf(-gv))) * uv);
        }
    }
    if (RSTAMPS(a)) {  // the kq_rows stamp layout (tools/stamps.py); slot 7: units this wave took
        const int64_t o = ((int64_t)blockIdx.x * ROWS_WAVES + wave) * 8;
        if (lane == 0 && o + 7 < a.stamps_cap) {
            RSTAMPS(a)[o] = st0;
            RSTAMPS(a)[o + 1] = st1;
            RSTAMPS(a)[o + 2] = st2;
            RSTAMPS(a)[o + 3] = __builtin_amdgcn_s_memrealtime();
            RSTAMPS(a)[o + 4] = sx;
            RSTAMPS(a)[o + 5] = sq;
            RSTAMPS(a)[o + 6] = sf;
            RSTAMPS(a)[o + 7] = (uint64_t)(ki + 1);
        }
    }
}
template <int TMASK, bool FUSEDQ, int PRO>
__global__ void __launch_bounds__(ROWS_WAVES * 64) kq_rows_dyn(const RowsArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint64_t st0 = RSTAMPS(a) ? __builtin_amdgcn_s_memrealtime() : 0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const RowsDynLayout L =
        rows_dyn_layout(a.nb, TMASK, a.bR, a.rpw, __builtin_amdgcn_readfirstlane((int)(blockDim.x >> 6)));
    constexpr int TYPE = TMASK == 1 ? Q4_K : TMASK == 2 ? Q5_K : Q6_K;
    rows_dyn_body<TYPE, FUSEDQ, PRO>(a, smem, L, wave, lane, st0);
}

#define KQ_ROWS_DYN_INST(TM, FQ, PR) template __global__ void kq_rows_dyn<TM, FQ, PR>(const RowsArgs a);
#define KQ_ROWS_DYN_INST_T(TM)        \
    KQ_ROWS_DYN_INST(TM, true, 0)     \
    KQ_ROWS_DYN_INST(TM, true, 1)     \
    KQ_ROWS_DYN_INST(TM, true, 2)     \
    KQ_ROWS_DYN_INST(TM, false, 0)
KQ_ROWS_DYN_INST_T(1)
KQ_ROWS_DYN_INST_T(2)
KQ_ROWS_DYN_INST_T(4)

}  // namespace kq
