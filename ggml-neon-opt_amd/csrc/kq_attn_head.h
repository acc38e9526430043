// kq_attn_head.h — decode attention of one query head on 256 threads (rope + f16 KV-cache
// write + KQ + soft_max + KQV), the body of kq_attn_decode (kq_ops.hip) and of the fused
// attention + o-proj kernel (kq_attn_oproj.hip).
#pragma once

#include "kq_attn_device.h"
#include "kq_device.h"
#include "kq_ops_device.h"

namespace kq {

// ------------------------------------------------------------ decode attention
// One workgroup per query head h (kv head g = h / (n_head/n_head_kv)), 256 threads.
//  0. Every load that does not depend on the position is issued together with the
//     position itself: this token's q/k/v, K-cache row t (the cell thread t scores in
//     the first pass) and the first VPF 8-cell groups of this thread's V-cache row(s).
//     Only the rope-table row waits for the position, so a launch pays two memory
//     latencies instead of four. Prefetched cells at or after pos are never used (the
//     new cell comes from LDS, later cells are masked).
//  1. rope(q_h), rope(k_g) at `pos` -> f16; v_g -> f16. The first query head of each
//     kv group writes the new cell to the caches (K [cell][kvw], V transposed
//     [ch][n_ctx]); every workgroup uses its own LDS copy of that cell, so no
//     workgroup reads a cache cell written in this launch.
//  2. kq[c] = vec_dot_f16(k_cache[c], q16) for c <= pos (NEON FP16 structure), * scale;
//     cells pos < c < n_kv are masked (-INF) and contribute exact zeros below
//     (the cache is zero-initialised, so their dot products are finite).
//  3. soft_max: max; v_expf(w - max) per cell, group sums of 4 in the vaddvq order,
//     the double sum over groups in order (one lane), p = e * (float)(1.0/sum) -> f16.
//  4. kqv[d] = vec_dot_f16(v_cache[g*hd+d][0..n_kv), p16): thread (d, j) runs
//     accumulator j (8 lanes) over cells 32it+8j+l, then the f16 reduce tree.
// A position outside the cache fails loudly: NaN output, caches untouched.
// Caches past KQ_ATTN_BATCH_CTX cells (kq_attn_decode<HD, true, DS>, DS = 4 or 8): the head
// is split over DS workgroups by output; q/k/v, the rope row and the first chunk of K rows
// arrive by LDS-DMA with the position, K whole rows per instruction into a two-slot ring
// per wave (KDMA below), soft_max on each thread's own cells (head_dim 64), and the
// workgroup's V rows by LDS-DMA under soft_max ("Split by output").
// Timing diagnostics (MI355X_ATTN_DIAG stops) only in experiment builds
// (make variant-ops NAME=adiag VFLAGS=-DKQ_ATTN_DIAG=1); the product kernel has none.
#ifndef KQ_ATTN_DIAG
#define KQ_ATTN_DIAG 0
#endif
// Cells whose K row / V chunk is loaded with the position, before it is known (the rest,
// up to the position, after it): 0 = every cell of the register path (TPH) / 8 V iterations.
#ifndef KQ_ATTN_PFC
// 0 (all of them) -> 64: TinyLlama token +2 % (tools/ab_ao.sh); 64 -> 32: +0.5 % (tg128, three
// interleaved rounds), 8B equal; 128: -1 % (tools/attn_pfc_ab.sh, profiles/r05_attn_pfc_ab.txt)
#define KQ_ATTN_PFC 32
#endif
// a diagnostic stop's output: depends on every value it keeps live, always a float in [1, 2)
// (garbage bits would send the next GEMV's rms_norm and soft_max down their slow paths)
__device__ __forceinline__ float adiag_finite(uint32_t bits) { return __uint_as_float((bits & 0x007fffffu) | 0x3f800000u); }
// Experiment build (KQ_ATTN_EARLY=1): the cells past the prefetched ones, up to the position,
// requested as soon as the position is known (before rope, KQ and soft_max) instead of where
// they are used: K rows up to the register path's TPH cells, V chunks of KQ_ATTN_VPOST more
// 32-cell iterations. Measured neutral to -1 % on the TinyLlama / 8B tokens
// (profiles/r04_attn_ab.txt), so off.
#ifndef KQ_ATTN_EARLY
#define KQ_ATTN_EARLY 0
#endif
#ifndef KQ_ATTN_VPOST
#define KQ_ATTN_VPOST 2
#endif
// V-cache iterations (32 cells each) requested together in KQV, past the prefetched ones
#ifndef KQ_ATTN_VB
#define KQ_ATTN_VB 8
#endif
#ifndef KQ_ATTN_VB64  // head_dim 64: half the registers per K row, twice the batch
#define KQ_ATTN_VB64 8
#endif
#ifndef KQ_ATTN_KR64
#define KQ_ATTN_KR64 2
#endif
#ifndef KQ_ATTN_KR128  // head_dim 128: a K row is 64 VGPRs; two per round cost the short-context
#define KQ_ATTN_KR128 1  // launch 0.7 us at Llama-3-8B (247 VGPRs, profiles/r05q_token8b_summary.md)
#endif
#ifndef KQ_ATTN_EARLYV  // 1: head_dim 64, KQV's first V batch requested with the position (measured -1 % tg1024)
#define KQ_ATTN_EARLYV 0
#endif
#ifndef KQ_ATTN_VLDS  // 1: experiment build with the LDS-staged V rows (launch_attn): measured neutral
#define KQ_ATTN_VLDS 0
#endif
#if KQ_ATTN_DIAG
#define ADIAG(a) ((a).diag)
#else
#define ADIAG(a) 0
#endif
// The per-head body, shared by kq_attn_decode (one 256-thread workgroup per head) and the
// fused attention + o-proj kernel (kq_attn_oproj.hip: several heads per workgroup, 256
// threads each; every __syncthreads() is reached by all of them in the same order since the
// control flow depends only on the position). t: the thread's index within the head's 256;
// smem: this head's LDS (attn_lds bytes); out: where output d of the head goes
// (out[d], global or LDS); may_write: this workgroup may store the new KV cell.
// TPH: threads per head (256; 128 for head_dim 64 in the fused kernel, where 4 heads share a
// workgroup and 256 threads each would cap it at 128 VGPRs): the register path holds one
// cell per thread (n_kv <= TPH), KQV runs HD * 4 / TPH (d, j) items per thread.
// VPF0: V-cache iterations (32 cells each) prefetched with the position (0: 8 / ITEMS).
// OUT_WT: out is global memory, stored write-through (sc1) for the next launch (kq_rows'
// outputs likewise, KQ_ROWS_YSC1).
// SC1_IN: q / k / v were written in this launch by other workgroups (the persistent layer,
// kq_layer.hip): every load of them is an agent-scope (sc1) load, as the hand-off requires.
// One LDS-DMA instruction (default cache policy: the V cache is re-read token after token)
// for lanes [0, n) at LDS byte address m0 (wave-uniform), the lane mask set inside the asm.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void attn_dma16_lanes(const void *src, uint32_t m0, int lane, int n) {
    uint64_t save;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "v_cmp_gt_i32_e32 vcc, %2, %3\n\t"
        "s_and_b64 exec, exec, vcc\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %4, off\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(save)
        : "s"(m0), "s"(n), "v"(lane), "v"(src)
        : "memory", "m0", "vcc");
}
// ... all 64 lanes
__device__ __forceinline__ void attn_dma16(const void *src, uint32_t m0) {
    asm volatile(
        "s_mov_b32 m0, %0\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off"
        :
        : "s"(m0), "v"(src)
        : "memory", "m0");
}
#pragma clang diagnostic pop

// K-cache ring of the split head_dim-64 kernel (KDMA below): per wave KQ_ATTN_KD slots of 64
// rows (8 KiB)
#ifndef KQ_ATTN_KD
#define KQ_ATTN_KD 2
#endif
// 1: KDMA's soft_max on the cells each thread scored (max kept from KQ, group sums across the
// quad's lanes, every wave summing the groups itself): three barriers instead of five
#ifndef KQ_ATTN_KSM
#define KQ_ATTN_KSM 1
#endif
constexpr int ATTN_KSLOT = 64 * 128;

// attn_lds (kq_ops.hip) on the device: the per-head LDS layout below, before any staged V rows
__device__ __forceinline__ int attn_lds_dev(int hd, int n_ctx) {
    const int gsum = (n_ctx / 4) * 8 <= hd * 64 ? 0 : (n_ctx / 4) * 8;
    return 6 * hd + n_ctx * 6 + hd * 64 + 16 + gsum;
}

// DS > 1 (kq_attn_decode past KQ_ATTN_BATCH_CTX cells, BATCH): the head is split over DS
// workgroups by output dimension; workgroup ds computes the whole KQ and soft_max (every slice
// needs every weight) and KQV for outputs [ds HD/DS, (ds + 1) HD/DS) only, from its slice of
// the V rows, staged in LDS by LDS-DMA as soon as the position is known. One workgroup's
// cache reads for KQV drop to 1/DS and arrive in one round under KQ and soft_max, where the
// unsplit head waits for them in n_kv / (32 VB) dependent batches after soft_max. The
// accumulation order of every output is unchanged (bit-exact).
template <int HD, int TPH = 256, int VPF0 = 0, bool OUT_WT = false, bool SC1_IN = false, bool BATCH = false,
          int DS = 1, bool KD1 = false>
__device__ __forceinline__ void attn_head(const AttnArgs &a, int h, int t, uint8_t *smem, float *out,
                                          bool may_write, int ds = 0) {
    auto ldin = [](const float *p) {
        if (SC1_IN) return __uint_as_float(__hip_atomic_load((const uint32_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        return *p;
    };
    static_assert(HD == 64 || HD == 128, "head_dim");
    constexpr int KV4 = HD / 8;          // 16-B pieces of one K-cache row
    static_assert(TPH == 256 || (TPH == 128 && HD == 64), "threads per head");
    // BATCH (kq_attn_decode): the cache loads past the prefetched cells are batched (KR K rows
    // per round, KQ_ATTN_VB V chunks); the fused kernels' register budgets keep one K row and
    // one V chunk per step (PAIR off)
    constexpr bool PAIR = BATCH && TPH == 256 && !SC1_IN;
    static_assert(DS == 1 || (PAIR && (HD / DS) % 4 == 0 && HD / DS * 4 <= TPH), "output slices");
    constexpr int RS = HD / DS;  // V rows (outputs) of this workgroup
    // KDMA (split head_dim-64 kernel, caches past the register path): KQ's K rows arrive by
    // LDS-DMA in chunks of 256 cells, each wave loading the 64 rows its own lanes score, eight
    // whole rows (1 KiB, 8 lanes per row) per instruction. The per-thread row loads of the
    // other paths put 64 different rows under every load instruction, which the texture
    // path serves at about one cache line per cycle (measured: ~0.85 us per 256 cells per
    // workgroup); here an instruction touches 8 rows' lines. Within a row the 16-B chunks are
    // stored at position k ^ ((lane >> 1) & 7) so that each thread's row reads are free of
    // bank conflicts; the dot product itself is unchanged (bit-exact).
    // head_dim 128: a row is 256 B, two lanes per cell (each holding half the row; the odd
    // lane continues the even lane's accumulators: the NEON order), 128 cells per chunk.
    // KD1 (experiment builds, KQ_ATTN_KDMA1): the unsplit head of a short cache (<= 256 cells)
    // on the same LDS-DMA path: K ring, staged q | k | v, V rows in LDS
    constexpr bool KDMA = PAIR && (DS > 1 || KD1);
    constexpr int CPC = HD == 64 ? 256 : 128;  // (KDMA) cells per chunk, CPC / 4 per wave
    // (KDMA) soft_max on each thread's own cells: head_dim 64 (one cell per lane)
    constexpr bool KSM = KDMA && HD == 64 && KQ_ATTN_KSM != 0;
    constexpr int VB = PAIR ? (HD == 64 ? KQ_ATTN_VB64 : KQ_ATTN_VB) : 4;
    constexpr int KR = HD == 64 ? KQ_ATTN_KR64 : KQ_ATTN_KR128;  // K rows per thread per round (register budget)
    constexpr int ITEMS = HD * 4 / TPH;  // KQV (d, j) items per thread
    constexpr int VPF = VPF0 > 0 ? VPF0 : KQ_ATTN_PFC > 0 ? (KQ_ATTN_PFC / 32 < 8 / ITEMS ? KQ_ATTN_PFC / 32 : 8 / ITEMS)
                                                         : 8 / ITEMS;  // prefetched 32-cell iterations per item
    constexpr int KPF = KQ_ATTN_PFC > 0 && KQ_ATTN_PFC < TPH ? KQ_ATTN_PFC : TPH;  // K rows prefetched (thread t < KPF)
    static_assert(VPF + (KQ_ATTN_EARLY ? KQ_ATTN_VPOST : 0) <= (BATCH && TPH == 256 && !SC1_IN ? KQ_ATTN_VB : 4),
                  "KQV's first batch holds the prefetched V iterations");
    const int gsz = a.n_head / a.n_head_kv;
    const int g = h / gsz;
    const int kvw = a.n_head_kv * HD;
    if (ADIAG(a) == 4) return;  // diagnostics (MI355X_ATTN_DIAG): empty launch

    // LDS (attn_lds): q16 | k16 | v16 (HD f16 each) | w (n_ctx f32) | p16 (n_ctx f16) |
    // red (HD*32 f16 accumulators) | scal (max, 1/sum, 2 pad) [| gsum]; every piece 16-B aligned
    uint16_t *q16 = (uint16_t *)smem;
    uint16_t *k16 = q16 + HD;
    uint16_t *v16 = k16 + HD;
    float *w = (float *)(smem + 6 * HD);
    uint16_t *p16 = (uint16_t *)(w + a.n_ctx);
    h16 *red = (h16 *)(p16 + a.n_ctx);
    float *scal = (float *)(red + HD * 32);
    // per group of 4 cells: (double)((e0 + e1) + (e2 + e3)); lives in `red` (free until
    // KQV) when it fits, past scal otherwise
    double *gsum = (a.n_ctx / 4) * 8 <= HD * 64 ? (double *)red : (double *)(scal + 4);
    const int VSTR = 2 * a.n_ctx + 16;
    uint8_t *const vlds = smem + (attn_lds_dev(HD, a.n_ctx) + 15) / 16 * 16;
    uint8_t *const kring = vlds + RS * VSTR;  // (KDMA) after the V rows
    // (KDMA) chunk c of K rows, cells [CPC c, CPC c + CPC) clamped to lim - 1, into this
    // wave's ring slot: wave wv's CPC / 4 rows, 1 KiB (8 or 4 whole rows) per instruction.
    // Lane ln of the wave reads the 128 B at slot + 128 ln: a whole row (head_dim 64) or half
    // of one (128: row ln / 2, half ln & 1), its 16-B chunk k at position k ^ ((ln >> 1) & 7)
    auto issue_k = [&](int c, int lim) {
        const int wv = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;
        const uint32_t slot = (uint32_t)(uintptr_t)(LDS void *)(kring + (wv * KQ_ATTN_KD + c % KQ_ATTN_KD) * ATTN_KSLOT);
        const int r = ln >> 3, pp = ln & 7;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int lr = 8 * i + r;  // the lane that reads these 128 B
            int row = CPC * c + (CPC / 4) * wv + (HD == 64 ? lr : lr >> 1);
            row = row < lim ? row : lim - 1;  // (rows past n_kv are never read)
            const int k = (HD == 64 ? 0 : 8 * (lr & 1)) + (pp ^ ((lr >> 1) & 7));
            const uint8_t *src = (const uint8_t *)(a.k_cache + (int64_t)row * kvw + (int64_t)g * HD) + 16 * k;
            attn_dma16(src, __builtin_amdgcn_readfirstlane(slot + 1024 * i));
        }
    };

    // ---- 0. position-independent loads, issued with the position
    const int pos_in = *a.pos;
    float x0 = 0.f, x1 = 0.f, y0 = 0.f, y1 = 0.f;
    float rc = 0.f, rs = 0.f;  // rope_row: cos/sin of the thread's pair, staged with the position
    if constexpr (KDMA) {
        // q | k | v | the rope row (rope_row) by one LDS-DMA of wave 0 into the first KiB of the
        // V-row area (free until KQ is done), then the first chunk of K rows, all before the
        // position is known. Every memory operation of this path is then an LDS-DMA whose
        // waits are counted here, so rope waits for its inputs only (vmcnt retires in order:
        // a compiler-visible load here would make every later wait cover the K rows too).
        if (t < 64) {  // (head_dim 128: two instructions, q | k then v | rope)
            constexpr int L = HD / 4;  // lanes per vector
#pragma unroll
            for (int i = 0; i < HD / 64; ++i) {
                const int e = 64 * i + t;  // 16-B piece of the 4 HD floats
                const float *src = e < L       ? a.q + (int64_t)h * HD + 4 * e
                                   : e < 2 * L ? a.k + (int64_t)g * HD + 4 * (e - L)
                                   : e < 3 * L ? a.v + (int64_t)g * HD + 4 * (e - 2 * L)
                                   : a.rope_row ? a.rope_table + 4 * (e - 3 * L)
                                                : a.q + (int64_t)h * HD;
                attn_dma16(src, (uint32_t)(uintptr_t)(LDS void *)(vlds + 1024 * i));
            }
        }
        issue_k(0, a.n_ctx);
    } else if (t < HD / 2) {
        if (a.rope_row) {
            rc = a.rope_table[2 * t];
            rs = a.rope_table[2 * t + 1];
        }
        const float *qp = a.q + (int64_t)h * HD + 2 * t;
        const float *kp = a.k + (int64_t)g * HD + 2 * t;
        x0 = ldin(qp);
        x1 = ldin(qp + 1);
        y0 = ldin(kp);
        y1 = ldin(kp + 1);
    } else if (t < HD / 2 + HD) {
        x0 = ldin(a.v + (int64_t)g * HD + (t - HD / 2));
    }
    uint4 kpre[KV4] = {};
    if (!KDMA && t < a.n_ctx && t < KPF && ADIAG(a) != 5) {  // (diag 5: no cache loads, stop after rope; timing only)
        const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)t * kvw + (int64_t)g * HD);
#pragma unroll
        for (int i = 0; i < KV4; ++i) kpre[i] = kr[i];
    }
    // V rows staged in LDS (launch_attn sets a.v_lds) only in the KQ_ATTN_VLDS build: as a run-time
    // choice its LDS / global select turned KQV's cache loads into flat loads (tg1024 -4 %, r5t)
    const bool vl = KDMA || (PAIR && KQ_ATTN_VLDS && a.v_lds);
    uint4 vpre[ITEMS][VPF] = {};
#pragma unroll
    for (int ii = 0; ii < ITEMS && !vl; ++ii) {
        const int item = t + TPH * ii, d = item >> 2, j = item & 3;
        const uint16_t *vr = a.v_cache + (int64_t)(g * HD + d) * a.n_ctx + 8 * j;
#pragma unroll
        for (int it = 0; it < VPF; ++it)
            if (32 * it < a.n_ctx && ADIAG(a) != 5) vpre[ii][it] = *(const uint4 *)(vr + 32 * it);
    }

    const bool bad = pos_in < 0 || pos_in >= a.n_ctx;  // no cache cell for this position
    const int pos = bad ? 0 : pos_in;
    int n_kv = (pos + 1 + 31) / 32 * 32;
    n_kv = n_kv < a.n_ctx ? n_kv : a.n_ctx;
    constexpr int VPOST = KQ_ATTN_EARLY ? KQ_ATTN_VPOST : 0;
    uint4 vpost[ITEMS][VPOST > 0 ? VPOST : 1] = {};
    if (KQ_ATTN_EARLY && ADIAG(a) != 5) {
        if (KPF < TPH && t >= KPF && t < pos && t < a.n_ctx) {  // this thread's K row, c = t < pos
            const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)t * kvw + (int64_t)g * HD);
#pragma unroll
            for (int i = 0; i < KV4; ++i) kpre[i] = kr[i];
        }
#pragma unroll
        for (int ii = 0; ii < ITEMS; ++ii) {
            const int item = t + TPH * ii, d = item >> 2, j = item & 3;
            const uint16_t *vr = a.v_cache + (int64_t)(g * HD + d) * a.n_ctx + 8 * j;
#pragma unroll
            for (int k = 0; k < VPOST; ++k) {
                const int it = VPF + k;
                if (32 * it <= pos) vpost[ii][k] = *(const uint4 *)(vr + 32 * it);  // (32 it <= pos < n_ctx)
            }
        }
    }
    // V rows of the head's kv group (DS > 1: the slice's RS rows), cells [0, n_kv), into LDS
    // (vl): wave w takes rows [w RS / 4, (w + 1) RS / 4); local row r at vlds + r * VSTR;
    // completion: vmcnt(0) + barrier before KQV. Issued once KQ's cache loads have been used:
    // vmcnt retires in issue order, so a wait for any load issued after the DMAs (rope's inputs,
    // KQ's K rows) would wait for them too; soft_max issues no memory loads and runs under them.
    // A cell past pos holds whatever the cache holds (its weight is an exact 0); the new cell is
    // patched from v16 as on the register path.
    auto issue_v_rows = [&]() {
        if (!vl) return;
        // every earlier load has been used; the builtin (unlike an asm wait) tells the compiler,
        // which would otherwise wait vmcnt(0) later for loads it cannot prove consumed (a kpre
        // row on a path that skipped it) — and so for these DMAs behind them. On every path.
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        if (bad) return;
        const int wv = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;
        const int gran = n_kv / 8;  // 16-B granules of a row
#pragma unroll 1
        for (int r = wv * (RS / 4); r < (wv + 1) * (RS / 4); ++r) {
            const uint8_t *src = (const uint8_t *)(a.v_cache + (int64_t)(g * HD + ds * RS + r) * a.n_ctx);
#pragma unroll 1
            for (int i = 0; 64 * i < gran; ++i) {
                const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(LDS void *)(vlds + r * VSTR + 1024 * i));
                const int n = __builtin_amdgcn_readfirstlane(gran - 64 * i);
                attn_dma16_lanes(src + 1024 * i + 16 * ln, m0, ln, n < 64 ? n : 64);
            }
        }
    };

    // EARLYV (head_dim 64, kq_attn_decode): KQV's first batch of V chunks past the prefetched
    // ones requested as soon as the position is known, under KQ and soft_max
    constexpr bool EARLYV = PAIR && HD == 64 && KQ_ATTN_EARLYV;
    uint4 vb0[ITEMS][EARLYV ? VB : 1];
    if (EARLYV && !vl) {
        const int n_it0 = (pos + 32) / 32;
#pragma unroll
        for (int ii = 0; ii < ITEMS; ++ii) {
            const int item = t + TPH * ii, d = item >> 2, j = item & 3;
            const uint16_t *vr = a.v_cache + (int64_t)(g * HD + d) * a.n_ctx;
#pragma unroll
            for (int k = VPF + VPOST; k < (EARLYV ? VB : 1); ++k)
                if (k < n_it0) vb0[ii][k] = *(const uint4 *)(vr + 32 * k + 8 * j);
        }
    }
    if constexpr (KDMA) {  // the staged q | k | v | rope row landed (wave 0: all but chunk 0's 8 DMAs)
        if (t < 64) __builtin_amdgcn_s_waitcnt(0x0F78);  // vmcnt(8)
        __syncthreads();
        const float *stg = (const float *)vlds;
        if (t < HD / 2) {
            x0 = stg[2 * t], x1 = stg[2 * t + 1];
            y0 = stg[HD + 2 * t], y1 = stg[HD + 2 * t + 1];
            rc = stg[3 * HD + 2 * t], rs = stg[3 * HD + 2 * t + 1];  // (used with rope_row only)
        } else if (t < HD / 2 + HD) {
            x0 = stg[2 * HD + (t - HD / 2)];
        }
        if (!a.rope_row) {  // the position's row of the whole table: loaded now and waited for
                            // here (with chunk 0: the slow path), so no load of the compiler's
                            // is pending where this branch rejoins the rope_row path
            if (t < HD / 2) {
                const float *row = a.rope_table + (int64_t)pos * HD;
                rc = row[2 * t];
                rs = row[2 * t + 1];
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
    }
    const float *tc = a.rope_table + (a.rope_row ? 0 : (int64_t)pos * (HD / 2) * 2);
    const bool writer = may_write && !bad && (h % gsz) == 0 && ds == 0;
    if (t < HD / 2) {
        const float c = (KDMA || a.rope_row) ? rc : tc[2 * t], s = (KDMA || a.rope_row) ? rs : tc[2 * t + 1];
        const float2 rq = rope_pair(x0, x1, c, s);
        q16[2 * t] = h2u(f2h_rne(rq.x));
        q16[2 * t + 1] = h2u(f2h_rne(rq.y));
        const float2 rk = rope_pair(y0, y1, c, s);
        const uint16_t k0 = h2u(f2h_rne(rk.x)), k1 = h2u(f2h_rne(rk.y));
        k16[2 * t] = k0;
        k16[2 * t + 1] = k1;
        if (writer) *(uint32_t *)(a.k_cache + (int64_t)pos * kvw + (int64_t)g * HD + 2 * t) = k0 | ((uint32_t)k1 << 16);
    } else if (t < HD / 2 + HD) {
        const int d = t - HD / 2;
        const uint16_t vv = h2u(f2h_rne(x0));
        v16[d] = vv;
        if (writer) a.v_cache[(int64_t)(g * HD + d) * a.n_ctx + pos] = vv;
    }
    __syncthreads();
    if (ADIAG(a) == 1 || ADIAG(a) == 5) {  // diagnostics: stop after the loads and rope
        vm_wait<0>();  // (staged V DMAs, vl) land before the wave ends
        if (t < HD) out[t] = adiag_finite(__float_as_uint(x0) ^ kpre[0].x ^ vpre[0][0].x ^ vpre[0][VPF - 1].y);
        return;
    }

    if ((!KDMA || HD == 64) && n_kv <= TPH) {  // one cell per thread: score, max, exp and group sum stay in registers
        const int c = t;
        float sc = -INFINITY;
        if (KDMA) __builtin_amdgcn_s_waitcnt(0x0F70);  // (KDMA) chunk 0 of the K rows landed
        if (c < n_kv && c <= pos) {
            uint4 kv[KV4];
            if (c == pos) {
#pragma unroll
                for (int i = 0; i < KV4; ++i) kv[i] = ((const uint4 *)k16)[i];
            } else if (KDMA) {  // chunk 0's ring slot of this wave: cell t at lane t & 63
                const int ln = t & 63, sw = (ln >> 1) & 7;
                const uint8_t *rowp = kring + (__builtin_amdgcn_readfirstlane(t >> 6) * KQ_ATTN_KD) * ATTN_KSLOT + 128 * ln;
#pragma unroll
                for (int i = 0; i < KV4; ++i) kv[i] = *(const uint4 *)(rowp + 16 * (i ^ sw));
            } else if (!KQ_ATTN_EARLY && KPF < TPH && c >= KPF) {  // a cell past the prefetched ones (below the position)
                const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)c * kvw + (int64_t)g * HD);
#pragma unroll
                for (int i = 0; i < KV4; ++i) kv[i] = kr[i];
            } else {  // prefetched with the position, or (KQ_ATTN_EARLY) right after it
#pragma unroll
                for (int i = 0; i < KV4; ++i) kv[i] = kpre[i];
            }
            sc = vec_dot_f16_rows<HD>(kv, (const uint4 *)q16) * a.scale;
        }
        issue_v_rows();
        const float wmx = wave_fmax(sc);  // max (order-free): per wave, then over the 4 waves
        if ((t & 63) == 0) scal[t >> 6] = wmx;
        __syncthreads();
        if (ADIAG(a) == 2) {  // diagnostics: stop after KQ
            vm_wait<0>();  // (staged V DMAs, vl) land before the wave ends
            if (t < HD) out[t] = adiag_finite(__float_as_uint(sc) ^ vpre[0][0].x ^ vpre[0][VPF - 1].y);
            return;
        }
        const float mx = TPH == 256 ? fmaxf(fmaxf(scal[0], scal[1]), fmaxf(scal[2], scal[3])) : fmaxf(scal[0], scal[1]);
        const float ec = c < n_kv && sc != -INFINITY ? v_expf(sc - mx) : 0.0f;
        // group sum of cells 4g..4g+3 (lanes 4g..4g+3) in the vaddvq order (e0 + e1) + (e2 + e3)
        const float s01 = ec + dpp_mov_f32<0xB1>(ec);   // lane 4g: e0 + e1, lane 4g+2: e2 + e3
        const float g4 = s01 + dpp_mov_f32<0x4E>(s01);  // lane 4g: (e0 + e1) + (e2 + e3)
        if ((t & 3) == 0 && c < n_kv) gsum[t >> 2] = (double)g4;
        __syncthreads();
        // every wave computes the same sum (no barrier to publish it): ggml's in-order double
        // sum, as a tree where that is exact (softmax_group_sum)
        const double sum = softmax_group_sum(gsum, n_kv / 4, t & 63);
        const float inv = (float)(1.0 / sum);
        if (c < n_kv) p16[c] = h2u(f2h_rne(ec * inv));
        __syncthreads();
        if (ADIAG(a) == 3) {  // diagnostics: stop after soft_max
            vm_wait<0>();  // (staged V DMAs, vl) land before the wave ends
            if (t < HD) out[t] = adiag_finite((uint32_t)p16[t] ^ vpre[0][0].x ^ vpre[0][VPF - 1].y);
            return;
        }
    } else {
        if constexpr (KDMA) {
            const int wv = __builtin_amdgcn_readfirstlane(t >> 6), ln = t & 63;
            const int n_ch = (n_kv + CPC - 1) / CPC;  // chunks; wave wv scores cells CPC c + (CPC / 4) wv + ...
            const int sw = (ln >> 1) & 7;             // this lane's 128 B: chunk k at position k ^ sw
            // head_dim 128: this lane's half of q (chunks 8 (ln & 1) + k)
            uint4 qh[8];
            if (HD == 128) {
#pragma unroll
                for (int i = 0; i < 8; ++i) qh[i] = ((const uint4 *)q16)[8 * (ln & 1) + i];
            }
            // chunk 0 was issued with the position (prologue); the cache stores of the new cell,
            // issued since, are older than chunk 1 and covered by its waits
            if (n_ch > 1) issue_k(1, n_kv);
            static_assert(KQ_ATTN_KD == 2 || KQ_ATTN_KD == 3, "the waits below cover two or three slots per wave");
            if (KQ_ATTN_KD == 3 && n_ch > 2) issue_k(2, n_kv);
            float mloc = -INFINITY;  // (KQ_ATTN_KSM) the max over this thread's cells
            for (int c = 0; c < n_ch; ++c) {
                // chunk c landed: the younger chunks in flight (8 DMAs each) may still be
                if (KQ_ATTN_KD == 3 && c + 2 < n_ch) __builtin_amdgcn_s_waitcnt(0x4F70);  // vmcnt(16)
                else if (c + 1 < n_ch) __builtin_amdgcn_s_waitcnt(0x0F78);               // vmcnt(8)
                else __builtin_amdgcn_s_waitcnt(0x0F70);
                if constexpr (HD == 64) {
                const int cell = 256 * c + t;
                if (cell < n_kv) {
                    uint4 kv[KV4];
                    if (cell == pos) {
#pragma unroll
                        for (int i = 0; i < KV4; ++i) kv[i] = ((const uint4 *)k16)[i];
                    } else {
                        const uint8_t *rowp = kring + (wv * KQ_ATTN_KD + c % KQ_ATTN_KD) * ATTN_KSLOT + 128 * ln;
#pragma unroll
                        for (int i = 0; i < KV4; ++i) kv[i] = *(const uint4 *)(rowp + 16 * (i ^ sw));
                    }
                    const float sc = cell <= pos ? vec_dot_f16_rows<HD>(kv, (const uint4 *)q16) * a.scale : -INFINITY;
                    w[cell] = sc;
                    mloc = fmaxf(mloc, sc);
                }
                } else {  // head_dim 128: lanes 2m, 2m + 1 score cell 128 c + 32 wv + m
                    const int cell = 128 * c + 32 * wv + (ln >> 1);
                    const bool live = cell < n_kv;  // (uniform per lane pair: both or neither)
                    uint4 kv[8];
                    if (cell == pos) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) kv[i] = ((const uint4 *)k16)[8 * (ln & 1) + i];
                    } else {
                        const uint8_t *rowp = kring + (wv * KQ_ATTN_KD + c % KQ_ATTN_KD) * ATTN_KSLOT + 128 * ln;
#pragma unroll
                        for (int i = 0; i < 8; ++i) kv[i] = *(const uint4 *)(rowp + 16 * (i ^ sw));
                    }
                    // ggml_vec_dot_f16 (NEON FP16), accumulator j over chunks j, 4+j, 8+j, 12+j:
                    // every lane runs its own two chunks per accumulator from 0 (the even lane's
                    // are the first two steps), then again from the even lane's result (the odd
                    // lane's are the last two); the odd lane reduces (acc0 + acc2) + (acc1 + acc3)
                    uint32_t x[4][4], y[4][4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t c0[4] = {kv[j].x, kv[j].y, kv[j].z, kv[j].w};
                        const uint32_t c1[4] = {kv[4 + j].x, kv[4 + j].y, kv[4 + j].z, kv[4 + j].w};
                        const uint32_t q0[4] = {qh[j].x, qh[j].y, qh[j].z, qh[j].w};
                        const uint32_t q1[4] = {qh[4 + j].x, qh[4 + j].y, qh[4 + j].z, qh[4 + j].w};
#pragma unroll
                        for (int k = 0; k < 4; ++k) x[j][k] = pk_fma_w(c1[k], q1[k], pk_fma_w(c0[k], q0[k], 0u));
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const uint32_t e = dpp_w<0xA0>(x[j][k]);  // quad_perm [0,0,2,2]: the even lane's
                            y[j][k] = pk_fma_w(c1[k], q1[k], pk_fma_w(c0[k], q0[k], e));
                        }
                    }
                    h16 sv[8];
#pragma unroll
                    for (int l = 0; l < 8; ++l) {
                        const h16 s0 = lane_of(y[0], l) + lane_of(y[2], l);
                        const h16 s1 = lane_of(y[1], l) + lane_of(y[3], l);
                        sv[l] = s0 + s1;
                    }
                    const float dot = f16x8_reduce(sv);
                    if (live && (ln & 1)) w[cell] = cell <= pos ? dot * a.scale : -INFINITY;
                }
                if (c + KQ_ATTN_KD < n_ch) issue_k(c + KQ_ATTN_KD, n_kv);  // (this slot's reads were used above)
            }
            if constexpr (KSM) {
                // soft_max over the thread's own cells 256 c + t (written by this thread: no
                // barrier before reading them back). max: per wave, then over the 4 waves
                const float wmx = wave_fmax(mloc);
                if ((t & 63) == 0) scal[t >> 6] = wmx;
                issue_v_rows();
                __syncthreads();
                if (ADIAG(a) == 2) {  // diagnostics: stop after KQ
                    vm_wait<0>();
                    if (t < HD) out[t] = adiag_finite(__float_as_uint(w[t]));
                    return;
                }
                const float mx = fmaxf(fmaxf(scal[0], scal[1]), fmaxf(scal[2], scal[3]));
                // the group sums' double sum: each wave sums its own groups and publishes one
                // double with its min last-bit exponent and a non-finite flag; where the total
                // meets softmax_group_sum's exactness bound (every partial sum exact: any order
                // gives ggml's in-order bits) the four wave sums are the sum, else the in-order
                // sum over gsum
                SumExact se;
                for (int c = 0; c < n_ch; ++c) {  // (uniform trip count: every lane in the quad sums)
                    const int cell = 256 * c + t;
                    const float sv = cell < n_kv ? w[cell] : -INFINITY;
                    const float ec = sv == -INFINITY ? 0.0f : v_expf(sv - mx);
                    // group of cells 4g..4g+3 (lanes 4g..4g+3) in the vaddvq order (e0 + e1) + (e2 + e3)
                    const float s01 = ec + dpp_mov_f32<0xB1>(ec);
                    const float g4 = s01 + dpp_mov_f32<0x4E>(s01);
                    if (cell < n_kv) {
                        w[cell] = ec;
                        if ((t & 3) == 0) {
                            gsum[cell >> 2] = (double)g4;
                            se.add(g4);
                        }
                    }
                }
                const bool wbad = __any(se.bad);
                const int wgmin = wave_imin(se.gmin);
                const double wsum = wave_sum_exact_f64(se.part);  // (meaningful only where exact)
                if ((t & 63) == 0) {
                    *(double *)(kring + 16 * wv) = wsum;  // (the K ring is free: every chunk consumed)
                    *(int *)(kring + 16 * wv + 8) = wgmin;
                    *(int *)(kring + 16 * wv + 12) = wbad;
                }
                __syncthreads();
                bool anybad = false;
                int gmin = 1 << 20;
                double s4[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    s4[q] = *(const double *)(kring + 16 * q);
                    const int gq = *(const int *)(kring + 16 * q + 8);
                    gmin = gq < gmin ? gq : gmin;
                    anybad = anybad || *(const int *)(kring + 16 * q + 12) != 0;
                }
                const double s4t = (s4[0] + s4[1]) + (s4[2] + s4[3]);
                const double sum = sum_exact_ok(s4t, gmin, anybad)
                                       ? s4t
                                       : (KQ_SEQ_SUM_WAVE ? seq_sum_wave(gsum, n_kv / 4, t & 63) : seq_sum_lds(gsum, n_kv / 4));
                const float inv = (float)(1.0 / sum);
                for (int c = 0; c < n_ch; ++c) {
                    const int cell = 256 * c + t;
                    if (cell < n_kv) p16[cell] = h2u(f2h_rne(w[cell] * inv));
                }
                __syncthreads();
                if (ADIAG(a) == 3) {  // diagnostics: stop after soft_max
                    vm_wait<0>();
                    if (t < HD) out[t] = adiag_finite((uint32_t)p16[t]);
                    return;
                }
            }
        } else if constexpr (PAIR) {
            // KQ + scale + mask; the first pass (c == t) scores the prefetched row. KR cells per
            // thread per round, every row requested before any is used.
            for (int c0 = t; c0 < n_kv; c0 += KR * TPH) {
                uint4 kv[KR][KV4];  // (branches, not selects: a select of the three sources takes
                                    // kpre's address and puts it in scratch)
#pragma unroll
                for (int r = 0; r < KR; ++r) {
                    const int c = c0 + r * TPH;
                    if (c < n_kv && c <= pos) {
                        if (c == pos) {
#pragma unroll
                            for (int i = 0; i < KV4; ++i) kv[r][i] = ((const uint4 *)k16)[i];
                        } else if (r == 0 && c == t && (KQ_ATTN_EARLY || t < KPF)) {
#pragma unroll
                            for (int i = 0; i < KV4; ++i) kv[r][i] = kpre[i];
                        } else {
                            const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)c * kvw + (int64_t)g * HD);
#pragma unroll
                            for (int i = 0; i < KV4; ++i) kv[r][i] = kr[i];
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < KR; ++r) {
                    const int c = c0 + r * TPH;
                    if (c < n_kv) w[c] = c <= pos ? vec_dot_f16_rows<HD>(kv[r], (const uint4 *)q16) * a.scale : -INFINITY;
                }
            }
        } else {
            // KQ + scale + mask; the first pass (c == t) scores the prefetched row
            for (int c = t; c < n_kv; c += TPH) {
                float s = -INFINITY;
                if (c <= pos) {
                    uint4 kv[KV4];
                    if (c == pos) {
#pragma unroll
                        for (int i = 0; i < KV4; ++i) kv[i] = ((const uint4 *)k16)[i];
                    } else if (c == t && (KQ_ATTN_EARLY || t < KPF)) {
#pragma unroll
                        for (int i = 0; i < KV4; ++i) kv[i] = kpre[i];
                    } else {
                        const uint4 *kr = (const uint4 *)(a.k_cache + (int64_t)c * kvw + (int64_t)g * HD);
#pragma unroll
                        for (int i = 0; i < KV4; ++i) kv[i] = kr[i];
                    }
                    s = vec_dot_f16_rows<HD>(kv, (const uint4 *)q16) * a.scale;
                }
                w[c] = s;
            }
        }
        if constexpr (!KSM) {
        issue_v_rows();
        __syncthreads();
        if (ADIAG(a) == 2) {  // diagnostics: stop after KQ
            vm_wait<0>();  // (staged V DMAs, vl) land before the wave ends
            if (t < HD) out[t] = adiag_finite(__float_as_uint(w[t]) ^ vpre[0][0].x ^ vpre[0][VPF - 1].y);
            return;
        }
        // max (order-free), then exp + group sums
        if (t < 64) {
            float m = -INFINITY;
            for (int c = t; c < n_kv; c += 64) m = fmaxf(m, w[c]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
            if (t == 0) scal[0] = m;
        }
        __syncthreads();
        const float mx = scal[0];
        for (int gi = t; gi < n_kv / 4; gi += TPH) {
            float e[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float wv = w[4 * gi + k];
                e[k] = wv == -INFINITY ? 0.0f : v_expf(wv - mx);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) w[4 * gi + k] = e[k];
            gsum[gi] = (double)((e[0] + e[1]) + (e[2] + e[3]));  // the vaddvq group sum, in parallel
        }
        __syncthreads();
        if (t < 64) {  // ggml's in-order double sum over the groups (a tree where exact)
            double sum = softmax_group_sum(gsum, n_kv / 4, t);
            sum = 1.0 / sum;
            if (t == 0) scal[1] = (float)sum;
        }
        __syncthreads();
        const float inv = scal[1];
        for (int c = t; c < n_kv; c += TPH) p16[c] = h2u(f2h_rne(w[c] * inv));
        __syncthreads();
        if (ADIAG(a) == 3) {  // diagnostics: stop after soft_max
            vm_wait<0>();  // (staged V DMAs, vl) land before the wave ends
            if (t < HD) out[t] = adiag_finite((uint32_t)p16[t] ^ vpre[0][0].x ^ vpre[0][VPF - 1].y);
            return;
        }
        }
    }

    // KQV: thread (d, j) -> accumulator j of output d. The V chunks past the prefetched ones
    // are requested KQ_ATTN_VB iterations at a time before any of them is used (a loop that
    // loads and then uses each chunk pays one memory latency per 32 cells: tg1024 -18 %).
    if (vl) {  // the staged V rows landed (every wave's DMAs); then the new cell patched into
               // them from v16, so the loop below reads LDS only, without per-cell branches
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), seen by the compiler (no stale waits below)
        __syncthreads();
        if (!bad)
            for (int r = t; r < RS; r += TPH) *(uint16_t *)(vlds + r * VSTR + 2 * pos) = v16[ds * RS + r];
        __syncthreads();
    }
    if (ADIAG(a) == 6) {  // diagnostics: stop before KQV's arithmetic (the staged V rows landed)
        if (t < HD) out[t] = adiag_finite((uint32_t)p16[t] ^ *(const uint32_t *)(vlds + 16 * t));
        return;
    }
    const int n_it = (pos + 32) / 32;  // iterations holding a cell <= pos; later ones add exact zeros
#pragma unroll
    for (int ii = 0; ii < (DS > 1 ? 1 : ITEMS); ++ii) {
        const int item = t + TPH * ii;
        const int vr_l = item >> 2, j = item & 3;  // (DS > 1: the local V row; threads past RS * 4 idle)
        if (DS > 1 && vr_l >= RS) break;
        const int d = DS > 1 ? ds * RS + vr_l : vr_l;
        const uint16_t *vr = a.v_cache + (int64_t)(g * HD + d) * a.n_ctx;
        uint32_t acc[4] = {};  // lanes 2k, 2k+1 of accumulator j in word k
        if (PAIR && vl) {  // V rows in LDS (new cell patched): 8 iterations' reads, then their FMAs
            const uint8_t *vrow = vlds + vr_l * VSTR + 16 * j;
            const uint8_t *prow = (const uint8_t *)p16 + 16 * j;
            int it = 0;
            for (; it + 8 <= n_it; it += 8) {
                uint4 vb[8], pb[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    vb[k] = *(const uint4 *)(vrow + 64 * (it + k));
                    pb[k] = *(const uint4 *)(prow + 64 * (it + k));
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    acc[0] = pk_fma_w(vb[k].x, pb[k].x, acc[0]);
                    acc[1] = pk_fma_w(vb[k].y, pb[k].y, acc[1]);
                    acc[2] = pk_fma_w(vb[k].z, pb[k].z, acc[2]);
                    acc[3] = pk_fma_w(vb[k].w, pb[k].w, acc[3]);
                }
            }
            for (; it < n_it; ++it) {
                const uint4 vv = *(const uint4 *)(vrow + 64 * it), pp = *(const uint4 *)(prow + 64 * it);
                acc[0] = pk_fma_w(vv.x, pp.x, acc[0]);
                acc[1] = pk_fma_w(vv.y, pp.y, acc[1]);
                acc[2] = pk_fma_w(vv.z, pp.z, acc[2]);
                acc[3] = pk_fma_w(vv.w, pp.w, acc[3]);
            }
        } else if constexpr (PAIR) {
            for (int it0 = 0; it0 < n_it; it0 += VB) {
                uint4 vb[VB];
#pragma unroll
                for (int k = 0; k < VB; ++k) {
                    const int it = it0 + k;
                    if (!vl && it0 == 0 && k < VPF) {
                        vb[k] = vpre[ii][k < VPF ? k : 0];
                    } else if (VPOST > 0 && it0 == 0 && k < VPF + VPOST) {
                        vb[k] = vpost[ii][k - VPF < (VPOST > 0 ? VPOST : 1) ? k - VPF : 0];
                    } else if (EARLYV && !vl && it0 == 0) {
                        vb[k] = vb0[ii][k < (EARLYV ? VB : 1) ? k : 0];  // requested with the position (it < n_it)
                    } else if (it < n_it) {
                        vb[k] = vl ? *(const uint4 *)(vlds + vr_l * VSTR + 2 * (32 * it + 8 * j))
                                   : *(const uint4 *)(vr + 32 * it + 8 * j);
                    }
                }
#pragma unroll
                for (int k = 0; k < VB; ++k) {
                    const int it = it0 + k;
                    if (it < n_it) {
                        const int c0 = 32 * it + 8 * j;
                        const uint4 pp = *(const uint4 *)(p16 + c0);
                        uint32_t vw[4] = {vb[k].x, vb[k].y, vb[k].z, vb[k].w};
                        const uint32_t pw[4] = {pp.x, pp.y, pp.z, pp.w};
                        if (pos >= c0 && pos < c0 + 8) {  // the new cell: LDS copy
                            const int l = pos - c0;
                            vw[l >> 1] = (vw[l >> 1] & (0xffff0000u >> (16 * (l & 1)))) | ((uint32_t)v16[d] << (16 * (l & 1)));
                        }
#pragma unroll
                        for (int q = 0; q < 4; ++q) acc[q] = pk_fma_w(vw[q], pw[q], acc[q]);
                    }
                }
            }
        } else {  // one V chunk per iteration (the fused kernels)
            for (int it = 0; it < n_it; ++it) {  // VPF prefetched iterations, then global loads
                const int c0 = 32 * it + 8 * j;
                uint4 vv;
                if (it < VPF) {
#pragma unroll
                    for (int k = 0; k < VPF; ++k)
                        if (k == it) vv = vpre[ii][k];
                } else if (VPOST > 0 && it < VPF + VPOST) {
#pragma unroll
                    for (int k = 0; k < (VPOST > 0 ? VPOST : 1); ++k)
                        if (k == it - VPF) vv = vpost[ii][k];
                } else {
                    vv = *(const uint4 *)(vr + c0);
                }
                const uint4 pp = *(const uint4 *)(p16 + c0);
                uint32_t vw[4] = {vv.x, vv.y, vv.z, vv.w};
                const uint32_t pw[4] = {pp.x, pp.y, pp.z, pp.w};
                if (pos >= c0 && pos < c0 + 8) {  // the new cell: LDS copy
                    const int l = pos - c0;
                    vw[l >> 1] = (vw[l >> 1] & (0xffff0000u >> (16 * (l & 1)))) | ((uint32_t)v16[d] << (16 * (l & 1)));
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] = pk_fma_w(vw[k], pw[k], acc[k]);
            }
        }
        const float o = f16x8_reduce_quad(acc);  // accumulators j = 0..3 of output d: one quad of lanes
        if (j == 0) {
            const float ov = bad ? __builtin_nanf("") : o;
            if (OUT_WT) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(out + d), "v"(ov) : "memory");
            else out[d] = ov;
        }
    }
}

}  // namespace kq
