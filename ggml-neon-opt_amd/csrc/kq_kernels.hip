// kq_kernels.hip — gfx950 (CDNA4, wave64) kernels for the ggml K-quant MUL_MAT hot path.
//
// Replaces, on the device, the reference's
//   ggml_vec_dot_q4_K_q8_K (NEON, README.md:686-779; optimized README.md:1455-1480),
//   ggml_vec_dot_q6_K_q8_K (README.md:369, out.folded:160), the Q5_K sibling,
//   quantize_row_q8_K_ref (out.folded:184-186) and the row loop of
//   ggml_compute_forward_mul_mat / _one_chunk (README.md:136-137, ggml-cpu.c:1389/:1194).
//
// Numerics contract: every integer quantity (Q8_K qs/bsums/d, 6-bit scale and
// min unpack, nibble x int8 dots, bsums x mins) is bit-exact; the per-row fp32
// accumulation is carried out in superblock order with exactly the reference's
// operations (fmsub/fmadd, README.md:551/:614), so outputs are bit-identical to
// the reference NEON function. The kernel file is compiled with
// -ffp-contract=off: only the explicit fmaf() calls fuse.
//
// Work decomposition (decode GEMV, HBM-bound; details at kq_gemv below): a
// workgroup owns 8-row tasks, its 4 waves split each task's superblocks into
// K-ranges, weights stream into per-wave LDS rings by LDS-DMA
// (global_load_lds_dwordx4), 8 lanes own one superblock and dot their 32 quants
// against LDS activations with v_dot4_i32_i8, 3 DPP adds reduce an octet, and
// the reference's fp32 chain runs in superblock order (wave 0 in registers,
// waves 1-3 through exact LDS records).
#include "kq_device.h"

// Diagnostics (timing only: MI355X_GEMV_DIAG bits, per-wave stamps) exist only in
// experiment builds (-DKQ_GEMV_DIAG=1); in the product build they compile out.
#ifndef KQ_GEMV_DIAG
#define KQ_GEMV_DIAG 0
#endif
#if KQ_GEMV_DIAG
#define GDIAG(a) ((a).diag)
#define GSTAMPS(a) ((a).stamps)
#else
#define GDIAG(a) 0
#define GSTAMPS(a) ((uint64_t *)nullptr)
#endif

namespace kq {

// ------------------------------------------------------------------ Q8_K quantize kernel
// One wave per superblock; y rows are contiguous (nb blocks of 292 B).
__global__ void __launch_bounds__(WG_THREADS) kq_quantize_q8K(const float *__restrict__ x, int64_t x_stride,
                                                              uint8_t *__restrict__ y, int nb, int64_t nblocks) {
    const int lane = threadIdx.x & 63;
    const int64_t bi = (int64_t)blockIdx.x * WAVES_PER_WG + (threadIdx.x >> 6);
    if (bi >= nblocks) return;
    const int64_t row = bi / nb;
    const int b = (int)(bi - row * nb);
    const float *xb = x + row * x_stride + (int64_t)b * QK;
    const Q8Lane q = quant_block_wave(xb, lane);
    uint8_t *yb = y + bi * 292;
    *(uint32_t *)(yb + 4 + 4 * lane) = q.qs4;
    if ((lane & 3) == 0) *(int16_t *)(yb + 260 + 2 * (lane >> 2)) = (int16_t)q.bsum;
    if (lane == 0) *(float *)yb = q.d;
}

struct StepInfo {
    int m, row0, rows;
};

// Task t -> (matrix, first row, rows in task). All inputs are wave-uniform, so this
// runs on the scalar unit with scalar loads from the kernel-argument segment.
__device__ __forceinline__ StepInfo task_info(const GemvArgs &a, int t) {
    int m = 0;
#pragma unroll
    for (int i = 1; i < MI355X_MAX_FUSED; ++i)
        if (i < a.n_desc && t >= a.task_prefix[i]) m = i;
    StepInfo si;
    si.m = m;
    si.row0 = (t - a.task_prefix[m]) * a.R;
    const int left = a.n_rows[m] - si.row0;
    si.rows = left < a.R ? left : a.R;
    return si;
}


// K-range of wave w when a task's nb superblocks are split over the 4 waves.
__host__ __device__ __forceinline__ void wave_krange(int nb, int w, int &lo, int &cnt) {
    const int q = nb / WAVES_PER_WG, r = nb % WAVES_PER_WG;
    cnt = q + (w < r ? 1 : 0);
    lo = w * q + (w < r ? w : r);
}

// Per-task state of a lane: consumer row (octet g) and the two DMA pieces it fetches.
struct TaskLane {
    int m, type, bb, P, row0, rows;  // wave-uniform
    bool valid;                      // octet g maps to a real row
    const uint8_t *crow;             // consumer row base
    const uint8_t *drow[2];          // DMA piece rows (instruction 0: lane, 1: lane + 64)
    int dj[2];                       // DMA piece index within the block
    bool dact1;                      // lane active in DMA instruction 1

    template <int TMASK>
    __device__ __forceinline__ void load(const GemvArgs &a, int t, int lane) {
        const StepInfo si = task_info(a, t);
        m = si.m;
        row0 = si.row0;
        rows = si.rows;
        type = a.type[m];
        bb = block_bytes(type);
        P = pieces_of(type);
        const int g = lane >> 3;
        valid = g < rows;
        const uint8_t *w = a.w[m];
        const int64_t rs = a.row_stride[m];
        crow = w + (int64_t)(row0 + (valid ? g : rows - 1)) * rs;
        if (TMASK == 1) P = 9;  // compile-time divisor below
        if (TMASK == 4) P = 14;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int pi = lane + 64 * i;
            const int gi = pi / P;
            dj[i] = pi - gi * P;
            drow[i] = w + (int64_t)(row0 + (gi < rows ? gi : rows - 1)) * rs;
        }
        dact1 = lane + 64 < 8 * P;
    }
};

// Decode / small-batch GEMV: dst[c][row] for NCOL activation columns.
//
// Work: a workgroup owns 8-row tasks (octet g of every wave <-> row row0+g). The
// task's nb superblocks are split into 4 contiguous K-ranges, one per wave.
// Weights: each wave streams its range through a ring of D LDS slots; a step is
// one superblock of each of the 8 rows, fetched as 16-B pieces by two
// global_load_lds_dwordx4 (every piece 16-B aligned, so no access can cross a
// page) and waited for with a counted s_waitcnt vmcnt. The loop is not unrolled:
// the slot is an LDS address, so prefetch depth costs no registers and the code
// stays small (the instruction footprint dominates short launches).
// Activations: each wave stages only its own K-range: f32 by LDS-DMA, quantized
// in place into raw 292-B Q8_K blocks (FUSEDQ), or raw Q8_K bytes by LDS-DMA.
// Chain: wave 0 keeps the fp32 chain of its range in registers; waves 1-3 store
// exact records; after one s_barrier per task (no vmcnt drain) wave 0 continues
// the chain through them in superblock order and stages the 8 results.
template <int NCOL, bool FUSEDQ, bool DEBUG, int TMASK>
__global__ void __launch_bounds__(WG_THREADS) kq_gemv(const GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint64_t st0 = GSTAMPS(a) ? __builtin_amdgcn_s_memrealtime() : 0;
    if (GDIAG(a) & 2) return;  // diagnostics: empty launch (same grid / LDS)
    const int nb = a.nb, D = a.ring;
    constexpr int SLOT = slot_bytes(TMASK);
    const LdsLayout L = lds_layout(NCOL, nb, a.out_per_wg, FUSEDQ, SLOT, D);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably uniform
    const int g = lane >> 3, p = lane & 7;
    const int spw = L.spw;
    uint8_t *ring = smem + L.ring + wave * D * SLOT;
    uint8_t *act = smem + L.act + wave * L.act_per_wave;
    Rec *recs = (Rec *)(smem + L.recs);      // [slot 2][wave-1 3][NCOL][row 8][spw]
    float *outs = (float *)(smem + L.outs);  // [task k][NCOL][row 8], wave 0 only

    const int col0 = blockIdx.y * NCOL;
    const int ncol = (a.m_total - col0) < NCOL ? (a.m_total - col0) : NCOL;
    const int t0 = blockIdx.x, tstride = gridDim.x;
    const int my_tasks = a.tasks_total > t0 ? (a.tasks_total - t0 + tstride - 1) / tstride : 0;
    int lo, S;
    wave_krange(nb, wave, lo, S);
    const int Q = my_tasks * S;
    // byte offset of each column's first raw Q8_K block inside its LDS region
    int actsh[NCOL];
#pragma unroll
    for (int c = 0; c < NCOL; ++c)
        actsh[c] = FUSEDQ ? 0 : (int)((uintptr_t)(a.xq + (int64_t)(col0 + c) * a.xq_col_stride + (int64_t)lo * 292) & 15);

    // ---- issue cursor: step q -> (task k, step s); DMA into slot q % D
    TaskLane it;
    int ik = 0, is = 0;
    uint8_t *const ring_end = ring + D * SLOT;
    uint8_t *islot = ring;  // slot of the next issued step (wraps)
    auto issue = [&]() {
        const int blk = lo + is;
        uint8_t *slot = islot;
        const int type = TMASK == 1 ? Q4_K : TMASK == 4 ? Q6_K : it.type;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint8_t *src;
            if (type == Q6_K) {
                const uintptr_t blkp = (uintptr_t)(it.drow[i] + (int64_t)blk * 210);
                src = (const uint8_t *)(blkp & ~(uintptr_t)15) + 16 * it.dj[i];
            } else {
                src = it.drow[i] + (int64_t)blk * it.bb + 16 * it.dj[i];
            }
            if (i == 0 || it.dact1) dma16(src, (LDS void *)(slot + 1024 * i));
        }
        islot = islot + SLOT == ring_end ? ring : islot + SLOT;
        if (++is == S) {
            is = 0;
            if (++ik < my_tasks) it.load<TMASK>(a, t0 + ik * tstride, lane);
        }
    };

    // ---- compute cursor
    TaskLane ct;
    int ck = 0, cs = 0;
    float acc[NCOL];
#pragma unroll
    for (int c = 0; c < NCOL; ++c) acc[c] = 0.f;

    auto task_end = [&]() {
        // every wave: make this task's records visible, then meet the other waves
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (wave == 0) {
            const Rec *rs = recs + (ck & 1) * (WAVES_PER_WG - 1) * NCOL * 8 * spw;
            const int ctype = TMASK == 1 ? Q4_K : TMASK == 4 ? Q6_K : ct.type;
#pragma unroll
            for (int c = 0; c < NCOL; ++c) {
                if (c < ncol) {
                    float v = acc[c];
                    for (int w = 1; w < WAVES_PER_WG; ++w) {
                        int wlo, wcnt;
                        wave_krange(nb, w, wlo, wcnt);
                        const Rec *rw = rs + (((w - 1) * NCOL + c) * 8 + g) * spw;
                        for (int i = 0; i < wcnt; ++i) v = chain_step(ctype, rw[i], v);
                    }
                    if (!DEBUG && p == 0) outs[(ck * NCOL + c) * 8 + g] = v;
                    acc[c] = 0.f;
                }
            }
        }
    };

    const uint8_t *cslot = ring;  // slot of the next computed step (wraps)
    auto compute = [&]() {
        const int blk = lo + cs;
        const int type = TMASK == 1 ? Q4_K : TMASK == 4 ? Q6_K : ct.type;
        const uint8_t *slot = cslot;
        cslot = cslot + SLOT == ring_end ? ring : cslot + SLOT;
        if (!(GDIAG(a) & 8)) {  // diagnostics bit 3: stream weights only, no arithmetic
        uint32_t sh = 0;
        if (type == Q6_K) sh = (uint32_t)((uintptr_t)(ct.crow + (int64_t)blk * 210) & 15u);
        Regs rr;
        lds_block<TMASK>(rr, slot + g * ct.P * 16, sh, type, p);
        Rec *rw = recs + (((ck & 1) * (WAVES_PER_WG - 1) + (wave - 1)) * NCOL * 8 + g) * spw + cs;
#pragma unroll
        for (int c = 0; c < NCOL; ++c) {
            if (c < ncol) {
                const uint8_t *ab = act + c * L.act_col + actsh[c] + cs * 292;  // raw Q8_K block
                int isum = 0, imin = 0;
                uint32_t dh = rr.dh;
                lane_partials<TMASK>(rr, ab + 4, (const int16_t *)(ab + 260), type, p, isum, imin, dh);
                isum = octet_sum(isum);
                imin = octet_sum(imin);
                const float yd = *(const float *)ab;
                const Rec rec = make_rec<TMASK>(type, isum, imin, rr, dh, yd);
                if (wave == 0) acc[c] = chain_step(type, rec, acc[c]);  // all 8 lanes of the octet
                else if (p == 0) rw[c * 8 * spw] = rec;
                if (DEBUG && c == 0 && p == 0 && ct.valid) {
                    const int64_t o = ((int64_t)(ct.row0 + g) * nb + blk) * 2;
                    a.dbg[o] = isum;
                    a.dbg[o + 1] = imin;
                }
            }
        }
        }
        if (++cs == S) {
            task_end();
            cs = 0;
            if (++ck < my_tasks) ct.load<TMASK>(a, t0 + ck * tstride, lane);
        }
    };

    // ---- prologue: activation K-range of this wave -> LDS, first D weight steps in flight
    const int tfirst = t0 < a.tasks_total ? t0 : a.tasks_total - 1;
    it.load<TMASK>(a, tfirst, lane);
    ct = it;
    uint64_t sa = 0, sb = 0, sc = 0;
    if (GSTAMPS(a)) sa = __builtin_amdgcn_s_memrealtime();
    if (FUSEDQ) {
        const float *xc = a.x + (int64_t)col0 * a.x_col_stride + (int64_t)lo * QK;
        for (int i = 0; i < S; ++i) dma16(xc + (int64_t)i * QK + 4 * lane, (LDS void *)(act + 1024 * i));
    } else {
        for (int c = 0; c < ncol; ++c) {
            const uintptr_t start = (uintptr_t)(a.xq + (int64_t)(col0 + c) * a.xq_col_stride + (int64_t)lo * 292);
            const uint8_t *s16 = (const uint8_t *)(start & ~(uintptr_t)15);
            const int np = (int)((S * 292 + (start & 15) + 15) / 16);
            for (int k = 0; k * 64 < np; ++k) {
                const int pc = k * 64 + lane;
                if (pc < np) dma16(s16 + 16 * pc, (LDS void *)(act + c * L.act_col + 1024 * k));
            }
        }
    }
    const int pre = Q < D ? Q : D;
    for (int j = 0; j < pre; ++j) issue();
    if (GSTAMPS(a)) sb = __builtin_amdgcn_s_memrealtime();
    vm_wait_steps(pre);  // activation DMAs are older than the ring's 2*pre
    if (GSTAMPS(a)) sc = __builtin_amdgcn_s_memrealtime();
    if (FUSEDQ) {
        // quantize in place: block i's f32 staging [1024i, 1024i+1024) -> raw Q8_K [292i, 292i+292)
#pragma unroll 1
        for (int i = 0; i < S; ++i) {
            const f32x4 v = *(const f32x4 *)(act + 1024 * i + 16 * lane);
            const Q8Lane q = quant_values_wave(v, lane);
            uint8_t *qb = act + 292 * i;
            *(uint32_t *)(qb + 4 + 4 * lane) = q.qs4;
            if ((lane & 3) == 0) *(int16_t *)(qb + 260 + 2 * (lane >> 2)) = (int16_t)q.bsum;
            if (lane == 0) *(float *)qb = q.d;
        }
    }
    wave_lds_fence();  // this wave's staged activations before its own reads
    uint64_t st1 = 0, st2 = 0;
    if (GSTAMPS(a)) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        st1 = __builtin_amdgcn_s_memrealtime();
    }
    if (GDIAG(a) & 1) return;  // diagnostics: prologue only

    // ---- main loop: wait for step q's slot, compute it, refill the slot with step q+D
    if (S > 0) {
#pragma unroll 1
        for (int q = 0; q < Q; ++q) {
            // steps issued after q: min(D, Q - q) - 1 (debug stores also count: wait for all)
            vm_wait_steps(DEBUG ? 0 : (Q - q < D ? Q - q : D) - 1);
            compute();
            if (q + D < Q) issue();
        }
    } else {
        for (int k = 0; k < my_tasks; ++k) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (GSTAMPS(a)) st2 = __builtin_amdgcn_s_memrealtime();

    // ---- flush wave 0's staged results: task k -> rows row0..row0+7, NCOL columns
    if (!DEBUG && wave == 0 && my_tasks > 0) {
        wave_lds_fence();
        for (int k = 0; k < my_tasks; ++k) {
            const StepInfo si = task_info(a, t0 + k * tstride);
            const int c = lane >> 3, r = lane & 7;  // NCOL * 8 <= 64
            if (c < ncol && r < si.rows)
                a.y[si.m][(int64_t)(col0 + c) * a.y_col_stride[si.m] + si.row0 + r] = outs[k * NCOL * 8 + lane];
        }
    }
    if (GSTAMPS(a)) {
        const int64_t o = ((int64_t)blockIdx.x * WAVES_PER_WG + wave) * 8;
        if (lane == 0 && o + 7 < a.stamps_cap) {
            const uint64_t st3 = __builtin_amdgcn_s_memrealtime();
            GSTAMPS(a)[o] = st0;
            GSTAMPS(a)[o + 1] = st1;
            GSTAMPS(a)[o + 2] = st2;
            GSTAMPS(a)[o + 3] = st3;
            GSTAMPS(a)[o + 4] = sa;
            GSTAMPS(a)[o + 5] = sb;
            GSTAMPS(a)[o + 6] = sc;
        }
    }
}

// ------------------------------------------------------------------ explicit instances
#define KQ_GEMV_INST(NC, FQ, DB, TM) template __global__ void kq_gemv<NC, FQ, DB, TM>(const GemvArgs a);
#define KQ_GEMV_INST_TM(NC, FQ, DB) KQ_GEMV_INST(NC, FQ, DB, 1) KQ_GEMV_INST(NC, FQ, DB, 4) KQ_GEMV_INST(NC, FQ, DB, 7)

KQ_GEMV_INST_TM(1, true, false)
KQ_GEMV_INST_TM(1, false, false)
KQ_GEMV_INST_TM(2, false, false)
KQ_GEMV_INST_TM(4, false, false)
KQ_GEMV_INST_TM(8, false, false)
KQ_GEMV_INST_TM(1, false, true)


// ------------------------------------------------------------------ streaming ceiling (diagnostic)
// mi355x_debug_stream: the bytes of a buffer pulled into per-wave LDS rings by LDS-DMA
// (nt), 2-KB steps, 4 in flight, 12 waves per CU, one contiguous range per wave, no
// arithmetic -- the time a decode GEMV launch of that many weight bytes could approach
// (tools/stream_size.hip; bench.py gemv_large "stream_us"). Not on any product path.
__global__ void __launch_bounds__(256) kq_stream_ceiling(const uint8_t *buf, int64_t per_wave, int waves_total,
                                                         uint32_t *sink) {
    constexpr int IPS = 2, D = 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = blockIdx.x * 4 + wave;
    if (gw >= waves_total) return;
    uint8_t *ring = smem + wave * D * IPS * 1024;
    const uint8_t *src = buf + (int64_t)gw * per_wave;
    const int T = (int)(per_wave / (IPS * 1024));
    for (int t = 0; t < D && t < T; ++t)
#pragma unroll
        for (int i = 0; i < IPS; ++i)
            dma16_nt(src + (int64_t)t * IPS * 1024 + i * 1024 + 16 * lane, (LDS void *)(ring + (t % D) * IPS * 1024 + 1024 * i));
    uint32_t acc = 0;
    for (int t = 0; t < T; ++t) {
        if (T - t >= D)
            vm_wait<IPS * (D - 1)>();
        else
            vm_wait<0>();
        acc += *(volatile uint32_t *)(ring + (t % D) * IPS * 1024 + 4 * lane);
        if (t + D < T)
#pragma unroll
            for (int i = 0; i < IPS; ++i)
                dma16_nt(src + (int64_t)(t + D) * IPS * 1024 + i * 1024 + 16 * lane,
                         (LDS void *)(ring + (t % D) * IPS * 1024 + 1024 * i));
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

}  // namespace kq
