// kq_chain.hip — persistent decode chain: one launch runs every MUL_MAT stage of a
// token's graph (ggml_backend_cpu_graph_compute's node loop, ggml-cpu.cpp:186,
// README.md:162, with each node's ggml_compute_forward_mul_mat, ggml-cpu.c:1389).
//
// Why: a decode GEMV of TinyLlama size streams 2.4-6.5 MB, ~1 us of HBM time, but
// a launch costs ~4.4 us (wave start spread, activation fetch, first weight DMA
// latency). Inside one persistent launch
//  * every wave prefetches its first ring of stage s+1 weights (which do not depend
//    on the activation) before it waits for stage s+1's activation, so the weight
//    latency hides behind the hand-off;
//  * the hand-off is the activation fetch itself: producers store each output as a
//    {value, tag} pair written through to memory (sc0 sc1), consumers re-read
//    (sc0 sc1) until every pair of their blocks carries this launch's tag. No
//    counter barrier, no L2 writeback/invalidate (measured 1.6 us/stage vs 2.6 us
//    for a counter barrier and 6-9 us with agent-scope fences: tools/barrier_bench.hip).
//
// Per stage and per wave the arithmetic is kq_rows' (kq_rows.hip): same wave
// split, same quad partials, same records and fp32 chain replay per row, so every
// output is bit-identical to the per-launch path and to ggml_vec_dot_q4_K_q8_K.
//
// The grid is one workgroup per CU and every workgroup must be resident (they
// wait on each other): the host launches exactly num_cus workgroups with more than
// half the LDS of a CU. A hand-off that does not complete within ~20 ms sets
// sync[2] and proceeds (bounded spin; the host reports MI355X_E_TIMEOUT).
#include "kq_rows_device.h"

namespace kq {

namespace {

constexpr uint64_t kHandoffTicks = 2000000;  // s_memrealtime is 100 MHz: 20 ms

// The stage table through the constant address space: uniform scalar loads (s_load)
// into SGPRs instead of per-lane vector loads.
typedef const ChainStage __attribute__((address_space(4))) *StagePtr;

__device__ __forceinline__ u32x4 load_sys16(const uint32_t *p) {
    u32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(r) : "v"(p) : "memory");
    return r;
}

__device__ __forceinline__ void store_sys8(uint32_t *p, uint32_t v, uint32_t tag) {
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    const u2 w = {v, tag};
    asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(w) : "memory");
}

// Wave-uniform state of a wave's weight stream; survives a stage boundary so the
// next stage's first ring is fetched before its activation is ready.
struct Stream {
    const uint8_t *s16, *last16;
    int T, it, islot;
    uint32_t mis;
};

__device__ __forceinline__ WaveWork stage_work(StagePtr st, int gw) {
    WaveWork ww;
    int m = 0;
#pragma unroll
    for (int i = 1; i < MI355X_MAX_FUSED; ++i)
        if (i < st->n_desc && gw >= st->wave_prefix[i]) m = i;
    ww.m = m;
    const int j = gw - st->wave_prefix[m];
    const int base = st->rbase[m], rem = st->rrem[m];
    ww.r0 = j * base + (j < rem ? j : rem);
    ww.nrows = gw < st->waves_total ? base + (j < rem ? 1 : 0) : 0;
    return ww;
}

template <int TYPE>
__device__ __forceinline__ Stream stream_open(StagePtr st, const WaveWork &ww) {
    constexpr int BSZ = block_bytes(TYPE);
    Stream S;
    const int G = ww.nrows * st->nb;
    S.T = (G + ROWS_SB - 1) / ROWS_SB;
    const uint8_t *src = st->w[ww.m] + (int64_t)ww.r0 * st->nb * BSZ;
    S.mis = (uint32_t)((uintptr_t)src & 15u);
    S.s16 = src - S.mis;
    S.last16 = G > 0 ? (const uint8_t *)((uintptr_t)(src + (int64_t)G * BSZ - 1) & ~(uintptr_t)15) : S.s16;
    S.it = 0;
    S.islot = 0;
    return S;
}

template <int TYPE>
__device__ __forceinline__ void stream_issue(Stream &S, uint8_t *ring, int lane) {
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int GRAN = rows_gran(TYPE);
    constexpr int NI = rows_ni(TYPE);
    constexpr int SLOT = rows_slot(TYPE);
    constexpr int D = rows_depth(TYPE);
    const uint8_t *base = S.s16 + (int64_t)S.it * (ROWS_SB * BSZ) + 16 * lane;
    uint8_t *islot = ring + S.islot;
    if (S.it + 1 < S.T) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
            if (i + 1 < NI || lane < GRAN - 64 * (NI - 1)) dma16_nt(base + 1024 * i, (LDS void *)(islot + 1024 * i));
    } else {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const uint8_t *p = base + 1024 * i;
            if (i + 1 < NI || lane < GRAN - 64 * (NI - 1))
                dma16_nt(p < S.last16 ? p : S.last16, (LDS void *)(islot + 1024 * i));
        }
    }
    S.islot = S.islot + SLOT == D * SLOT ? 0 : S.islot + SLOT;
    ++S.it;
}

// Open the wave's stream of stage `st` and fill its ring (weights only).
template <int TYPE>
__device__ __forceinline__ void stream_prefetch(Stream &S, StagePtr st, const WaveWork &ww, uint8_t *ring,
                                                int lane) {
    S = stream_open<TYPE>(st, ww);
    constexpr int D = rows_depth(TYPE);
    while (S.it < D && S.it < S.T) stream_issue<TYPE>(S, ring, lane);
}

// The stage's Q8_K activation into LDS (Q8L blocks), 16 lanes per superblock,
// 4 superblocks per wave per pass. From the bus: poll until every pair of the
// wave's blocks carries `tag`.
struct Tm {  // diagnostics of one stage (wave 0): s_memrealtime stamps, poll count
    uint64_t poll0, ok, quant, comp, flush;
    int npoll;
};

__device__ __forceinline__ const uint32_t *poll_addr(StagePtr st, int wave, int lane, int i) {
    const int nb = st->nb;
    const int bi = 4 * ROWS_WAVES * i + 4 * wave + (lane >> 4);
    const int b = bi < nb ? bi : nb - 1;
    return st->xbus + 2 * ((int64_t)b * QK + 16 * (lane & 15));
}

__device__ __forceinline__ void stage_activation(StagePtr st, uint8_t *act, int wave, int lane, uint32_t tag,
                                                 uint32_t *flag, Tm &tm) {
    constexpr int PASS = 4 * ROWS_WAVES;
    const int nb = st->nb;
#pragma unroll 1
    for (int i = 0; PASS * i + 4 * wave < nb; ++i) {
        const int bi = PASS * i + 4 * wave + (lane >> 4);
        const int b = bi < nb ? bi : nb - 1;
        u32x4 v[4];
        if (st->xbus) {
            const uint32_t *xp = poll_addr(st, wave, lane, i);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            if (i == 0) tm.poll0 = t0;
            u32x4 p[8];
            for (;;) {
                if (i == 0) ++tm.npoll;
#pragma unroll
                for (int k = 0; k < 8; ++k) p[k] = load_sys16(xp + 4 * k);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                bool ok = true;
#pragma unroll
                for (int k = 0; k < 8; ++k) ok = ok && p[k].y == tag && p[k].w == tag;
                if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
                    if (i == 0) tm.ok = __builtin_amdgcn_s_memrealtime();
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > kHandoffTicks) {
                    if (lane == 0) atomicOr(flag, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = u32x4{p[2 * k].x, p[2 * k].z, p[2 * k + 1].x, p[2 * k + 1].z};
        } else {
            const float *xp = st->x + (int64_t)b * QK + 16 * (lane & 15);
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = *(const u32x4 *)(xp + 4 * k);
        }
        if (bi < nb) quant16_store(v, lane & 15, act + Q8L_STRIDE * b);
    }
    tm.quant = __builtin_amdgcn_s_memrealtime();
}

// Stage compute of one wave: kq_rows' main loop and flush (rows_body, kq_rows.hip),
// continuing the stream whose first ring stream_prefetch issued.
template <int TYPE>
__device__ __forceinline__ void stage_rows(const ChainArgs &a, StagePtr st, const WaveWork &ww, Stream &S,
                                           uint8_t *smem, int wave, int lane, uint32_t tag, Tm &tm) {
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int NI = rows_ni(TYPE);
    constexpr int SLOT = rows_slot(TYPE);
    constexpr int D = rows_depth(TYPE);
    const int nb = st->nb, bR = st->bR;
    const int q = lane >> 2, s = lane & 3;
    uint8_t *const ring = smem + a.ring + wave * a.ring_stride;
    uint8_t *const ring_end = ring + D * SLOT;
    Rec *const recs = (Rec *)(smem + a.recs + wave * a.recs_stride);
    float *const outs = (float *)(smem + a.outs + wave * a.outs_stride);
    const uint8_t *const actq = smem + a.act;
    const int G = ww.nrows * nb;
    const int T = S.T;

    while (S.it < D && S.it < T) stream_issue<TYPE>(S, ring, lane);  // (already full unless T < D)
    int io = q, rr = 0;
    while (io >= nb) {
        io -= nb;
        ++rr;
    }
    int bend = bR * nb < G ? bR * nb : G;
    int brow = 0;
    const uint8_t *cslot = ring;
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
        // steps t .. S.it-1 are in flight and nothing else (the activation wait drained
        // older loads); keep the younger ones going
        if (T - t >= D) vm_wait<NI * (D - 1)>();
        else vm_wait_k<NI>(T - t - 1);
        if (ROWS_SB * t + q < G) {
            const uint8_t *blk = cslot + S.mis + q * BSZ;
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
                    rec.c = h2f(r.dh) * yd;
                    rec.e = 0.f;
                } else {
                    rec.a = isum;
                    rec.b = imin;
                    rec.c = yd * h2f(r.dh & 0xffffu);
                    rec.e = yd * h2f(r.dh >> 16);
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
        if (S.it < T) stream_issue<TYPE>(S, ring, lane);
        if (ROWS_SB * (t + 1) >= bend) {
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
    tm.comp = __builtin_amdgcn_s_memrealtime();
    if (ww.nrows > 0) {
        wave_lds_fence();
        float *y = st->y[ww.m] + ww.r0;
        uint32_t *bus = st->bus[ww.m];
        if (bus) {  // the hand-off copy first: it is on the next stage's critical path
            bus += 2 * (int64_t)ww.r0;
            for (int k = 0; k < ww.nrows; k += 64)
                if (k + lane < ww.nrows) store_sys8(bus + 2 * (k + lane), __float_as_uint(outs[k + lane]), tag);
        }
        for (int k = 0; k < ww.nrows; k += 64)
            if (k + lane < ww.nrows) y[k + lane] = outs[k + lane];
    }
    tm.flush = __builtin_amdgcn_s_memrealtime();
}

template <int TYPE>
__device__ __forceinline__ void prefetch_as(Stream &S, StagePtr st, const WaveWork &ww, uint8_t *ring, int lane) {
    stream_prefetch<TYPE>(S, st, ww, ring, lane);
}

}  // namespace

__global__ void __launch_bounds__(ROWS_WAVES * 64) kq_chain(const ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = wave * gridDim.x + blockIdx.x;
    uint8_t *const ring = smem + a.ring + wave * a.ring_stride;
    // this launch's tag: one more than the last launch's (bumped by the last workgroup out)
    uint32_t tag;
    {
        u32x4 e = load_sys16(a.sync);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tag = __builtin_amdgcn_readfirstlane(e.x) + 1u;
    }
    const bool stamps = a.stamps != nullptr;

    const StagePtr stages = (StagePtr)a.st;
    Stream S;
    int type;
    WaveWork ww;
    {
        const StagePtr s0 = stages;
        ww = stage_work(s0, gw);
        type = s0->type[ww.m];
        if (type == Q6_K) prefetch_as<Q6_K>(S, s0, ww, ring, lane);
        else if (type == Q5_K) prefetch_as<Q5_K>(S, s0, ww, ring, lane);
        else prefetch_as<Q4_K>(S, s0, ww, ring, lane);
    }

#pragma unroll 1
    for (int si = 0; si < a.n_stages; ++si) {
        const StagePtr st = stages + si;
        Tm tm = {0, 0, 0, 0, 0, 0};
        stage_activation(st, smem + a.act, wave, lane, tag, a.sync + 2, tm);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // Q8_K row complete
        const uint64_t t_x = stamps ? __builtin_amdgcn_s_memrealtime() : 0;
        if (type == Q6_K) stage_rows<Q6_K>(a, st, ww, S, smem, wave, lane, tag, tm);
        else if (type == Q5_K) stage_rows<Q5_K>(a, st, ww, S, smem, wave, lane, tag, tm);
        else stage_rows<Q4_K>(a, st, ww, S, smem, wave, lane, tag, tm);
        if (si + 1 < a.n_stages) {  // next stage's weights do not wait for its activation
            const StagePtr nx = stages + si + 1;
            ww = stage_work(nx, gw);
            type = nx->type[ww.m];
            if (type == Q6_K) prefetch_as<Q6_K>(S, nx, ww, ring, lane);
            else if (type == Q5_K) prefetch_as<Q5_K>(S, nx, ww, ring, lane);
            else prefetch_as<Q4_K>(S, nx, ww, ring, lane);
        }
        if (stamps && wave == 0 && lane == 0) {
            const int64_t o = ((int64_t)blockIdx.x * a.n_stages + si) * 8;
            if (o + 7 < a.stamps_cap) {
                a.stamps[o] = t_x;
                a.stamps[o + 1] = tm.comp;
                a.stamps[o + 2] = tm.flush;
                a.stamps[o + 3] = __builtin_amdgcn_s_memrealtime();  // next stage's ring issued
                a.stamps[o + 4] = tm.poll0;
                a.stamps[o + 5] = tm.ok;
                a.stamps[o + 6] = (uint64_t)tm.npoll;
                a.stamps[o + 7] = tm.quant;
            }
        }
        asm volatile("s_barrier" ::: "memory");  // every wave is done with this stage's activation
    }
    // the last workgroup out publishes this launch's tag as the epoch
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t done = __hip_atomic_fetch_add(a.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done + 1 == gridDim.x) {
            __hip_atomic_store(a.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sync, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace kq
