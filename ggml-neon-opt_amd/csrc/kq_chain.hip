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
// Roles: per stage the first `pollers` waves of a workgroup (1-6, by K) fetch and
// quantize the activation and stream no weights, so their polls never queue behind
// weight DMAs (vector-memory returns are in order); the other waves stream rows.
// The stage table is read one dword per lane and fields come from v_readlane:
// the next stage's descriptor is loaded a whole stage ahead.
//
// The grid is one workgroup per CU and every workgroup must be resident (they
// wait on each other): the host launches exactly num_cus workgroups with more than
// half the LDS of a CU. A hand-off that does not complete within ~20 ms sets
// sync[2] and proceeds (bounded spin; the host reports MI355X_E_TIMEOUT).
#include "kq_rows_device.h"

namespace kq {

namespace {

constexpr uint64_t kHandoffTicks = 2000000;  // s_memrealtime is 100 MHz: 20 ms

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

// Stage descriptor, one dword per lane (lane i <- dword i of the 256-B table slot).
// Loaded by inline asm (invisible to the compiler's waitcnt bookkeeping); the caller
// guarantees completion (an s_waitcnt covering it) before desc_pin.
__device__ __forceinline__ uint32_t desc_load(const uint8_t *table, int si, int lane) {
    uint32_t v;
    const uint32_t *p = (const uint32_t *)(table + (int64_t)si * kChainSlotBytes) + lane;
    asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}

#define CH_OFF(f) ((int)(offsetof(ChainStage, f) / 4))

__device__ __forceinline__ int rl(uint32_t v, int i) { return __builtin_amdgcn_readlane((int)v, i); }
__device__ __forceinline__ uint64_t rl64(uint32_t v, int i) {
    return (uint64_t)(uint32_t)rl(v, i) | ((uint64_t)(uint32_t)rl(v, i + 1) << 32);
}

// A wave's view of one stage: its role, rows and the resolved matrix.
struct WaveStage {
    int nb, bR, pollers, type;
    WaveWork ww;
    const uint8_t *w;
    float *y;
    uint32_t *bus;
    const float *x;
    const uint32_t *xbus;
};

__device__ __forceinline__ WaveStage resolve(uint32_t dv, int wave) {
    WaveStage r;
    r.nb = rl(dv, CH_OFF(nb));
    r.bR = rl(dv, CH_OFF(bR));
    r.pollers = rl(dv, CH_OFF(pollers));
    const int n_desc = rl(dv, CH_OFF(n_desc));
    const int waves_total = rl(dv, CH_OFF(waves_total));
    // streaming waves: gw = (wave - pollers) * gridDim.x + blockIdx.x (spread over every CU)
    const int gw = wave >= r.pollers ? (wave - r.pollers) * (int)gridDim.x + (int)blockIdx.x : 0x7fffffff;
    int m = 0;
#pragma unroll
    for (int i = 1; i < MI355X_MAX_FUSED; ++i)
        if (i < n_desc && gw >= rl(dv, CH_OFF(wave_prefix) + i)) m = i;
    const int j = gw - rl(dv, CH_OFF(wave_prefix) + m);
    const int base = rl(dv, CH_OFF(rbase) + m), rem = rl(dv, CH_OFF(rrem) + m);
    r.ww.m = m;
    r.ww.r0 = j * base + (j < rem ? j : rem);
    r.ww.nrows = gw < waves_total ? base + (j < rem ? 1 : 0) : 0;
    r.type = rl(dv, CH_OFF(type) + m);
    r.w = (const uint8_t *)rl64(dv, CH_OFF(w) + 2 * m);
    r.y = (float *)rl64(dv, CH_OFF(y) + 2 * m);
    r.bus = (uint32_t *)rl64(dv, CH_OFF(bus) + 2 * m);
    r.x = (const float *)rl64(dv, CH_OFF(x));
    r.xbus = (const uint32_t *)rl64(dv, CH_OFF(xbus));
    return r;
}

// Wave-uniform state of a wave's weight stream; survives a stage boundary so the
// next stage's first ring is fetched before its activation is ready.
struct Stream {
    const uint8_t *s16, *last16;
    int T, it, islot;
    uint32_t mis;
};

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

// Open the wave's stream of a stage and fill its ring (weights only).
template <int TYPE>
__device__ __forceinline__ void stream_prefetch(Stream &S, const WaveStage &ws, uint8_t *ring, int lane, int pre) {
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int D = rows_depth(TYPE);
    const int G = ws.ww.nrows * ws.nb;
    S.T = (G + ROWS_SB - 1) / ROWS_SB;
    const uint8_t *src = ws.w + (int64_t)ws.ww.r0 * ws.nb * BSZ;
    S.mis = (uint32_t)((uintptr_t)src & 15u);
    S.s16 = src - S.mis;
    S.last16 = G > 0 ? (const uint8_t *)((uintptr_t)(src + (int64_t)G * BSZ - 1) & ~(uintptr_t)15) : S.s16;
    S.it = 0;
    S.islot = 0;
    while (S.it < D && S.it < pre && S.it < S.T) stream_issue<TYPE>(S, ring, lane);
}

__device__ __forceinline__ void prefetch(Stream &S, const WaveStage &ws, uint8_t *ring, int lane, int pre) {
    if (ws.type == Q6_K) stream_prefetch<Q6_K>(S, ws, ring, lane, pre);
    else if (ws.type == Q5_K) stream_prefetch<Q5_K>(S, ws, ring, lane, pre);
    else stream_prefetch<Q4_K>(S, ws, ring, lane, pre);
}

struct Tm {  // diagnostics of one stage (wave 0): s_memrealtime stamps, poll count
    uint64_t poll0, ok, quant, comp, flush;
    int npoll;
};

// The stage's Q8_K activation into LDS (Q8L blocks): poller wave p quantizes
// superblocks 4*pollers*i + 4p + (lane >> 4), 16 lanes each. From the bus: poll
// until every pair of the wave's blocks carries `tag`.
__device__ __forceinline__ void stage_activation(const WaveStage &ws, uint8_t *act, int wave, int lane, uint32_t tag,
                                                 uint32_t *flag, Tm &tm, int si, const uint32_t *sig,
                                                 uint32_t sig_target) {
    const int nb = ws.nb;
    const int pass = 4 * ws.pollers;
    if (wave >= ws.pollers) return;
    if (ws.xbus) {  // no global polling before this workgroup's own streaming waves have flushed
        while (__hip_atomic_load(sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < sig_target)
            __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll 1
    for (int i = 0; pass * i + 4 * wave < nb; ++i) {
        const int bi = pass * i + 4 * wave + (lane >> 4);
        const int b = bi < nb ? bi : nb - 1;
        u32x4 v[4];
        if (ws.xbus) {
            const uint32_t *xp = ws.xbus + 2 * ((int64_t)b * QK + 16 * (lane & 15));
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            if (i == 0) tm.poll0 = t0;
            u32x4 p[8];
            for (;;) {
                if (i == 0) ++tm.npoll;
#pragma unroll
                for (int k = 0; k < 8; ++k) p[k] = load_sys16(xp + 4 * k);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // the loads are invisible to the compiler: pin their registers past the wait
                asm volatile("" : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]),
                             "+v"(p[7]));
                bool ok = true;
#pragma unroll
                for (int k = 0; k < 8; ++k) ok = ok && p[k].y == tag && p[k].w == tag;
                if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
                    if (i == 0) tm.ok = __builtin_amdgcn_s_memrealtime();
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > kHandoffTicks) {
                    if (lane == 0) {  // flag + what was still missing (host prints it)
                        atomicOr(flag, 1u);
                        flag[1] = (uint32_t)si;
                        flag[2] = blockIdx.x;
                        flag[3] = (uint32_t)b;
                        flag[4] = p[0].y;
                        flag[5] = tag;
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = u32x4{p[2 * k].x, p[2 * k].z, p[2 * k + 1].x, p[2 * k + 1].z};
        } else {
            const float *xp = ws.x + (int64_t)b * QK + 16 * (lane & 15);
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = *(const u32x4 *)(xp + 4 * k);
        }
        if (bi < nb) quant16_store(v, lane & 15, act + Q8L_STRIDE * b);
    }
    tm.quant = __builtin_amdgcn_s_memrealtime();
}

// Stage compute of one streaming wave: kq_rows' main loop and flush (rows_body,
// kq_rows.hip), continuing the stream whose first ring `prefetch` issued.
template <int TYPE>
__device__ __forceinline__ void stage_rows(const ChainArgs &a, const WaveStage &ws, Stream &S, uint8_t *smem,
                                           const uint8_t *actq, int wave, int lane, uint32_t tag, Tm &tm) {
    constexpr int BSZ = block_bytes(TYPE);
    constexpr int NI = rows_ni(TYPE);
    constexpr int SLOT = rows_slot(TYPE);
    constexpr int D = rows_depth(TYPE);
    const int nb = ws.nb, bR = ws.bR;
    const WaveWork &ww = ws.ww;
    const int q = lane >> 2, s = lane & 3;
    uint8_t *const ring = smem + a.ring + wave * a.ring_stride;
    uint8_t *const ring_end = ring + D * SLOT;
    Rec *const recs = (Rec *)(smem + a.recs + wave * a.recs_stride);
    float *const outs = (float *)(smem + a.outs + wave * a.outs_stride);
    const int G = ww.nrows * nb;
    const int T = S.T;
    while (S.it < D && S.it < T) stream_issue<TYPE>(S, ring, lane);  // the rest of the ring

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
        // in flight: steps t .. S.it-1 plus possibly older/younger non-DMA loads, which
        // only make these counted waits more conservative (returns are in order)
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
        if (ws.bus) {  // the hand-off copy first: it is on the next stage's critical path
            uint32_t *bus = ws.bus + 2 * (int64_t)ww.r0;
            for (int k = 0; k < ww.nrows; k += 64)
                if (k + lane < ww.nrows) store_sys8(bus + 2 * (k + lane), __float_as_uint(outs[k + lane]), tag);
        }
        float *y = ws.y + ww.r0;
        for (int k = 0; k < ww.nrows; k += 64)
            if (k + lane < ww.nrows) y[k + lane] = outs[k + lane];
    }
    tm.flush = __builtin_amdgcn_s_memrealtime();
}

// A streaming wave is done with its stage (outputs issued): count it in LDS.
__device__ __forceinline__ void signal_done(uint32_t *sig, int lane) {
    if (lane == 0) __hip_atomic_fetch_add(sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void rows(const ChainArgs &a, const WaveStage &ws, Stream &S, uint8_t *smem,
                                     const uint8_t *actq, int wave, int lane, uint32_t tag, Tm &tm) {
    if (ws.type == Q6_K) stage_rows<Q6_K>(a, ws, S, smem, actq, wave, lane, tag, tm);
    else if (ws.type == Q5_K) stage_rows<Q5_K>(a, ws, S, smem, actq, wave, lane, tag, tm);
    else stage_rows<Q4_K>(a, ws, S, smem, actq, wave, lane, tag, tm);
}

}  // namespace

__global__ void __launch_bounds__(ROWS_WAVES * 64) kq_chain(const ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *const ring = smem + a.ring + wave * a.ring_stride;
    const bool stamps = a.stamps != nullptr;
    // this launch's tag (one more than the last launch's, published by its last
    // workgroup out) and stage 0's descriptor
    uint32_t tag, dv;
    {
        const u32x4 e = load_sys16(a.sync);
        dv = desc_load(a.st, 0, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(dv));
        tag = __builtin_amdgcn_readfirstlane(e.x) + 1u;
    }
    uint32_t *const sig = (uint32_t *)(smem + a.sig);
    if (threadIdx.x == 0) *sig = 0u;  // (ordered before any increment by the first barrier)
    uint32_t sig_target = 0;          // streaming-wave completions of all earlier stages
    WaveStage cur = resolve(dv, wave);
    Stream S;
    S.T = 0;
    prefetch(S, cur, ring, lane, a.pre);
    uint32_t dn = a.n_stages > 1 ? desc_load(a.st, 1, lane) : 0u;  // one stage ahead

    // One workgroup barrier per stage. The activation is double-buffered (stage s in
    // act[s & 1]): pollers quantize stage s+1's activation while the streaming waves
    // still compute stage s, and can never run two stages ahead (stage s+2's
    // activation needs stage s+1's outputs, which needs every streaming wave past s).
#pragma unroll 1
    for (int si = 0; si < a.n_stages; ++si) {
        Tm tm = {0, 0, 0, 0, 0, 0};
        uint8_t *const act = smem + a.act + (si & 1) * a.act_stride;
        stage_activation(cur, act, wave, lane, tag, a.sync + 2, tm, si, sig, sig_target);  // pollers only
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");     // Q8_K row complete
        const uint64_t t_x = stamps ? __builtin_amdgcn_s_memrealtime() : 0;
        rows(a, cur, S, smem, act, wave, lane, tag, tm);                     // streaming waves only
        if (wave >= cur.pollers) signal_done(sig, lane);
        sig_target += ROWS_WAVES - cur.pollers;
        if (si + 1 < a.n_stages) {  // next stage's weights do not wait for its activation
            // dn is older than every DMA of this stage: the loop's last wait (T > 0) or
            // the pollers' activation wait covered it; otherwise wait here
            if (S.T == 0) vm_wait<0>();
            asm volatile("" : "+v"(dn));
            cur = resolve(dn, wave);
            prefetch(S, cur, ring, lane, a.pre);
            if (si + 2 < a.n_stages) dn = desc_load(a.st, si + 2, lane);
        }
        if (stamps && lane == 0 && (wave == 0 || wave == ROWS_WAVES - 1)) {
            // wave 0 (a poller): first poll, poll success, quantized, polls;
            // the last wave (streams rows): activation ready, computed, flushed, next ring issued
            const int64_t o = ((int64_t)blockIdx.x * a.n_stages + si) * 8;
            if (o + 7 < a.stamps_cap) {
                if (wave == 0) {
                    a.stamps[o] = tm.poll0;
                    a.stamps[o + 1] = tm.ok;
                    a.stamps[o + 2] = tm.quant;
                    a.stamps[o + 7] = (uint64_t)tm.npoll;
                } else {
                    a.stamps[o + 3] = t_x;
                    a.stamps[o + 4] = tm.comp;
                    a.stamps[o + 5] = tm.flush;
                    a.stamps[o + 6] = __builtin_amdgcn_s_memrealtime();
                }
            }
        }
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
