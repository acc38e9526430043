// kq_layer.hip — one decode layer of llm_build_llama (ggml_compute_forward_mul_mat's
// K-quant vec_dots, README.md:125-137, plus the layer's other ops) as ONE persistent
// launch: the row-owned persistent layer of VERDICT r4 #2 / MI355X_MICROARCH.md
// **engine-vs-launches**.
//
// Why: the launch chain (5 launches per layer) pays, per launch, a kernel boundary, the
// fetch of an activation the previous launch just wrote, and a weight stream that starts
// only after the launch has started. Here the weights do not depend on any activation, so
// every CU streams its rows of the NEXT stage into LDS while the current hand-off is still
// in flight; a stage's dot products then run from LDS as soon as its activation lands.
//
// Measured: bit-exact, and 1.45x the launch chain at Llama-3-8B width, so the
// engine is opt-in (mi355x_backend_set_layer_engine).
//
// Decomposition (one 512-thread workgroup per CU, all co-resident; b = blockIdx.x):
//  * every GEMV stage gives workgroup b the rows [b*N/G, (b+1)*N/G) of its matrix (q/k/v:
//    of the concatenation [q | k | v]; gate/up: the same rows of both). Each row's fp32
//    chain stays inside the workgroup: the 7 stream waves (0..6) split the workgroup's
//    contiguous row stream at 16-superblock steps and write the exact 16-B records of
//    kq_rows (the operands of the reference's update, README.md:551/:614) into LDS; the
//    control wave (7) replays each row's chain in superblock order (chain_step), so the
//    outputs are bit-identical to ggml_vec_dot_q4_K_q8_K (and Q5_K / Q6_K) row by row;
//  * stream wave w keeps a byte ring (D x the largest step) filled by non-temporal LDS-DMA
//    along ITS steps of every stage in order (q/k/v, o-proj, gate/up, down): when it has
//    consumed a stage, it already issues the next stage's weights, before that stage's
//    activation exists. The host builds every wave's step list once per weight set (source,
//    granules, ring position, stage row, issue gate: layer_table_fill); the wave holds it in
//    VGPRs and reads a step with v_readlane, so a step costs no memory access and no
//    branchy ring arithmetic. Every step is exactly 4 DMA instructions, so the counted
//    vmcnt wait of the oldest step is 4 x (steps in flight - 1);
//  * the activation of a stage is quantized once per workgroup into LDS (Q8L blocks,
//    quant16_store: quantize_row_q8_K_ref exactly), with the rms_norm prologue (the
//    exactness guard of kq_rows) for q/k/v and gate/up;
//  * attention: workgroup a*stride + (a%8)%stride runs heads [a*hpw, (a+1)*hpw) with all
//    512 threads (attn_head, as kq_attn_oproj: 2 heads of 256 threads at head_dim 128,
//    4 of 128 at 64).
// Hand-offs between stages (MI355X_MICROARCH.md, valid forms, row 1): the producing waves'
// outputs are stored sc1 (write-through), every storing wave drains with vmcnt(0), the
// workgroup barrier (attention) or the single storing wave, then ONE lane adds 1 to the
// edge's counter shard b & 7 (agent scope). A consumer's control wave polls every shard
// with sc1 loads (s_sleep between polls) until each reaches (epoch + 1) x its producers;
// the other waves load after the workgroup barrier it then joins, and EVERY load of handed-
// off bytes is an sc1 load. Counters are monotonic; `epoch` (word 0 of the block) counts
// this block's completed launches and is advanced by workgroup 0 once every workgroup has
// passed its last edge (so every workgroup read it before). A wait that does not complete
// within ~1 s sets *err and gives up (never a hang; the backend reports it).
#include <string.h>

#include <vector>

#include <hip/hip_ext.h>

#include "kq_attn_head.h"
#include "kq_internal.h"
#include "kq_rows_device.h"

namespace kq {

namespace {

// Timing stamps (experiment builds only: make variant-layer NAME=lst VFLAGS=-DKQ_LAYER_STAMPS=1):
// the control wave's lane 0 stores s_memrealtime at each phase boundary, slot i of
// stamps[b * 32 + i] (tools/layer_stamps.py). The product build has none.
#ifndef KQ_LAYER_STAMPS
#define KQ_LAYER_STAMPS 0
#endif
#define LY_STAMP(i)                                                                                  \
    do {                                                                                             \
        if (KQ_LAYER_STAMPS && a.stamps && lane == 0 && (int64_t)b * 32 + (i) < a.stamps_cap)        \
            a.stamps[(int64_t)b * 32 + (i)] = __builtin_amdgcn_s_memrealtime();                       \
    } while (0)

// Timing ablations (experiment builds only, outputs wrong): 1 no dot products in the stream
// loop, 2 no weight DMA (the ring's stale bytes are used), 4 no wait for the weight DMA.
#ifndef KQ_LAYER_DIAG
#define KQ_LAYER_DIAG 0
#endif

constexpr int LY_STREAM = LAYER_WAVES - 1;  // stream waves 0..6; wave 7 is the control wave
constexpr int LY_NI = 4;                    // DMA instructions per step, whatever its size
constexpr int LY_POLL_LIMIT = 1 << 20;      // polls (with s_sleep) before a wait gives up (~1 s)

// Workgroup barrier that waits for this wave's LDS operations only: the stream waves'
// weight DMAs stay in flight across it (MI355X_MICROARCH.md: barriers do not drain VMEM).
__device__ __forceinline__ void ly_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__host__ __device__ constexpr int ly_gran(int type) { return (15 + 16 * block_bytes(type) + 15) / 16; }

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float *p, float v) {
    __hip_atomic_store((uint32_t *)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16 B of a buffer written in this launch by other workgroups: an sc1 (agent-scope) buffer load
__device__ __forceinline__ u32x4 ld16_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ uint32_t *cnt_of(uint32_t *sync, int edge, int shard) {
    return sync + 32 * (1 + edge * 8 + shard);
}

// ---------------------------------------------------------------- stage geometry
struct LySeg {
    const uint8_t *w;
    int m, type, row0, nrows, rbase, steps;
};
// The workgroup's rows of every GEMV stage, computed once: [r0[s], r1[s]) of stage s's
// matrix (q/k/v: of the concatenation [q | k | v]; gate/up: of both).
// (No arrays indexed at run time anywhere in this kernel: they would live in scratch, and a
// scratch access is a vector-memory operation whose compiler-inserted wait drains the
// weight ring.)
struct LyRows {
    int qa, qb, ea, eb, fa, fb;  // [qa, qb) of [q | k | v], [ea, eb) of E, [fa, fb) of F
};
__host__ __device__ __forceinline__ LyRows ly_rows(const LayerArgs &a, int b) {
    LyRows r;
    const int nqkv = a.nq + 2 * a.nkv;
    r.qa = (int)((int64_t)b * nqkv / a.G);
    r.qb = (int)((int64_t)(b + 1) * nqkv / a.G);
    r.ea = (int)((int64_t)b * a.E / a.G);
    r.eb = (int)((int64_t)(b + 1) * a.E / a.G);
    r.fa = (int)((int64_t)b * a.F / a.G);
    r.fb = (int)((int64_t)(b + 1) * a.F / a.G);
    return r;
}
struct LyStage {
    LySeg s0, s1, s2;
    int nseg, nb, R, T;
};
// Segment of matrix M: rows [row0, row0 + n) (n may be 0: an empty segment, no steps).
template <int M>
__host__ __device__ __forceinline__ LySeg ly_seg(const LayerArgs &a, int nb, int rbase, int row0, int n) {
    LySeg g;
    n = n > 0 ? n : 0;
    g.w = a.w[M];
    g.m = M;
    g.type = a.type[M];
    g.row0 = row0;
    g.nrows = n;
    g.rbase = rbase;
    g.steps = (n * nb + ROWS_SB - 1) / ROWS_SB;
    return g;
}

// The workgroup's segments of GEMV stage s (0 q/k/v, 1 o-proj, 2 gate/up, 3 down): always
// three, the unused ones empty (no segment counter: a struct filled at a run-time index
// would live in scratch).
__host__ __device__ __forceinline__ void ly_stage(const LayerArgs &a, int s, const LyRows &rw, LyStage &st) {
    if (s == 0) {
        const int r0 = rw.qa, r1 = rw.qb;
        st.nb = a.nb_e;
        const int lo1 = a.nq, lo2 = a.nq + a.nkv;
        const int n0 = (r1 < lo1 ? r1 : lo1) - r0;
        const int u1 = r0 > lo1 ? r0 : lo1, v1 = r1 < lo2 ? r1 : lo2;
        const int u2 = r0 > lo2 ? r0 : lo2;
        st.s0 = ly_seg<0>(a, st.nb, 0, r0, n0);
        st.s1 = ly_seg<1>(a, st.nb, st.s0.nrows, u1 - lo1, v1 - u1);
        st.s2 = ly_seg<2>(a, st.nb, st.s0.nrows + st.s1.nrows, u2 - lo2, r1 - u2);
    } else if (s == 2) {
        st.nb = a.nb_e;
        st.s0 = ly_seg<4>(a, st.nb, 0, rw.fa, rw.fb - rw.fa);
        st.s1 = ly_seg<5>(a, st.nb, st.s0.nrows, rw.fa, rw.fb - rw.fa);
        st.s2 = ly_seg<5>(a, st.nb, 2 * st.s0.nrows, 0, 0);
    } else {
        st.nb = s == 1 ? a.nb_e : a.nb_f;
        st.s0 = s == 1 ? ly_seg<3>(a, st.nb, 0, rw.ea, rw.eb - rw.ea) : ly_seg<6>(a, st.nb, 0, rw.ea, rw.eb - rw.ea);
        st.s1 = ly_seg<6>(a, st.nb, st.s0.nrows, 0, 0);
        st.s2 = ly_seg<6>(a, st.nb, st.s0.nrows, 0, 0);
    }
    st.nseg = 3;
    st.R = st.s0.nrows + st.s1.nrows + st.s2.nrows;
    st.T = st.s0.steps + st.s1.steps + st.s2.steps;
}

// ---------------------------------------------------------------- each stream wave's step list
// Step = 16 consecutive superblocks of one segment's stream (fewer at its end). Stage s's
// T steps of the workgroup go to stream wave w as [T*w/7, T*(w+1)/7). The host writes every
// (workgroup, wave) list once per layer launch (layer_table_fill): a 16-B header
// {count of stage 0, 1, 2, 3} and 16 B per step, {src16 (8 B), ngran | mis << 8 | type << 12 |
// cnt << 14 | sb0 << 19, rrow0 | need << 8 | pos16 << 16}: src16 is the 16-B boundary below the step's first byte, mis
// the offset above it, ngran the 16-B granules to fetch, (rrow0, sb0) the stage row and
// block of its first superblock; the last word also holds the step's place in the wave's
// weight ring (pos16 << 16) and its issue gate (need << 8, see layer_table_fill). The wave
// loads its list into registers at entry (lane i
// holds step i) and reads a step with v_readlane: no memory access and no branch per step.
// (Measured: the scalar bookkeeping of a step cost ~0.4 us when it branched on the list
// half, looped over the row wrap and searched a 37-case wait switch, as much as the dot
// products of the step's 16 superblocks.)
constexpr int LY_LIST_MAX = 64;  // steps per wave and layer
__host__ __device__ __forceinline__ int ly_tcode(int type) { return type == Q4_K ? 0 : type == Q5_K ? 1 : 2; }

struct LyList {
    u32x4 e;       // step `lane`
    int c[4];      // steps of each stage
    int n;
};

__device__ __forceinline__ void ly_list_load(const LayerArgs &a, int b, int w, int lane, LyList &L) {
    const uint8_t *p = a.tab + (int64_t)b * a.tab_stride + (int64_t)w * (a.tab_stride / LY_STREAM);
    const u32x4 h = *(const u32x4 *)p;
    L.c[0] = __builtin_amdgcn_readfirstlane((int)h.x);
    L.c[1] = __builtin_amdgcn_readfirstlane((int)h.y);
    L.c[2] = __builtin_amdgcn_readfirstlane((int)h.z);
    L.c[3] = __builtin_amdgcn_readfirstlane((int)h.w);
    L.n = L.c[0] + L.c[1] + L.c[2] + L.c[3];
    const u32x4 *e = (const u32x4 *)(p + 16);
    const u32x4 z = {0u, 0u, 0u, 0u};
    L.e = lane < L.n ? e[lane] : z;
}

struct LyStep {
    const uint8_t *src16, *last16;
    uint32_t mis;
    int ngran, type, cnt, rrow0, sb0, pos;
};
__device__ __forceinline__ LyStep ly_step(const LyList &L, int idx) {
    const uint32_t lo = __builtin_amdgcn_readlane(L.e.x, idx), hi = __builtin_amdgcn_readlane(L.e.y, idx);
    const uint32_t z = __builtin_amdgcn_readlane(L.e.z, idx), w = __builtin_amdgcn_readlane(L.e.w, idx);
    LyStep d;
    d.src16 = (const uint8_t *)(uintptr_t)(((uint64_t)hi << 32) | lo);
    d.ngran = (int)(z & 0xffu);
    d.mis = (z >> 8) & 15u;
    const int tc = (int)((z >> 12) & 3u);
    d.type = tc == 0 ? Q4_K : tc == 1 ? Q5_K : Q6_K;
    d.cnt = (int)((z >> 14) & 31u);
    d.sb0 = (int)((z >> 19) & 127u);
    d.rrow0 = (int)(w & 0xffu);
    d.pos = (int)(w >> 16) * 16;
    d.last16 = d.src16 + 16 * (d.ngran - 1);
    return d;
}

// LY_NI (4) LDS-DMA instructions (nt), instruction i for lanes [0, n[i]) at LDS byte address
// m0[i]: one exec save / restore around the four.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void ly_dma4(const void *const (&src)[4], const uint32_t (&m0)[4], const int (&n)[4], int lane) {
    uint64_t save;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "v_cmp_gt_i32_e32 vcc, %5, %9\n\t"
        "s_and_b64 exec, %0, vcc\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %10, off nt\n\t"
        "v_cmp_gt_i32_e32 vcc, %6, %9\n\t"
        "s_and_b64 exec, %0, vcc\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %11, off nt\n\t"
        "v_cmp_gt_i32_e32 vcc, %7, %9\n\t"
        "s_and_b64 exec, %0, vcc\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %12, off nt\n\t"
        "v_cmp_gt_i32_e32 vcc, %8, %9\n\t"
        "s_and_b64 exec, %0, vcc\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %13, off nt\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(save)
        : "s"(m0[0]), "s"(m0[1]), "s"(m0[2]), "s"(m0[3]), "s"(n[0]), "s"(n[1]), "s"(n[2]), "s"(n[3]), "v"(lane),
          "v"(src[0]), "v"(src[1]), "v"(src[2]), "v"(src[3])
        : "memory", "m0", "vcc");
}
#pragma clang diagnostic pop

// The step's granules into the ring at LDS byte address s0 (ngran * 16 bytes): exactly LY_NI
// DMA instructions on every path (an instruction past the step's granules re-reads the last
// granule into its own place: the same bytes, so the order in which the two land does not
// matter).
__device__ __forceinline__ void ly_issue(const LyStep &d, uint32_t s0, int lane) {
    if (KQ_LAYER_DIAG & 2) return;
    const void *src[LY_NI];
    uint32_t m0[LY_NI];
    int n[LY_NI];
#pragma unroll
    for (int i = 0; i < LY_NI; ++i) {
        const int k = d.ngran - 64 * i;
        const uint8_t *p = d.src16 + 1024 * i + 16 * lane;
        src[i] = k > 0 ? (const void *)(p < d.last16 ? p : d.last16) : (const void *)d.last16;
        m0[i] = __builtin_amdgcn_readfirstlane(k > 0 ? s0 + 1024u * (uint32_t)i : s0 + 16u * (uint32_t)(d.ngran - 1));
        n[i] = __builtin_amdgcn_readfirstlane(k > 0 ? (k < 64 ? k : 64) : 1);
    }
    ly_dma4(src, m0, n, lane);
}

// ---------------------------------------------------------------- one stream wave's ring
// A byte ring of RB bytes per wave: a step takes exactly its ngran * 16 bytes, placed after
// the previous one, or at the start when it would cross the end (the tail then idles until
// the consumer passes it). Issue and consumption place the same steps by the same rule, so
// the consumer finds each step where it was issued. At most LY_MAXQ steps in flight (the
// counted wait covers 4 x (in flight - 1) DMA instructions).
constexpr int LY_MAXQ = 10;
constexpr int LY_PRE = 2;  // steps a stream wave issues before the stage-0 activation barriers
// s_waitcnt until at most k younger steps' DMAs (LY_NI each) are in flight, 0 <= k < LY_MAXQ
__device__ __forceinline__ void ly_wait(int k) {
    switch (k) {
        case 0: vm_wait<0>(); break;
        case 1: vm_wait<LY_NI>(); break;
        case 2: vm_wait<2 * LY_NI>(); break;
        case 3: vm_wait<3 * LY_NI>(); break;
        case 4: vm_wait<4 * LY_NI>(); break;
        case 5: vm_wait<5 * LY_NI>(); break;
        case 6: vm_wait<6 * LY_NI>(); break;
        case 7: vm_wait<7 * LY_NI>(); break;
        case 8: vm_wait<8 * LY_NI>(); break;
        default: vm_wait<9 * LY_NI>(); break;
    }
}
struct LyRing {
    uint32_t base;  // LDS byte address of this wave's ring
    int ii;         // steps issued (the next list index to issue)
    int nc;         // steps consumed
};

// Issue every step whose gate has opened: step k may go once `need` (its list field) steps
// are consumed, the host's placement (layer_table_fill) having checked that it then
// overwrites nothing still held and that at most LY_MAXQ steps are in flight.
__device__ __forceinline__ void ly_top_up(const LyList &L, LyRing &r, int lane, int most = LY_LIST_MAX) {
    while (r.ii < L.n && r.ii < most) {
        const uint32_t w = __builtin_amdgcn_readlane(L.e.w, r.ii);
        if ((int)((w >> 8) & 0xffu) > r.nc) break;
        ly_issue(ly_step(L, r.ii), r.base + ((w >> 16) << 4), lane);
        ++r.ii;
    }
}

// This wave's steps of stage s (nb superblocks per row, R stage rows in the workgroup):
// each step's records into LDS (block-major [sb][row]).
__device__ __forceinline__ void ly_consume(const LyList &L, LyRing &r, int s, int nb, int R, int lane,
                                          const uint8_t *smem, const uint8_t *act, Rec *recs, uint64_t *stp = nullptr) {
    const int j0 = s == 0 ? 0 : s == 1 ? L.c[0] : s == 2 ? L.c[0] + L.c[1] : L.c[0] + L.c[1] + L.c[2];
    const int j1 = j0 + (s == 0 ? L.c[0] : s == 1 ? L.c[1] : s == 2 ? L.c[2] : L.c[3]);
    const int q = lane >> 2, sl = lane & 3;
    const uint32_t inv_nb = (65536u + (uint32_t)nb - 1u) / (uint32_t)nb;  // (x * inv_nb) >> 16 == x / nb for x < 128
    for (int j = j0; j < j1; ++j) {
        if (KQ_LAYER_STAMPS && stp && lane == 0 && j - j0 < 12) stp[j - j0] = __builtin_amdgcn_s_memrealtime();
        if (!(KQ_LAYER_DIAG & 6)) ly_wait(r.ii - j - 1);  // this step's DMAs landed (younger ones may not)
        const LyStep d = ly_step(L, j);
        const uint8_t *slot = smem + (r.base - (uint32_t)(uintptr_t)(LDS void *)smem) + d.pos;
        // this quad's superblock: 16 consecutive ones span at most 16 / nb + 1 rows
        const int sbq = d.sb0 + q, dr = (int)(((uint32_t)sbq * inv_nb) >> 16);
        const int row = d.rrow0 + dr, sb = sbq - dr * nb;
        if ((KQ_LAYER_DIAG & 1) && q < d.cnt && sl == 0) recs[sb * R + row] = Rec{0, 0, 0.f, 0.f};  // ablation
        if (!(KQ_LAYER_DIAG & 1) && q < d.cnt) {  // (uniform over the quad: DPP sums inside it)
            const int bsz = block_bytes(d.type);
            const uint8_t *blk = slot + d.mis + q * bsz;
            const uint8_t *ab = act + sb * Q8L_STRIDE;
            const QuadOut o = d.type == Q4_K ? quad_q4K(blk, ab, sl) : d.type == Q5_K ? quad_q5K(blk, ab, sl)
                                                                                       : quad_q6K(blk, ab, sl);
            const int isum = quad_sum(o.isum);
            const int imin = quad_sum(o.imin);
            if (sl == 0) {
                const float yd = *(const float *)ab;
                Rec rec;
                if (d.type == Q6_K) {
                    rec.a = isum - 32 * imin;
                    rec.b = 0;
                    rec.c = h2f(o.dh) * yd;  // d_all * y.d
                    rec.e = 0.f;
                } else {
                    rec.a = isum;
                    rec.b = imin;
                    rec.c = yd * h2f(o.dh & 0xffffu);  // y.d * fp16(x.d)
                    rec.e = yd * h2f(o.dh >> 16);      // y.d * fp16(x.dmin)
                }
                recs[sb * R + row] = rec;
            }
        }
        r.nc = j + 1;
        ly_top_up(L, r, lane);
    }
}

// ---------------------------------------------------------------- control-wave pieces
// Wait until every shard of edge e holds (epoch + 1) x its producers (wave-uniform result).
__device__ __forceinline__ void ly_poll(const LayerArgs &a, int e, uint32_t epoch, int lane) {
    uint32_t ex = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) ex = (lane & 7) == k ? a.expect[e][k] : ex;
    const uint32_t want = (epoch + 1u) * ex;
    const uint32_t *c = cnt_of(a.sync, e, lane & 7);
    for (int it = 0;; ++it) {
        const uint32_t v = lane < 8 ? ld_sc1(c) : want;
        if (__ballot((int)(v - want) < 0) == 0) break;
        if ((it & 255) == 255 && ld_sc1((const uint32_t *)a.err) != 0) break;  // another wait gave up
        if (it >= LY_POLL_LIMIT) {
            if (lane == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// one lane adds the workgroup's arrival (after the caller's stores drained)
__device__ __forceinline__ void ly_signal(const LayerArgs &a, int e, int b, int lane) {
    if (lane == 0) __hip_atomic_fetch_add(cnt_of(a.sync, e, b & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Row r's chain over its nb records, in superblock order (the reference's fp32 updates):
// records read 8 ahead (independent LDS reads), the dependent fp32 updates after them.
template <int TYPE>
__device__ __forceinline__ float ly_chain_t(const Rec *recs, int R, int nb, int r) {
    float v = 0.f;
    int i = 0;
    for (; i + 8 <= nb; i += 8) {
        Rec rc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) rc[k] = recs[(i + k) * R + r];
#pragma unroll
        for (int k = 0; k < 8; ++k) v = chain_step(TYPE, rc[k], v);
    }
    for (; i < nb; ++i) v = chain_step(TYPE, recs[i * R + r], v);
    return v;
}
__device__ __forceinline__ float ly_chain(const Rec *recs, int R, int nb, int r, int type) {
    return type == Q4_K ? ly_chain_t<Q4_K>(recs, R, nb, r) : type == Q5_K ? ly_chain_t<Q5_K>(recs, R, nb, r)
                                                                          : ly_chain_t<Q6_K>(recs, R, nb, r);
}

// ---------------------------------------------------------------- activation builds
// The stage activation (nb superblocks of src) into Q8L blocks at `act`, by every wave of
// the workgroup: wave w, lane l handles superblock j = 32 i + 4 w + (l >> 4), elements
// 16 (l & 15) .. +16. src was written in this launch: sc1 loads. norm: rms_norm then MUL by
// norm_w (kq_rows' prologue arithmetic: the fixed-order sum, the exactness guard with
// ggml's sequential sum, (x * scale) * w).
template <bool NORM>
__device__ __forceinline__ void ly_build(const float *src, int nb, const float *norm_w, float eps, uint8_t *act,
                                         double *sums, int wave, int lane) {
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(src, (uint32_t)nb * QK * 4u);
    const int np = (nb + 4 * LAYER_WAVES - 1) / (4 * LAYER_WAVES);  // passes (<= 2: nb <= 64)
    u32x4 xv[2][4], wv[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int j = 4 * LAYER_WAVES * i + 4 * wave + (lane >> 4);
        const int jj = j < nb ? j : nb - 1;
        if (i < np) {
#pragma unroll
            for (int k = 0; k < 4; ++k) xv[i][k] = ld16_sc1(rs, (uint32_t)(jj * QK + 16 * (lane & 15) + 4 * k) * 4u);
            if (NORM) {  // the norm weights with x: not behind the sum's barrier
                const u32x4 *wp = (const u32x4 *)(norm_w + (int64_t)jj * QK + 16 * (lane & 15));
#pragma unroll
                for (int k = 0; k < 4; ++k) wv[i][k] = wp[k];
            }
        }
    }
    if (NORM) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i >= np) continue;  // (uniform)
            const int j = 4 * LAYER_WAVES * i + 4 * wave + (lane >> 4);
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
            if (j < nb && (lane & 15) == 0) sums[j] = sq;
        }
        ly_bar();
        const int64_t n = (int64_t)nb * QK;
        double tot = seq_sum_lanes(sums, nb, lane);  // superblocks in order (every wave the same)
        if (rms_mean_ambiguous(div_by_count(tot, n), n)) {  // ggml's sequential order (sc1 loads)
            tot = 0.0;
            for (int64_t c0 = 0; c0 < n; c0 += 64) {
                const float v = c0 + lane < n ? __uint_as_float(ld_sc1((const uint32_t *)(src + c0 + lane))) : 0.0f;
                const double sq = (double)(v * v);
                const uint64_t bb = __builtin_bit_cast(uint64_t, sq);
                const int m = n - c0 < 64 ? (int)(n - c0) : 64;
                for (int i = 0; i < m; ++i) {
                    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bb, i);
                    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bb >> 32), i);
                    tot += __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
                }
            }
        }
        const float mean = (float)div_by_count(tot, n);
        const float scale = 1.0f / sqrtf(mean + eps);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i >= np) continue;
#pragma unroll
            for (int k = 0; k < 4; ++k) xv[i][k] = normmul4(xv[i][k], wv[i][k], scale);
        }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        if (i >= np) continue;
        const int j = 4 * LAYER_WAVES * i + 4 * wave + (lane >> 4);
        if (j < nb) quant16_store(xv[i], lane & 15, act + j * Q8L_STRIDE);
    }
}

// Stage 0's activation by the control wave alone (the stream waves are issuing the first
// weight steps meanwhile): rms_norm(x) * attn_norm -> Q8L; x comes from the previous launch
// (plain loads). nb <= 16: four passes of four superblocks, held in registers. The loads are
// issued at entry, ahead of every weight DMA of the workgroup (ly_load0, then a barrier):
// behind the entry burst they took ~6 us.
__device__ __forceinline__ void ly_load0(const LayerArgs &a, int lane, u32x4 (&xv)[4][4], u32x4 (&wv)[4][4]) {
    const int nb = a.nb_e;
    const int np = (nb + 3) / 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i < np) {
            const int j = 4 * i + (lane >> 4);
            const int jj = j < nb ? j : nb - 1;
            const u32x4 *xp = (const u32x4 *)(a.x + (int64_t)jj * QK + 16 * (lane & 15));
            const u32x4 *wp = (const u32x4 *)(a.attn_norm + (int64_t)jj * QK + 16 * (lane & 15));
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                xv[i][k] = xp[k];
                wv[i][k] = wp[k];
            }
        }
    }
}

// ... the sum, the scale and (x * scale) * w into `stg` (nb x 256 floats, superblock-major);
// the Q8L blocks are then made by every wave (ly_quant0_all) after a barrier.
__device__ __forceinline__ void ly_norm0(const LayerArgs &a, uint8_t *stg, double *sums, int lane,
                                         const u32x4 (&xv)[4][4], const u32x4 (&wv)[4][4]) {
    const int nb = a.nb_e;
    const int np = (nb + 3) / 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i >= np) continue;
        const int j = 4 * i + (lane >> 4);
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
    wave_lds_fence();
    const int64_t n = (int64_t)nb * QK;
    double tot = seq_sum_lanes(sums, nb, lane);
    if (rms_mean_ambiguous(div_by_count(tot, n), n)) tot = seq_sumsq_wave(a.x, n, lane);
    const float mean = (float)div_by_count(tot, n);
    const float scale = 1.0f / sqrtf(mean + a.eps);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (i >= np) continue;
        const int j = 4 * i + (lane >> 4);
        if (j < nb) {
            u32x4 *d = (u32x4 *)(stg + j * (QK * 4) + 64 * (lane & 15));
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = normmul4(xv[i][k], wv[i][k], scale);
        }
    }
}

// staged floats -> Q8L blocks: wave w, lane l: superblock 4 w + (l >> 4) (nb <= 16: one pass)
__device__ __forceinline__ void ly_quant0_all(int nb, const uint8_t *stg, uint8_t *act, int wave, int lane) {
    const int j = 4 * wave + (lane >> 4);
    if (j < nb) {
        const u32x4 *sp = (const u32x4 *)(stg + j * (QK * 4) + 64 * (lane & 15));
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = sp[k];
        quant16_store(v, lane & 15, act + j * Q8L_STRIDE);
    }
}

}  // namespace

template <int HD>
__global__ void __launch_bounds__(LAYER_WAVES * 64) kq_layer(const LayerArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int b = (int)blockIdx.x;
    const bool ctrl = wave == LY_STREAM;
    uint8_t *const act = smem + a.o_aux;
    Rec *const recs = (Rec *)(smem + a.o_aux + a.act_bytes);
    double *const sums = (double *)(smem + a.o_sums);
    float *const res = (float *)(smem + a.o_res);  // x, then x1, of this workgroup's o / down rows
    const int ai = b / a.attn_stride;
    const bool attn_wg = ai < a.n_attn && b == ai * a.attn_stride + (ai & 7) % a.attn_stride;
    const LyRows rw = ly_rows(a, b);
    if (ctrl) LY_STAMP(0);

    LyList L;
    LyRing ring;
    ring.base = (uint32_t)(uintptr_t)(LDS void *)smem + (uint32_t)(wave * a.D * a.slot);
    ring.ii = ring.nc = 0;
    if (!ctrl) ly_list_load(a, b, wave, lane, L);
    uint32_t epoch = 0;
    // ---- stage 0 (q/k/v): the control wave's activation loads go first; then the stream
    // waves issue their first steps while it builds the normed activation and stashes x of
    // the rows it will add to
    u32x4 xv[4][4], wv[4][4];
    float xres = 0.f;
    if (ctrl) {
        ly_load0(a, lane, xv, wv);
        if (lane < rw.eb - rw.ea) xres = a.x[rw.ea + lane];
        epoch = __builtin_amdgcn_readfirstlane(ld_sc1(a.sync));
    }
    ly_bar();  // A0: the activation requests are queued ahead of every weight DMA
    // Before the stage-0 barriers the stream waves issue only LY_PRE steps: a whole ring
    // issued there stalls on the memory queue's back-pressure and holds the barrier (stamps:
    // the activation +2.7 us at 8B, +4.9 us at TinyLlama). The rest goes out after the
    // staging barrier, by the waves without a superblock to quantize first.
    if (!ctrl) {
        ly_top_up(L, ring, lane, LY_PRE);
    } else {
        if (KQ_LAYER_STAMPS) {  // the activation loads' latency (stamps builds only)
            vm_wait<0>();
            LY_STAMP(1);
        }
        ly_norm0(a, (uint8_t *)recs, sums, lane, xv, wv);
        if (lane < rw.eb - rw.ea) res[lane] = xres;
        for (int r = lane + 64; r < rw.eb - rw.ea; r += 64) res[r] = a.x[rw.ea + r];
    }
    ly_bar();  // S0: the normed activation staged (in the records' space)
    // (a wave with a quad-quarter j >= nb has nothing to do; the quant needs every lane of
    // its 16-lane row, which ly_quant0_all's uniform-per-row condition keeps)
    const bool quants = 4 * wave < a.nb_e;
    if (!ctrl && !quants) ly_top_up(L, ring, lane);
    ly_quant0_all(a.nb_e, (const uint8_t *)recs, act, wave, lane);
    if (!ctrl && quants) ly_top_up(L, ring, lane);
    if (ctrl) LY_STAMP(2);
    ly_bar();  // B0: the Q8L activation in LDS
    if (!ctrl) ly_consume(L, ring, 0, a.nb_e, rw.qb - rw.qa, lane, smem, act, recs);
    ly_bar();  // C0: every record of the workgroup's q/k/v rows
    if (ctrl) {
        LY_STAMP(3);
        LyStage st;
        ly_stage(a, 0, rw, st);
        for (int r = lane; r < st.R; r += 64) {
            const int k = st.s2.nrows > 0 && r >= st.s2.rbase ? 2 : st.s1.nrows > 0 && r >= st.s1.rbase ? 1 : 0;
            const int type = k == 0 ? st.s0.type : k == 1 ? st.s1.type : st.s2.type;
            const int m = k == 0 ? st.s0.m : k == 1 ? st.s1.m : st.s2.m;
            const int row = k == 0 ? st.s0.row0 + r : k == 1 ? st.s1.row0 + (r - st.s1.rbase) : st.s2.row0 + (r - st.s2.rbase);
            const float v = ly_chain(recs, st.R, st.nb, r, type);
            st_sc1((m == 0 ? a.y[0] : m == 1 ? a.y[1] : a.y[2]) + row, v);
        }
        vm_wait<0>();
        ly_signal(a, 0, b, lane);
        LY_STAMP(4);
    }
    // ---- attention (its workgroups only): heads [ai*hpw, ai*hpw + hpw), every thread
    if (attn_wg) {
        if (!ctrl) ly_top_up(L, ring, lane);
        else {
            ly_poll(a, 0, epoch, lane);
            LY_STAMP(5);
        }
        ly_bar();  // A1: q / k / v of every head written
        constexpr int TPH = HD == 64 ? 128 : 256;
        const int hi = (int)threadIdx.x / TPH, t = (int)threadIdx.x % TPH;
        const int h = ai * a.hpw + hi;
        attn_head<HD, TPH, 0, true, true>(a.at, h, t, smem + a.o_aux + hi * a.head_lds, a.att + (int64_t)h * HD, true);
        vm_wait<0>();  // this wave's sc1 output stores (and its weight DMAs) done
        ly_bar();      // D1
        if (ctrl) {
            ly_signal(a, 1, b, lane);
            LY_STAMP(6);
        }
    }
    // ---- stage 1: o-proj + x -> x1
    if (!ctrl) ly_top_up(L, ring, lane);
    else {
        ly_poll(a, 1, epoch, lane);
        LY_STAMP(7);
    }
    ly_bar();  // A2
    ly_build<false>(a.att, a.nb_e, nullptr, 0.f, act, sums, wave, lane);
    ly_bar();  // B2
    if (ctrl) LY_STAMP(8);
    if (!ctrl) ly_consume(L, ring, 1, a.nb_e, rw.eb - rw.ea, lane, smem, act, recs);
    ly_bar();  // C2
    if (ctrl) {
        LY_STAMP(9);
        LyStage st;
        ly_stage(a, 1, rw, st);
        for (int r = lane; r < st.R; r += 64) {
            const float v = ly_chain(recs, st.R, st.nb, r, st.s0.type) + res[r];  // ggml_add(mul_mat, x)
            res[r] = v;
            st_sc1(a.x1 + st.s0.row0 + r, v);
        }
        vm_wait<0>();
        ly_signal(a, 2, b, lane);
        LY_STAMP(10);
    }
    // ---- stage 2: ffn_norm(x1) -> gate / up -> SWIGLU -> h
    if (!ctrl) ly_top_up(L, ring, lane);
    else {
        ly_poll(a, 2, epoch, lane);
        LY_STAMP(11);
    }
    ly_bar();  // A3
    ly_build<true>(a.x1, a.nb_e, a.ffn_norm, a.eps, act, sums, wave, lane);
    ly_bar();  // B3
    if (ctrl) LY_STAMP(12);
    if (!ctrl)
        ly_consume(L, ring, 2, a.nb_e, 2 * (rw.fb - rw.fa), lane, smem, act, recs,
                   KQ_LAYER_STAMPS && a.stamps && wave == 0 && (int64_t)b * 32 + 32 <= a.stamps_cap ? a.stamps + (int64_t)b * 32 + 20 : nullptr);
    ly_bar();  // C3
    if (ctrl) {
        LY_STAMP(13);
        LyStage st;
        ly_stage(a, 2, rw, st);
        const int n = st.s0.nrows, r0 = st.s0.row0, n4 = a.F & ~3;
        for (int r = lane; r < n; r += 64) {
            const float gv = ly_chain(recs, st.R, st.nb, r, st.s0.type);
            const float uv = ly_chain(recs, st.R, st.nb, n + r, st.s1.type);
            // ggml_vec_swiglu_f32: NEON body, libm tail (as kq_rows' epilogue)
            st_sc1(a.h + r0 + r, r0 + r < n4 ? v_silu(gv) * uv : (gv / (1.0f + expf(-gv))) * uv);
        }
        vm_wait<0>();
        ly_signal(a, 3, b, lane);
        LY_STAMP(14);
    }
    // ---- stage 3: down + x1 -> x2
    if (!ctrl) {
        ly_top_up(L, ring, lane);
    } else {
        ly_poll(a, 3, epoch, lane);
        LY_STAMP(15);
        // every workgroup has passed its last edge's arrival, so every one of them read
        // `epoch` at entry: the next launch of this block may count from epoch + 1
        if (b == 0 && lane == 0) __hip_atomic_store(a.sync, epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    ly_bar();  // A4
    ly_build<false>(a.h, a.nb_f, nullptr, 0.f, act, sums, wave, lane);
    ly_bar();  // B4
    if (ctrl) LY_STAMP(16);
    if (!ctrl) ly_consume(L, ring, 3, a.nb_f, rw.eb - rw.ea, lane, smem, act, recs);
    ly_bar();  // C4
    if (ctrl) {
        LY_STAMP(17);
        LyStage st;
        ly_stage(a, 3, rw, st);
        for (int r = lane; r < st.R; r += 64)
            st_sc1(a.x2 + st.s0.row0 + r, ly_chain(recs, st.R, st.nb, r, st.s0.type) + res[r]);
        vm_wait<0>();
        LY_STAMP(18);
    }
}

template __global__ void kq_layer<64>(const LayerArgs a);
template __global__ void kq_layer<128>(const LayerArgs a);

// ------------------------------------------------------------------ host side
size_t attn_lds16(int hd, int n_ctx);  // kq_attn_oproj.hip

int layer_plan(LayerArgs &a, int hd, int n_head) {
    if (a.E <= 0 || a.F <= 0 || a.E % QK || a.F % QK) return MI355X_E_UNSUPPORTED;
    a.nb_e = a.E / QK;
    a.nb_f = a.F / QK;
    if (a.nb_e > 16 || a.nb_f > 4 * LAYER_WAVES * 2) return MI355X_E_UNSUPPORTED;  // ly_build0 / ly_build passes
    if (hd != 64 && hd != 128) return MI355X_E_UNSUPPORTED;
    a.hpw = hd == 64 ? 4 : 2;
    if (n_head <= 0 || n_head % a.hpw || a.at.n_head != n_head || a.at.head_dim != hd) return MI355X_E_UNSUPPORTED;
    if (!a.at.rope_row) return MI355X_E_UNSUPPORTED;
    a.G = num_cus();
    const int G = a.G;
    a.n_attn = n_head / a.hpw;
    a.attn_stride = G / a.n_attn;
    if (a.attn_stride < 1 || G < 8 || G % 8) return MI355X_E_UNSUPPORTED;
    int gran = 0;
    for (int m = 0; m < 7; ++m) {
        if (!a.w[m] || block_bytes(a.type[m]) == 0) return MI355X_E_UNSUPPORTED;
        if (a.type[m] != Q6_K && ((uintptr_t)a.w[m] & 15u)) return MI355X_E_UNSUPPORTED;
        gran = gran > ly_gran(a.type[m]) ? gran : ly_gran(a.type[m]);
    }
    if (a.nq <= 0 || a.nkv <= 0) return MI355X_E_UNSUPPORTED;
    a.slot = 16 * gran;
    // workgroup rows (the most any workgroup gets) and the records they need
    auto cdiv = [](int64_t x, int64_t y) { return (int)((x + y - 1) / y); };
    const int R0 = cdiv(a.nq + 2 * a.nkv, G) + 2, R1 = cdiv(a.E, G), R2 = 2 * cdiv(a.F, G);
    if (R0 > 255 || R1 > 255 || R2 > 255) return MI355X_E_UNSUPPORTED;  // a step's row field: 8 bits
    int64_t recs = (int64_t)R0 * a.nb_e;
    recs = recs > (int64_t)R1 * a.nb_e ? recs : (int64_t)R1 * a.nb_e;
    recs = recs > (int64_t)R2 * a.nb_e ? recs : (int64_t)R2 * a.nb_e;
    recs = recs > (int64_t)R1 * a.nb_f ? recs : (int64_t)R1 * a.nb_f;
    recs = recs > (int64_t)a.nb_e * QK * 4 / 16 ? recs : (int64_t)a.nb_e * QK * 4 / 16;  // stage 0's staged floats
    const int nb_max = a.nb_e > a.nb_f ? a.nb_e : a.nb_f;
    a.act_bytes = nb_max * Q8L_STRIDE;
    a.head_lds = (int)attn_lds16(hd, a.at.n_ctx);
    int64_t aux = (int64_t)a.act_bytes + recs * 16;
    const int64_t attn = (int64_t)a.hpw * a.head_lds;
    aux = aux > attn ? aux : attn;
    const int64_t fixed = ((aux + 15) & ~(int64_t)15) + (int64_t)nb_max * 8 + (int64_t)R1 * 4 + 64;
    const int64_t budget = 160 * 1024 - 16 - fixed;
    int D = (int)(budget / ((int64_t)LY_STREAM * a.slot));
    if (D > 10) D = 10;
    if (D < 2) return MI355X_E_UNSUPPORTED;
    a.D = D;
    a.stamps = diag_stamps(&a.stamps_cap);
    const int ring = LY_STREAM * D * a.slot + 16;  // + slack for Q6_K's realigning reads
    a.o_aux = (ring + 15) & ~15;
    a.o_sums = a.o_aux + (int)((aux + 15) & ~(int64_t)15);
    a.o_res = a.o_sums + nb_max * 8;
    a.lds = a.o_res + R1 * 4 + 64;
    if (a.lds > 160 * 1024) return MI355X_E_UNSUPPORTED;
    // producers per edge and shard (shard = workgroup index & 7)
    memset(a.expect, 0, sizeof(a.expect));
    for (int b = 0; b < G; ++b) {
        a.expect[0][b & 7] += 1;
        a.expect[2][b & 7] += 1;
        a.expect[3][b & 7] += 1;
    }
    for (int i = 0; i < a.n_attn; ++i) {
        const int b = i * a.attn_stride + (i & 7) % a.attn_stride;
        a.expect[1][b & 7] += 1;
    }
    if (layer_table_stride(a) < 0) return MI355X_E_UNSUPPORTED;  // a wave's list past LY_LIST_MAX
    return MI355X_OK;
}

// Every (workgroup, stream wave) step list (see LyList): bytes per workgroup, LY_STREAM
// lists of 16 + 16 x (the most steps any wave gets) bytes ...
int64_t layer_table_stride(const LayerArgs &a) {
    int most = 0;
    for (int b = 0; b < a.G; ++b) {
        const LyRows rw = ly_rows(a, b);
        for (int w = 0; w < LY_STREAM; ++w) {
            int n = 0;
            for (int s = 0; s < 4; ++s) {
                LyStage st;
                ly_stage(a, s, rw, st);
                n += st.T * (w + 1) / LY_STREAM - st.T * w / LY_STREAM;
            }
            most = n > most ? n : most;
        }
    }
    if (most > LY_LIST_MAX) return -1;
    return (int64_t)LY_STREAM * (16 + 16 * most);
}

// ... and the lists themselves (G x stride bytes at buf). Stage s's T steps of the
// workgroup: wave w takes [T w / 7, T (w + 1) / 7), in stream order.
void layer_table_fill(const LayerArgs &a, uint8_t *buf, int64_t stride) {
    memset(buf, 0, (size_t)(a.G * stride));
    const int64_t wstride = stride / LY_STREAM;
    for (int b = 0; b < a.G; ++b) {
        const LyRows rw = ly_rows(a, b);
        for (int w = 0; w < LY_STREAM; ++w) {
            uint8_t *list = buf + (int64_t)b * stride + (int64_t)w * wstride;
            int32_t *hdr = (int32_t *)list;
            uint32_t *ent = (uint32_t *)(list + 16);
            int n = 0;
            // the wave's byte ring: a step takes its ngran * 16 bytes after the previous one,
            // or from 0 when it would cross the end (the tail idles until consumed past);
            // held[k] = its bytes plus that tail. Step k may issue once steps [0, need) are
            // consumed: the held bytes of need..k fit the ring, and k - need < LY_MAXQ.
            const int rb = a.D * a.slot;
            int end = 0;
            std::vector<int> held;
            for (int s = 0; s < 4; ++s) {
                LyStage st;
                ly_stage(a, s, rw, st);
                const int j0 = st.T * w / LY_STREAM, j1 = st.T * (w + 1) / LY_STREAM;
                for (int j = j0; j < j1; ++j, ++n) {
                    const int k = j >= st.s0.steps ? (j >= st.s0.steps + st.s1.steps ? 2 : 1) : 0;
                    const LySeg g = k == 0 ? st.s0 : k == 1 ? st.s1 : st.s2;
                    const int jj = k == 0 ? j : k == 1 ? j - st.s0.steps : j - st.s0.steps - st.s1.steps;
                    const int bsz = block_bytes(g.type);
                    const int g0 = ROWS_SB * jj;
                    const int G = g.nrows * st.nb;
                    const int cnt = G - g0 < ROWS_SB ? G - g0 : ROWS_SB;
                    const uint8_t *src = g.w + ((int64_t)g.row0 * st.nb + g0) * bsz;
                    const uint32_t mis = (uint32_t)((uintptr_t)src & 15u);
                    const uint64_t s16 = (uint64_t)(uintptr_t)(src - mis);
                    const uint32_t ngran = (mis + (uint32_t)(cnt * bsz) + 15u) >> 4;
                    const int row = g0 / st.nb, sb0 = g0 - row * st.nb;
                    const int B = (int)ngran * 16;
                    const bool wrap = end + B > rb;
                    const int pos = wrap ? 0 : end;
                    held.push_back((wrap ? rb - end : 0) + B);
                    end = pos + B;
                    int need = n + 1 - LY_MAXQ > 0 ? n + 1 - LY_MAXQ : 0, sum = 0;
                    for (int k = n; k >= need; --k) {
                        if (sum + held[k] > rb) {
                            need = k + 1;
                            break;
                        }
                        sum += held[k];
                    }
                    uint32_t *e = ent + 4 * n;
                    e[0] = (uint32_t)s16;
                    e[1] = (uint32_t)(s16 >> 32);
                    e[2] = ngran | (mis << 8) | ((uint32_t)ly_tcode(g.type) << 12) | ((uint32_t)cnt << 14) |
                           ((uint32_t)sb0 << 19);
                    e[3] = (uint32_t)(g.rbase + row) | ((uint32_t)need << 8) | ((uint32_t)(pos >> 4) << 16);
                }
                hdr[s] = j1 - j0;
            }
        }
    }
}

int launch_layer(const LayerArgs &a, hipStream_t stream) {
    if (!a.tab || a.tab_stride <= 0) return MI355X_E_INVAL;
    const void *fn = a.at.head_dim == 64 ? (const void *)kq_layer<64> : (const void *)kq_layer<128>;
    allow_lds(fn, (size_t)a.lds);
    void *args[] = {const_cast<LayerArgs *>(&a)};
    hipEvent_t e0, e1;
    hipError_t e;
    if (timing_slot(stream, e0, e1)) {
        e = hipExtLaunchKernel(fn, dim3((unsigned)a.G), dim3(LAYER_WAVES * 64), args, (size_t)a.lds, stream, e0, e1, 0);
        double bytes = 0;
        const int64_t rows[7] = {a.nq, a.nkv, a.nkv, a.E, a.F, a.F, a.E};
        for (int m = 0; m < 7; ++m) bytes += (double)rows[m] * (m == 6 ? a.nb_f : a.nb_e) * block_bytes(a.type[m]);
        timing_log(std::string("kq::kq_layer<") + std::to_string(a.at.head_dim) + ">", bytes, e0, e1);
    } else {
        e = hipLaunchKernel(fn, dim3((unsigned)a.G), dim3(LAYER_WAVES * 64), args, (size_t)a.lds, stream);
    }
    if (e != hipSuccess) return (int)e;
    e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

}  // namespace kq
