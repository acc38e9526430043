// kq_attn_oproj.hip — decode attention and the attn_output GEMV (+ its residual ADD) in ONE
// launch, bit-exact with the two launches it replaces (kq_attn_decode, then kq_rows on the
// attention's output: ggml_vec_dot_q4_K_q8_K row by row, ggml-cpu.c:1389, README.md:551/:614).
//
// Why it is exact. The o-proj's K runs over the attention's heads; one Q8_K superblock of its
// activation is exactly the outputs of 256 / head_dim consecutive heads, and quantize_row_q8_K
// works on each superblock alone. So superblock s of the activation, and the integer parts of
// every row's superblock s (sumi, summins) with the fp32 operands of the reference's update
// (d * y.d, dmin * y.d), can be produced by a workgroup that only computed those heads. The
// serial fp32 chain over superblocks is then replayed in superblock order, as kq_rows does
// from its records (chain_step, kq_device.h): the same operations in the same order.
//
// Decomposition (TinyLlama: 8 superblocks x 32 row blocks = 256 workgroups):
//  * workgroup (s, rb): the attention of heads [s*HPS, s*HPS + HPS) on 512 / HPS threads each
//    (kq_attn_head.h; 512 threads per workgroup); the nsb workgroups of row block rb run on one
//    XCD (placement below); only row block 0 stores the new KV cell. The head outputs stay in
//    LDS, one wave quantizes them (quant16_store).
//  * its o-proj bytes (rows [rb*R, rb*R + R), superblock s) arrive by LDS-DMA issued at
//    entry, under the attention; lane quad q computes one row's superblock (quad_q4K/5K/6K)
//    and stores the 16-B record write-through (sc1) at recs[rb][row][s].
//  * hand-off (MI355X_MICROARCH.md, valid forms, row 1): every wave drains its record stores
//    (vmcnt(0)), workgroup barrier, ONE lane adds 1 to cnt[rb] (agent scope, relaxed); the
//    workgroup whose add returns the last count of the round replays row r's nsb records
//    (sc1 loads, EVERY load of them), adds the residual and stores y. No workgroup waits for
//    another: nothing can deadlock, and placement only changes speed.
// Counters start every launch at 0: the last arriver is the one whose add returns nsb - 1,
// and it stores 0 back (zeroed once when the backend allocates them), so an aborted launch
// cannot misalign the next one.
#include <string.h>

#include <hip/hip_ext.h>

#include "kq_attn_head.h"
#include "kq_internal.h"
#include "kq_rows_device.h"

// Timing-only ablations, compile time (experiment builds: make variant-ao NAME=ao1
// VFLAGS=-DKQ_AO_DIAG=1): 1 no attention (zeros), 2 stop after the attention, 4 stop after
// the record stores (no hand-off), 8 no weight DMA.
#ifndef KQ_AO_DIAG
#define KQ_AO_DIAG 0
#endif

namespace kq {

namespace {

__device__ __forceinline__ void store16_sc1(void *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ u32x4 load16_sc1(const void *p) {
    u32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(r) : "v"(p) : "memory");
    return r;
}

}  // namespace

// LDS: HPS heads x head_lds | activation f32[256] | Q8L block | flag | weight granules
__host__ __device__ inline int attn_oproj_wofs(int hps, int head_lds) { return hps * head_lds + 1024 + Q8L_STRIDE + 16; }

template <int HD, int TYPE>
__global__ void __launch_bounds__(512) kq_attn_oproj(const AttnOprojArgs p) {
    constexpr int HPS = 256 / HD;   // heads per superblock of the o-proj's K
    constexpr int TPH = 512 / HPS;  // threads per head: 128 (head_dim 64) or 256 (128)
    constexpr int P = pieces_of(TYPE);  // 16-B granules per block in LDS (Q6_K: from the 16-B boundary below)
    constexpr int BSZ = block_bytes(TYPE);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int nsb = p.nsb;
    // XCD-aware placement (workgroup b runs on XCD b % 8): the nsb workgroups of a row block
    // share one XCD, so its rows' weight lines (a superblock of 144-210 B straddles two 128-B
    // lines, shared with the neighbouring superblocks) are fetched into ONE L2, not nsb of them
    int s, rb;
    if ((p.n_rb & 7) == 0) {
        const int x = (int)blockIdx.x & 7, j = (int)blockIdx.x >> 3;
        rb = x * (p.n_rb >> 3) + j / nsb;
        s = j % nsb;
    } else {
        s = (int)blockIdx.x % nsb;
        rb = (int)blockIdx.x / nsb;
    }
    const int hi = (int)threadIdx.x / TPH, t = (int)threadIdx.x % TPH;
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int nwaves = (int)(blockDim.x >> 6);
    const int row0 = rb * p.R;
    const int nrows = p.n_rows - row0 < p.R ? p.n_rows - row0 : p.R;
    float *const act = (float *)(smem + HPS * p.head_lds);
    uint8_t *const q8 = (uint8_t *)(act + 256);
    int *const flag = (int *)(q8 + Q8L_STRIDE);
    uint8_t *const wl = smem + attn_oproj_wofs(HPS, p.head_lds);

    // ---- o-proj weights of this workgroup (superblock s of rows row0 ..), by LDS-DMA at
    // entry: granule gi = 64 j + lane of instruction j is piece gi % P of row gi / P; lanes
    // past the last row re-read the last granule into the padding behind it
    if (!(KQ_AO_DIAG & 8)) {
        const int G = nrows * P;
        const uint8_t *const wb = p.w + (int64_t)s * BSZ;
        for (int j = wave; 64 * j < G; j += nwaves) {
            int gi = 64 * j + lane;
            gi = gi < G ? gi : G - 1;
            const int r = gi / P, pc = gi - r * P;
            const uint8_t *src = wb + (int64_t)(row0 + r) * p.row_stride;
            if (TYPE == Q6_K) src = (const uint8_t *)((uintptr_t)src & ~(uintptr_t)15);
            dma16_nt(src + 16 * pc, (LDS void *)(wl + 1024 * j));
        }
    }

    // the residual of the row this thread may replay, loaded long before the hand-off's drain
    const float resv = p.res && (int)threadIdx.x < nrows ? p.res[row0 + (int)threadIdx.x] : 0.f;

    // ---- attention of head s*HPS + hi (threads [TPH hi, TPH hi + TPH)), output into act
    if (KQ_AO_DIAG & 1) {
        if (t < HD) act[hi * HD + t] = 0.f;
    } else {
        attn_head<HD, TPH>(p.at, s * HPS + hi, t, smem + hi * p.head_lds, act + hi * HD, rb == 0);
    }

    // ---- the superblock's Q8_K block (quantize_row_q8_K_ref, as kq_rows' fused quantization)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's weight DMAs landed
    __syncthreads();                                    // every head's output and every DMA in LDS
    if (KQ_AO_DIAG & 6) {  // ablations: the residual passes through (finite values downstream)
        if (s == 0 && (KQ_AO_DIAG & 2) && (int)threadIdx.x < nrows)
            p.y[row0 + (int)threadIdx.x] = p.res ? p.res[row0 + (int)threadIdx.x] : 0.f;
        if (KQ_AO_DIAG & 2) return;
    }
    if (threadIdx.x < 16) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *(const u32x4 *)(act + 16 * (int)threadIdx.x + 4 * k);
        quant16_store(v, (int)threadIdx.x, q8);
    }
    __syncthreads();

    // ---- records: quad q computes rows q, q + nq, ... of superblock s
    const int q = (int)threadIdx.x >> 2, sl = (int)threadIdx.x & 3;
    const int nq = (int)(blockDim.x >> 2);
    const float yd = *(const float *)q8;
    for (int r = q; r < nrows; r += nq) {  // (uniform over the quad: DPP sums inside it)
        const uint8_t *blk = wl + r * (P * 16);
        if (TYPE == Q6_K) blk += (uint32_t)((uintptr_t)(p.w + (int64_t)(row0 + r) * p.row_stride + (int64_t)s * BSZ) & 15u);
        const QuadOut o = TYPE == Q4_K ? quad_q4K(blk, q8, sl) : TYPE == Q5_K ? quad_q5K(blk, q8, sl) : quad_q6K(blk, q8, sl);
        const int isum = quad_sum(o.isum);
        const int imin = quad_sum(o.imin);
        if (sl == 0) {
            u32x4 rec;
            if (TYPE == Q6_K) {
                rec.x = (uint32_t)(isum - 32 * imin);
                rec.y = 0u;
                rec.z = __float_as_uint(h2f(o.dh) * yd);  // d_all * y.d
                rec.w = 0u;
            } else {
                rec.x = (uint32_t)isum;
                rec.y = (uint32_t)imin;
                rec.z = __float_as_uint(yd * h2f(o.dh & 0xffffu));  // y.d * fp16(x.d)
                rec.w = __float_as_uint(yd * h2f(o.dh >> 16));      // y.d * fp16(x.dmin)
            }
            store16_sc1(p.recs + ((int64_t)(rb * p.R + r) * nsb + s) * 16, rec);
        }
    }

    // ---- hand-off: every wave drains its write-through stores, then one lane counts the
    // workgroup in; the last of the round replays the row block
    if (KQ_AO_DIAG & 4) {
        if (s == 0 && (int)threadIdx.x < nrows) p.y[row0 + (int)threadIdx.x] = p.res ? p.res[row0 + (int)threadIdx.x] : 0.f;
        return;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t old = __hip_atomic_fetch_add(p.cnt + rb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = old == (uint32_t)(nsb - 1);
        // every arrival of this launch has happened: the last arriver re-arms the counter, so
        // each launch starts at 0 whatever an earlier (aborted or diagnostic) launch left
        if (last) __hip_atomic_store(p.cnt + rb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return;

    // ---- the last arriver: row r's chain over its nsb records, in superblock order
    const int r = (int)threadIdx.x;
    if (r >= nrows) return;
    const uint8_t *rr = p.recs + (int64_t)(rb * p.R + r) * nsb * 16;
    float v = 0.f;
    // two batches of 8 records (32 VGPRs in flight), the second only for nsb > 8 (uniform)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        if (half == 1 && nsb <= 8) break;
        u32x4 rv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int k = 8 * half + i;
            rv[i] = load16_sc1(rr + 16 * (k < nsb ? k : nsb - 1));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(rv[i]));
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (8 * half + i < nsb) {
                Rec rc;
                rc.a = (int)rv[i].x;
                rc.b = (int)rv[i].y;
                rc.c = __uint_as_float(rv[i].z);
                rc.e = __uint_as_float(rv[i].w);
                v = chain_step(TYPE, rc, v);
            }
        }
    }
    p.y[row0 + r] = p.res ? v + resv : v;  // ggml_add(mul_mat, residual): one f32 add
}

#define KQ_AO_INST(HD, T) template __global__ void kq_attn_oproj<HD, T>(const AttnOprojArgs p);
KQ_AO_INST(64, Q4_K)
KQ_AO_INST(64, Q5_K)
KQ_AO_INST(64, Q6_K)
KQ_AO_INST(128, Q4_K)
KQ_AO_INST(128, Q5_K)
KQ_AO_INST(128, Q6_K)

// ------------------------------------------------------------------ host side
size_t attn_lds16(int hd, int n_ctx) {
    // kq_ops.hip attn_lds (the per-head layout of attn_head), rounded to 16 B
    const size_t gsum = (size_t)(n_ctx / 4) * 8 <= (size_t)hd * 64 ? 0 : (size_t)(n_ctx / 4) * 8;
    const size_t b = (size_t)6 * hd + (size_t)n_ctx * 6 + (size_t)hd * 64 + 16 + gsum;
    return (b + 15) & ~(size_t)15;
}

namespace {
struct AoShape {
    int hps, nsb, n_rb, R;
    size_t lds, recs_bytes;
};

bool ao_shape(int hd, int n_head, int n_head_kv, int n_ctx, int type, int64_t K, int64_t n_rows, AoShape &sh) {
    if (hd != 64 && hd != 128) return false;
    if (type != Q4_K && type != Q5_K && type != Q6_K) return false;
    // every row block re-runs its superblock's heads: at long contexts that replicated
    // KV-cache traffic outgrows the launch it saves (n_rb x the group's cells per head)
    if (n_ctx > kAttnOprojMaxCtx) return false;
    sh.hps = 256 / hd;
    if (n_head_kv <= 0 || n_head % n_head_kv || (n_head / n_head_kv) % sh.hps) return false;  // a superblock's heads share one KV group
    if (K != (int64_t)n_head * hd || K % QK) return false;
    sh.nsb = (int)(K / QK);
    if (sh.nsb > 16 || n_rows <= 0 || n_rows > (1 << 24)) return false;
    int n_rb = 256 / sh.nsb;
    const int nrb_knob = (int)knob(KNOB_AO_NRB);  // A/B only
    if (nrb_knob > 0) n_rb = nrb_knob;
    if (n_rb < 1) n_rb = 1;
    const int64_t max_rb = (n_rows + 15) / 16;
    if (n_rb > max_rb) n_rb = (int)max_rb;
    int64_t R = (n_rows + n_rb - 1) / n_rb;
    R = (R + 3) & ~(int64_t)3;
    n_rb = (int)((n_rows + R - 1) / R);
    if (R > 512) return false;  // the last arriver: one row per thread
    sh.n_rb = n_rb;
    sh.R = (int)R;
    const size_t head = attn_lds16(hd, n_ctx);
    const size_t wgran = ((size_t)R * pieces_of(type) + 63) / 64 * 64;
    sh.lds = (size_t)attn_oproj_wofs(sh.hps, (int)head) + wgran * 16;
    sh.recs_bytes = (size_t)n_rb * (size_t)R * (size_t)sh.nsb * 16;
    return sh.lds <= 160 * 1024;  // LDS per CU
}
}  // namespace

size_t attn_oproj_buffer(int hd, int n_head, int n_head_kv, int n_ctx, int type, int64_t K, int64_t n_rows, int *nsb) {
    AoShape sh;
    if (!ao_shape(hd, n_head, n_head_kv, n_ctx, type, K, n_rows, sh)) return 0;
    if (nsb) *nsb = sh.nsb;
    return kAttnOprojCounterBytes + sh.recs_bytes;
}

int launch_attn_oproj(const AttnArgs &a, int type, const void *w, int64_t n_rows, size_t row_stride, const float *res,
                      float *y, uint8_t *buf, size_t buf_size, hipStream_t stream) {
    AoShape sh;
    const int64_t K = (int64_t)a.n_head * a.head_dim;
    if (!ao_shape(a.head_dim, a.n_head, a.n_head_kv, a.n_ctx, type, K, n_rows, sh)) return MI355X_E_UNSUPPORTED;
    if (!w || !y || !buf || buf_size < kAttnOprojCounterBytes + sh.recs_bytes) return MI355X_E_INVAL;
    if (sh.n_rb * 4 > (int)kAttnOprojCounterBytes) return MI355X_E_UNSUPPORTED;
    if (type != Q6_K && (((uintptr_t)w & 15u) || (row_stride & 15u))) return MI355X_E_UNSUPPORTED;
    if (row_stride < (size_t)sh.nsb * block_bytes(type)) return MI355X_E_INVAL;
    AttnOprojArgs p;
    memset(&p, 0, sizeof(p));
    p.at = a;
    p.w = (const uint8_t *)w;
    p.row_stride = (int64_t)row_stride;
    p.n_rows = (int)n_rows;
    p.nsb = sh.nsb;
    p.R = sh.R;
    p.n_rb = sh.n_rb;
    p.head_lds = (int)attn_lds16(a.head_dim, a.n_ctx);
    p.res = res;
    p.y = y;
    p.cnt = (uint32_t *)buf;
    p.recs = buf + kAttnOprojCounterBytes;
    const void *fn = a.head_dim == 64 ? (type == Q4_K   ? (const void *)kq_attn_oproj<64, Q4_K>
                                         : type == Q5_K ? (const void *)kq_attn_oproj<64, Q5_K>
                                                        : (const void *)kq_attn_oproj<64, Q6_K>)
                                      : (type == Q4_K   ? (const void *)kq_attn_oproj<128, Q4_K>
                                         : type == Q5_K ? (const void *)kq_attn_oproj<128, Q5_K>
                                                        : (const void *)kq_attn_oproj<128, Q6_K>);
    allow_lds(fn, sh.lds);
    const dim3 grid((unsigned)(sh.nsb * sh.n_rb)), block(512u);
    void *args[] = {&p};
    hipEvent_t e0, e1;
    hipError_t e;
    if (timing_slot(stream, e0, e1)) {
        e = hipExtLaunchKernel(fn, grid, block, args, sh.lds, stream, e0, e1, 0);
        const std::string name = std::string("kq::kq_attn_oproj<") + std::to_string(a.head_dim) + ", " +
                                 std::to_string(type) + ">";
        timing_log(name, (double)n_rows * sh.nsb * block_bytes(type) + (double)n_rows * 4.0 * (res ? 2 : 1), e0, e1);
    } else {
        e = hipLaunchKernel(fn, grid, block, args, sh.lds, stream);
    }
    if (e != hipSuccess) return (int)e;
    e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

}  // namespace kq
