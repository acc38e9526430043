// kq_backend.hip — the ggml-backend mirror: a HIP "device" that owns a stream,
// device buffers and a hipGraph cache, and executes MUL_MAT nodes.
//
// Sibling of the reference's CPU backend entry ggml_backend_cpu_graph_compute
// (ggml-cpu.cpp:186, README.md:162), called by the scheduler at
// ggml_backend_sched_compute_splits (ggml-backend.cpp:1553, README.md:163).
// Where the CPU backend fans the graph out to OpenMP threads and each thread
// walks every node (ggml_graph_compute_thread, ggml-cpu.c:2883), this backend
// enqueues one kernel per (fused) node on its HIP stream; repeated graphs
// (decode steps) are replayed from a captured hipGraph.
#include <algorithm>
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "kq_common.h"
#include "kq_internal.h"

struct mi355x_backend {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string name;
    void *workspace = nullptr;
    size_t workspace_size = 0;
    // captured hipGraphs by node-list key, most recently used last (the decode token and
    // a prompt batch alternate without recapturing)
    struct Captured {
        std::vector<uint64_t> key;
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
    };
    std::vector<Captured> graphs;
    bool fuse = true;
    bool attn_oproj = false;  // decode attention + o-proj GEMV in one launch (kq_attn_oproj.hip): measured
                              // slower than the two launches, so opt-in
    void *fx = nullptr;      // its arrival counters (zeroed at allocation) and records
    size_t fx_size = 0;
    int fx_nsb = 0;          // the superblock count the counters' rounds are aligned to
    bool layer_engine = false;  // each decode layer as one persistent launch (kq_layer.hip)
    uint32_t *ly_sync = nullptr;  // the persistent layers' counter blocks (zeroed at allocation), then err
    int ly_blocks = 0;
    std::vector<std::vector<uint32_t>> ly_keys;  // block i's (layer index, producers per edge and shard)
    struct LyTab {                 // step tables (kq::layer_table_fill) built for one full geometry `key`
        void *dev = nullptr;
        int64_t stride = 0;
        std::vector<uint64_t> key;
    };
    std::vector<LyTab> ly_tabs;    // one entry per distinct key (several models / cache sizes coexist)
    ncclComm_t comm = nullptr;  // row split: one RCCL communicator per backend (rank of a world)
    bool loop_nocopy = false;   // emulated rank, timing only (MI355X_LOOPBACK_NOCOPY)
    int rank = 0, world = 0;
    int loop_rank = -1, loop_world = 0;  // single-GPU emulation of one rank (tests)
};

namespace {

// Every backend entry point runs on the backend's own device and restores the
// caller's current device afterwards (ggml-cuda's ggml_cuda_set_device discipline):
// one process may hold several backends (llama.cpp's layer split).
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~DeviceGuard() {
        if (prev >= 0) hipSetDevice(prev);
    }
};

// The persistent layers' step tables depend on every field layer_table_fill reads: the
// weights and their types, the stage shapes, the ring geometry (D, slot: byte positions
// and issue gates) and the attention placement and LDS layout (which move with n_ctx).
constexpr size_t kMaxLyTabs = 256;

std::vector<uint64_t> ly_tab_key(const kq::LayerArgs &la) {
    std::vector<uint64_t> key = {(uint64_t)la.G,      (uint64_t)la.E,           (uint64_t)la.F,
                                 (uint64_t)la.nb_e,   (uint64_t)la.nb_f,        (uint64_t)la.nq,
                                 (uint64_t)la.nkv,    (uint64_t)la.n_attn,      (uint64_t)la.hpw,
                                 (uint64_t)la.attn_stride, (uint64_t)la.head_lds, (uint64_t)la.D,
                                 (uint64_t)la.slot,   (uint64_t)la.o_aux,       (uint64_t)la.act_bytes,
                                 (uint64_t)la.o_sums, (uint64_t)la.o_res,       (uint64_t)la.lds};
    for (int m = 0; m < 7; ++m) {
        key.push_back((uint64_t)(uintptr_t)la.w[m]);
        key.push_back((uint64_t)la.type[m]);
    }
    return key;
}

// ---- RCCL, resolved at run time: the copy already loaded in the process (torch
// bundles one) or /opt/rocm's. Only the entry points the row split uses.
struct Rccl {
    bool tried = false, ok = false;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

Rccl &rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        fprintf(stderr, "ggml_mi355x: librccl.so.1 not found (%s)\n", dlerror());
        return r;
    }
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.all_reduce && r.error_string;
    return r;
}

bool is_kquant(int t) { return t == MI355X_TYPE_Q4_K || t == MI355X_TYPE_Q5_K || t == MI355X_TYPE_Q6_K; }

constexpr size_t kMaxGraphs = 4;

void destroy_captured(mi355x_backend::Captured &c) {
    if (c.exec) hipGraphExecDestroy(c.exec);
    if (c.graph) hipGraphDestroy(c.graph);
    c.exec = nullptr;
    c.graph = nullptr;
}

void drop_graph(mi355x_backend *b) {
    for (auto &c : b->graphs) destroy_captured(c);
    b->graphs.clear();
}

// the captured graph of this node list (moved to the back: most recently used), or null
mi355x_backend::Captured *find_graph(mi355x_backend *b, const std::vector<uint64_t> &key) {
    for (size_t i = 0; i < b->graphs.size(); ++i)
        if (b->graphs[i].key == key) {
            if (i + 1 != b->graphs.size()) {
                mi355x_backend::Captured c = b->graphs[i];
                b->graphs.erase(b->graphs.begin() + (long)i);
                b->graphs.push_back(c);
            }
            return &b->graphs.back();
        }
    return nullptr;
}

const mi355x_backend::LyTab *find_ly_tab(const mi355x_backend *b, const std::vector<uint64_t> &key) {
    for (const auto &t : b->ly_tabs)
        if (t.dev && t.key == key) return &t;
    return nullptr;
}

// One launch: a MUL_MAT node, or a run of ne11 == 1 MUL_MAT nodes sharing src1
// (kind GEMV, with its fused neighbours), or any other single node.
struct Launch {
    int first, count;  // nodes[first .. first+count): the MUL_MAT run, or the single node
    int kind = 0;      // 0 single node, 1 MUL_MAT run (GEMV), 2 prefill prologue -> Q8L, 3 batched MUL_MAT + ADD,
                       // 4 batched MUL_MATs of one type on one activation in one tile-GEMM launch,
                       // 5 decode ATTN_DECODE -> MUL_MAT (-> ADD) in one launch (kq_attn_oproj),
                       // 6 a whole decode layer (15 nodes) in one persistent launch (kq_layer)
    const mi355x_tensor *q8_of = nullptr;  // kind 2: the node whose (never written) output the Q8L blocks stand for
    int pro = MI355X_PRO_NONE;
    const float *x = nullptr, *x2 = nullptr;  // GEMV input (prologue source) and its second operand
    float eps = 0.f;
    float *y[MI355X_MAX_FUSED] = {};
    const float *res[MI355X_MAX_FUSED] = {};
    const float *norm_w = nullptr;  // single RMS_NORM with its MUL fused
    float *norm_y = nullptr;
    float *epi_y = nullptr;  // GEMV run [gate, up] with the SWIGLU node fused as its epilogue
    int ly_block = -1;       // kind 6: its counter block
    kq::LayerArgs la;        // kind 6: the launch's arguments (sync / err set at enqueue)
};

// a persistent layer launch's counter block key (see graph_compute)
std::vector<uint32_t> ly_block_key(const Launch &l) {
    std::vector<uint32_t> k = {(uint32_t)l.ly_block};
    for (int e = 0; e < 4; ++e)
        for (int q = 0; q < 8; ++q) k.push_back(l.la.expect[e][q]);
    return k;
}

int find_ly_block(const mi355x_backend *b, const std::vector<uint32_t> &k) {
    for (size_t i = 0; i < b->ly_keys.size(); ++i)
        if (b->ly_keys[i] == k) return (int)i;
    return -1;
}

float f_of(int32_t bits) {
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

// Byte range [lo, hi) a tensor's data spans (ggml_nbytes: the last element of every
// dim; K-quant rows are whole blocks).
struct Span {
    uintptr_t lo = 0, hi = 0;
};
Span span_of(const mi355x_tensor *t) {
    Span s;
    if (!t || !t->data) return s;
    const int64_t blck = is_kquant(t->type) ? MI355X_QK_K : 1;
    uint64_t bytes = (uint64_t)(t->ne[0] / blck) * t->nb[0];
    for (int d = 1; d < 4; ++d)
        if (t->ne[d] > 1) bytes += (uint64_t)(t->ne[d] - 1) * t->nb[d];
    s.lo = (uintptr_t)t->data;
    s.hi = s.lo + (uintptr_t)bytes;
    return s;
}

// readers[i]: number of node operands (over all nodes) that read node i's output.
// A read is credited to the LATEST earlier node whose output overlaps the operand's
// bytes (ggml-alloc reuses a dead node's buffer for a later node, so the latest
// writer is the producer); reads through views at an offset count too. When the
// latest overlapping writer does not cover the whole operand, older overlapping
// writers are credited as well: over-counting only disables a fusion, it never
// elides a live output.
std::vector<int> count_readers(mi355x_tensor *const *nodes, int n) {
    std::vector<int> r(n, 0);
    std::vector<Span> out(n);
    for (int i = 0; i < n; ++i)
        if (nodes[i]->op != MI355X_OP_NONE) out[i] = span_of(nodes[i]);
    for (int j = 0; j < n; ++j)
        for (int s = 0; s < MI355X_MAX_SRC; ++s) {
            const mi355x_tensor *u = nodes[j]->src[s];
            if (!u) continue;
            const Span us = span_of(u);
            for (int i = j - 1; i >= 0; --i) {
                if (nodes[i] == u) {  // the operand IS node i (whatever its buffer)
                    ++r[i];
                    break;
                }
                const Span &o = out[i];
                if (o.hi <= o.lo || us.hi <= us.lo || !(o.lo < us.hi && us.lo < o.hi)) continue;
                ++r[i];
                if (o.lo <= us.lo && us.hi <= o.hi) break;  // fully produced by node i
            }
        }
    return r;
}

int64_t nelem(const mi355x_tensor *t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }

bool elidable(const mi355x_tensor *t, int readers) {
    return readers == 1 && !(t->flags & MI355X_TENSOR_FLAG_OUTPUT);
}

bool is_gemv_node(const mi355x_tensor *t) { return t->op == MI355X_OP_MUL_MAT && t->src[1]->ne[1] == 1; }

// A MUL_MAT of ne11 >= 16 columns on the int8-MFMA GEMM whose activation the previous
// launch already quantized into the workspace (q/k/v and gate/up of a prompt batch read
// one normed activation): the GEMM alone. q8_src tracks what the workspace holds.
struct Q8State {
    const void *src = nullptr;
    int64_t k = 0, m = 0;
    size_t nb = 0;
    bool f16 = false;  // the workspace holds kq_mmf's f16 activation image, not Q8L blocks
};

int enqueue_batched_mm(mi355x_backend *b, const mi355x_tensor *t, Q8State &q8, float *y = nullptr,
                       int64_t y_stride = 0, const float *res = nullptr, int64_t res_stride = 0) {
    const mi355x_tensor *w = t->src[0], *x = t->src[1];
    if (!y) {
        y = (float *)t->data;
        y_stride = (int64_t)(t->nb[1] / 4);
    }
    const int64_t K = w->ne[0], M = x->ne[1];
    const bool f16 = kq::mmf_applies(w->type, w->data, w->ne[1], w->nb[1], M, K);
    const bool same = q8.src == x->data && q8.k == K && q8.m == M && q8.nb == x->nb[1] && q8.f16 == f16;
    if (f16) {  // the stated-tolerance f16 path: image once per activation, then the GEMM
        int rc = 0;
        if (!same) {
            rc = kq::launch_f16img((const float *)x->data, (int64_t)(x->nb[1] / 4), (uint8_t *)b->workspace, K, M,
                                   b->stream);
            q8 = Q8State();
            if (rc) return rc;
            q8.src = x->data, q8.k = K, q8.m = M, q8.nb = x->nb[1], q8.f16 = true;
        }
        rc = kq::launch_mmf_gemm(w->type, w->data, K, w->ne[1], w->nb[1], (uint8_t *)b->workspace, M, y, y_stride,
                                 b->stream, res, res_stride);
        const uintptr_t o0 = (uintptr_t)y, o1 = o0 + (size_t)y_stride * 4 * (size_t)t->ne[1];
        const uintptr_t s0 = (uintptr_t)q8.src, s1 = s0 + q8.nb * (size_t)q8.m;
        if (rc || (o0 < s1 && s0 < o1)) q8 = Q8State();
        return rc;
    }
    if (!same) {
        const int rc = kq::launch_quantize_q8L((const float *)x->data, (int64_t)(x->nb[1] / 4), b->workspace, K, M,
                                               b->stream, true);
        if (rc) {
            q8 = Q8State();
            return rc;
        }
        q8.src = x->data;
        q8.k = K;
        q8.m = M;
        q8.nb = x->nb[1];
    }
    const int rc = kq::launch_mmq(w->type, w->data, K, w->ne[1], w->nb[1], (const uint8_t *)b->workspace, M, y,
                                  y_stride, b->stream, res, res_stride);
    // an output overlapping the quantized activation's bytes invalidates it
    const uintptr_t o0 = (uintptr_t)y, o1 = o0 + (size_t)y_stride * 4 * (size_t)t->ne[1];
    const uintptr_t s0 = (uintptr_t)q8.src, s1 = s0 + q8.nb * (size_t)q8.m;
    if (rc || (o0 < s1 && s0 < o1)) q8 = Q8State();
    return rc;
}

void attn_desc_of(const mi355x_tensor *t, mi355x_attn_desc &a) {
    a.q = (const float *)t->src[0]->data;
    a.k = (const float *)t->src[1]->data;
    a.v = (const float *)t->src[2]->data;
    a.pos = (const int32_t *)t->src[3]->data;
    a.k_cache = (uint16_t *)t->src[4]->data;
    a.v_cache = (uint16_t *)t->src[5]->data;
    a.rope_table = (const float *)t->src[6]->data;
    a.out = (float *)t->data;
    a.n_head = t->op_params[0];
    a.n_head_kv = t->op_params[1];
    a.head_dim = t->op_params[2];
    a.scale = f_of(t->op_params[3]);
    a.n_ctx = (int)t->src[4]->ne[1];
}

// A batched MUL_MAT that runs on the int8 GEMM (kq_mmq, Q8L activation blocks): always in
// the exact precision, and in the f16 one where kq_mmf is not the faster kernel
bool mm_exact(const mi355x_tensor *t) {
    const mi355x_tensor *w = t->src[0], *x = t->src[1];
    return !kq::mmf_applies(w->type, w->data, w->ne[1], w->nb[1], x->ne[1], w->ne[0]);
}

bool batched_mm_shares(const mi355x_backend *b, const mi355x_tensor *t) {
    if (t->op != MI355X_OP_MUL_MAT) return false;
    const mi355x_tensor *w = t->src[0], *x = t->src[1];
    if (x->ne[1] < 16 || (x->nb[1] & 3u) || (t->nb[1] & 3u) || ((uintptr_t)b->workspace & 15u)) return false;
    if (!kq::mmf_applies(w->type, w->data, w->ne[1], w->nb[1], x->ne[1], w->ne[0]) &&
        !kq::mmq_applies(w->type, w->data, w->ne[1], w->nb[1], x->ne[1]))
        return false;
    return b->workspace_size >= mi355x_mul_mat_workspace_size(w->type, w->ne[0], w->ne[1], x->ne[1]);
}

// MUL_MATs that can share one tile-GEMM launch: one type, or K-quants of different types
// (kq_mmq_mixed: a prompt batch's Q4_K / Q5_K q/k with the Q6_K attn_v of use_more_bits layers)
bool multi_types_ok(int a, int b) { return a == b || (is_kquant(a) && is_kquant(b)); }

// A decode attention whose output only the next node, a GEMV (the o-proj), reads: both
// run as one kq_attn_oproj launch when its shape allows (bit-identical: kq_attn_oproj.hip).
bool attn_oproj_fusable(const mi355x_backend *b, const mi355x_tensor *t, const mi355x_tensor *mm, int readers) {
    const int ko = (int)kq::knob(kq::KNOB_ATTN_OPROJ);  // A/B: 0 never, 2 every backend
    if (ko == 0 || (ko == 1 && !b->attn_oproj) || t->op != MI355X_OP_ATTN_DECODE || t->src[0]->ne[1] != 1) return false;
    if (kq::attn_impl() == MI355X_ATTN_GROUP || !elidable(t, readers)) return false;  // (per-head kernels)
    if (!is_gemv_node(mm) || mm->src[1] != t || !is_kquant(mm->src[0]->type)) return false;
    const mi355x_tensor *w = mm->src[0];
    if (w->ne[0] != t->ne[0] || w->ne[2] != 1 || w->ne[3] != 1 || mm->nb[0] != 4) return false;
    const int nh = t->op_params[0], nkv = t->op_params[1], hd = t->op_params[2];
    return kq::attn_oproj_buffer(hd, nh, nkv, (int)t->src[4]->ne[1], w->type, w->ne[0], w->ne[1], nullptr) > 0;
}

// ---- kind 6: the 15 nodes of one llm_build_llama decode layer as one kq_layer launch
bool contiguous_kq(const mi355x_tensor *w) {
    return is_kquant(w->type) && w->ne[0] % MI355X_QK_K == 0 && w->ne[2] == 1 && w->ne[3] == 1 &&
           w->nb[1] == (size_t)(w->ne[0] / MI355X_QK_K) * mi355x_row_size(w->type, MI355X_QK_K) &&
           (w->type == MI355X_TYPE_Q6_K || ((uintptr_t)w->data & 15u) == 0);
}
bool f32_vec(const mi355x_tensor *t, int64_t n, bool aligned16) {
    return t && t->type == MI355X_TYPE_F32 && nelem(t) == n && t->ne[0] == n && t->nb[0] == 4 && t->data &&
           (!aligned16 || ((uintptr_t)t->data & 15u) == 0);
}
// ADD(a, b) where one operand is node `mm` and the other is `res`'s bytes: true
bool add_of(const mi355x_tensor *ad, const mi355x_tensor *mm, const mi355x_tensor *res) {
    if (!ad || ad->op != MI355X_OP_ADD) return false;
    const int s = ad->src[0] == mm ? 0 : ad->src[1] == mm ? 1 : -1;
    if (s < 0) return false;
    const mi355x_tensor *o = ad->src[1 - s];
    return o && o->data == res->data && o->type == MI355X_TYPE_F32 && nelem(o) == nelem(res);
}
bool spans_overlap(const mi355x_tensor *p, const mi355x_tensor *q) {
    const Span a = span_of(p), c = span_of(q);
    return a.lo < c.hi && c.lo < a.hi;
}

bool layer_match(const mi355x_backend *b, mi355x_tensor *const *nodes, int n, int i, const std::vector<int> &readers,
                 kq::LayerArgs &la) {
    if (!b->layer_engine || i + 15 > n) return false;
    mi355x_tensor *const *t = nodes + i;
    const mi355x_tensor *n1 = t[0], *m1 = t[1], *q = t[2], *k = t[3], *v = t[4], *at = t[5], *o = t[6], *x1 = t[7];
    const mi355x_tensor *n2 = t[8], *m2 = t[9], *g = t[10], *u = t[11], *sw = t[12], *dn = t[13], *x2 = t[14];
    if (n1->op != MI355X_OP_RMS_NORM || m1->op != MI355X_OP_MUL || m1->src[0] != n1) return false;
    const mi355x_tensor *x = n1->src[0];
    const int64_t E = n1->ne[0];
    if (!f32_vec(x, E, true) || !f32_vec(n1, E, false) || !f32_vec(m1->src[1], E, true) || !f32_vec(m1, E, false))
        return false;
    if (!elidable(n1, readers[i]) || readers[i + 1] != 3 || (m1->flags & MI355X_TENSOR_FLAG_OUTPUT)) return false;
    for (const mi355x_tensor *mm : {q, k, v})
        if (!is_gemv_node(mm) || mm->src[1] != m1 || !contiguous_kq(mm->src[0]) || mm->src[0]->ne[0] != E ||
            !f32_vec(mm, mm->src[0]->ne[1], true))
            return false;
    if (at->op != MI355X_OP_ATTN_DECODE || at->src[0] != q || at->src[1] != k || at->src[2] != v) return false;
    if (at->src[6]->ne[1] != 1) return false;  // the position's rope row staged with the inputs
    const int nh = at->op_params[0], nkv = at->op_params[1], hd = at->op_params[2];
    if (k->src[0]->ne[1] != v->src[0]->ne[1] || (int64_t)nh * hd != q->src[0]->ne[1] || q->src[0]->ne[1] != E ||
        (int64_t)nkv * hd != k->src[0]->ne[1] || !f32_vec(at, E, true))
        return false;
    if (!is_gemv_node(o) || o->src[1] != at || !contiguous_kq(o->src[0]) || o->src[0]->ne[0] != E ||
        o->src[0]->ne[1] != E || !elidable(o, readers[i + 6]))
        return false;
    if (!add_of(x1, o, x) || !f32_vec(x1, E, true)) return false;
    if (n2->op != MI355X_OP_RMS_NORM || n2->src[0] != x1 || !elidable(n2, readers[i + 8]) || m2->op != MI355X_OP_MUL ||
        m2->src[0] != n2 || !f32_vec(m2->src[1], E, true) || readers[i + 9] != 2 ||
        (m2->flags & MI355X_TENSOR_FLAG_OUTPUT))
        return false;
    if (f_of(n1->op_params[0]) != f_of(n2->op_params[0])) return false;  // one eps per layer (llama)
    for (const mi355x_tensor *mm : {g, u})
        if (!is_gemv_node(mm) || mm->src[1] != m2 || !contiguous_kq(mm->src[0]) || mm->src[0]->ne[0] != E)
            return false;
    const int64_t F = g->src[0]->ne[1];
    if (u->src[0]->ne[1] != F || !elidable(g, readers[i + 10]) || !elidable(u, readers[i + 11])) return false;
    if (sw->op != MI355X_OP_SWIGLU || sw->src[0] != g || sw->src[1] != u || !f32_vec(sw, F, true)) return false;
    if (!is_gemv_node(dn) || dn->src[1] != sw || !contiguous_kq(dn->src[0]) || dn->src[0]->ne[0] != F ||
        dn->src[0]->ne[1] != E || !elidable(dn, readers[i + 13]))
        return false;
    if (!add_of(x2, dn, x1) || !f32_vec(x2, E, false)) return false;
    // written in the launch: q, k, v, att, x1, h, x2 -- none of them over an input or another
    const mi355x_tensor *wr[6] = {q, k, v, at, x1, sw};
    for (int a0 = 0; a0 < 6; ++a0) {
        if (spans_overlap(wr[a0], x) || spans_overlap(wr[a0], x2)) return false;
        for (int a1 = a0 + 1; a1 < 6; ++a1)
            if (spans_overlap(wr[a0], wr[a1])) return false;
    }
    memset(&la, 0, sizeof(la));
    la.E = (int)E;
    la.F = (int)F;
    la.nq = (int)q->src[0]->ne[1];
    la.nkv = (int)k->src[0]->ne[1];
    const mi355x_tensor *ws[7] = {q->src[0], k->src[0], v->src[0], o->src[0], g->src[0], u->src[0], dn->src[0]};
    for (int m = 0; m < 7; ++m) {
        la.type[m] = ws[m]->type;
        la.w[m] = (const uint8_t *)ws[m]->data;
    }
    la.y[0] = (float *)q->data;
    la.y[1] = (float *)k->data;
    la.y[2] = (float *)v->data;
    la.x = (const float *)x->data;
    la.attn_norm = (const float *)m1->src[1]->data;
    la.ffn_norm = (const float *)m2->src[1]->data;
    la.eps = f_of(n1->op_params[0]);
    la.att = (float *)at->data;
    la.x1 = (float *)x1->data;
    la.h = (float *)sw->data;
    la.x2 = (float *)x2->data;
    mi355x_attn_desc d;
    attn_desc_of(at, d);
    d.rope_row = 1;
    if (kq::attn_args_from(&d, la.at) != 0) return false;
    return kq::layer_plan(la, hd, nh) == MI355X_OK;
}

std::vector<Launch> plan_launches(const mi355x_backend *b, mi355x_tensor *const *nodes, int n, bool fuse) {
    std::vector<Launch> out;
    const std::vector<int> readers = fuse ? count_readers(nodes, n) : std::vector<int>(n, 0);
    auto index_of = [&](const mi355x_tensor *u, int lo, int hi) {
        for (int i = lo; i < hi; ++i)
            if (nodes[i] == u) return i;
        return -1;
    };
    int i = 0, ly_blocks = 0;
    while (i < n) {
        const mi355x_tensor *t = nodes[i];
        Launch l;
        l.first = i;
        l.count = 1;
        int head = i;  // first MUL_MAT of a run
        if (fuse && layer_match(b, nodes, n, i, readers, l.la)) {
            l.kind = 6;
            l.count = 15;
            l.ly_block = ly_blocks++;
            out.push_back(l);
            i += 15;
            continue;
        }
        if (fuse && i + 1 < n && attn_oproj_fusable(b, t, nodes[i + 1], readers[i])) {
            const mi355x_tensor *mm = nodes[i + 1];
            l.kind = 5;
            l.count = 2;
            l.y[0] = (float *)mm->data;
            int end = i + 2;
            if (end < n && nodes[end]->op == MI355X_OP_ADD && elidable(mm, readers[i + 1])) {
                const mi355x_tensor *ad = nodes[end];
                const int s_mm = ad->src[0] == mm ? 0 : ad->src[1] == mm ? 1 : -1;
                const mi355x_tensor *other = s_mm >= 0 ? ad->src[1 - s_mm] : nullptr;
                if (other && index_of(other, i, end) < 0 && ad->ne[0] == mm->ne[0] && ad->ne[1] == 1 &&
                    ad->type == MI355X_TYPE_F32 && other->type == MI355X_TYPE_F32 && nelem(other) == ad->ne[0] &&
                    other->nb[0] == 4 && ad->nb[0] == 4) {
                    l.res[0] = (const float *)other->data;
                    l.y[0] = (float *)ad->data;
                    l.count = 3;
                    ++end;
                }
            }
            out.push_back(l);
            i = end;
            continue;
        }
        // prologue fusion: RMS_NORM -> MUL -> MUL_MAT run, SWIGLU -> MUL_MAT run
        if (fuse && t->op == MI355X_OP_RMS_NORM && i + 2 < n && nodes[i + 1]->op == MI355X_OP_MUL &&
            nodes[i + 1]->src[0] == t && elidable(t, readers[i]) && is_gemv_node(nodes[i + 2]) &&
            nodes[i + 2]->src[1] == nodes[i + 1] && nodes[i + 1]->ne[0] == t->ne[0] && t->ne[1] == 1) {
            int cnt = 0;
            while (i + 2 + cnt < n && cnt < MI355X_MAX_FUSED && is_gemv_node(nodes[i + 2 + cnt]) &&
                   nodes[i + 2 + cnt]->src[1] == nodes[i + 1])
                ++cnt;
            if (readers[i + 1] == cnt && !(nodes[i + 1]->flags & MI355X_TENSOR_FLAG_OUTPUT)) {
                l.pro = MI355X_PRO_RMS_NORM;
                l.x = (const float *)t->src[0]->data;
                l.x2 = (const float *)nodes[i + 1]->src[1]->data;
                l.eps = f_of(t->op_params[0]);
                head = i + 2;
            }
        } else if (fuse && t->op == MI355X_OP_SWIGLU && i + 1 < n && is_gemv_node(nodes[i + 1]) &&
                   nodes[i + 1]->src[1] == t && elidable(t, readers[i]) && t->ne[1] == 1) {
            l.pro = MI355X_PRO_SWIGLU;
            l.x = (const float *)t->src[0]->data;
            l.x2 = (const float *)t->src[1]->data;
            head = i + 1;
        }
        const mi355x_tensor *h = nodes[head];
        if (h->op == MI355X_OP_MUL_MAT && h->src[1]->ne[1] == 1 && (l.pro != MI355X_PRO_NONE || head == i)) {
            int cnt = 1;
            while (head + cnt < n && cnt < MI355X_MAX_FUSED) {
                const mi355x_tensor *u = nodes[head + cnt];
                if (!is_gemv_node(u)) break;
                if (u->src[1]->data != h->src[1]->data || u->src[0]->ne[0] != h->src[0]->ne[0]) break;
                ++cnt;
            }
            l.kind = 1;
            l.first = head;
            l.count = cnt;
            if (l.pro == MI355X_PRO_NONE) l.x = (const float *)h->src[1]->data;
            for (int k = 0; k < cnt; ++k) l.y[k] = (float *)nodes[head + k]->data;
            int end = head + cnt;
            // epilogue fusion: ADD(mul_mat, residual) right after the run (the last
            // MUL_MAT's output, or any of the run's outputs, one ADD each)
            while (fuse && end < n && nodes[end]->op == MI355X_OP_ADD) {
                const mi355x_tensor *ad = nodes[end];
                int k = -1, other = -1;
                for (int s2 = 0; s2 < 2 && k < 0; ++s2) {
                    const int j = index_of(ad->src[s2], head, head + cnt);
                    if (j >= 0) {
                        k = j - head;
                        other = 1 - s2;
                    }
                }
                if (k < 0 || l.res[k] || !elidable(nodes[head + k], readers[head + k])) break;
                if (index_of(ad->src[other], i, end) >= 0) break;  // residual produced inside the fused range
                if (ad->ne[0] != nodes[head + k]->ne[0] || ad->ne[1] != 1 || ad->type != MI355X_TYPE_F32) break;
                l.res[k] = (const float *)ad->src[other]->data;
                l.y[k] = (float *)ad->data;
                ++end;
            }
            // epilogue fusion: SWIGLU(gate, up) of a two-MUL_MAT run whose outputs only it reads
            if (fuse && end < n && cnt == 2 && nodes[end]->op == MI355X_OP_SWIGLU && !l.res[0] && !l.res[1]) {
                const mi355x_tensor *sg = nodes[end];
                if (sg->src[0] == nodes[head] && sg->src[1] == nodes[head + 1] && elidable(nodes[head], readers[head]) &&
                    elidable(nodes[head + 1], readers[head + 1]) && nodes[head]->ne[0] == nodes[head + 1]->ne[0] &&
                    sg->ne[0] == nodes[head]->ne[0] && sg->ne[1] == 1 && sg->type == MI355X_TYPE_F32) {
                    l.epi_y = (float *)sg->data;
                    ++end;
                }
            }
            out.push_back(l);
            i = end;
            continue;
        }
        // prefill (batched, ne11 >= 16) fusions: the normed / swiglu'd activation goes straight
        // into the GEMMs' Q8L blocks (never written as f32), and MUL_MAT -> ADD as the GEMM's
        // epilogue; only where every consumer takes the shared-activation GEMM. On the f16
        // path (kq_mmf) only where every consumer stays on the int8 GEMM: kq_mmf reads an f16
        // image of the f32 activation.
        if (fuse) {
            auto shares_run = [&](int first, const mi355x_tensor *src, int &cnt) {
                cnt = 0;
                while (first + cnt < n && nodes[first + cnt]->op == MI355X_OP_MUL_MAT &&
                       nodes[first + cnt]->src[1] == src && batched_mm_shares(b, nodes[first + cnt]) &&
                       mm_exact(nodes[first + cnt]))
                    ++cnt;
                return cnt > 0;
            };
            int cnt = 0;
            if (t->op == MI355X_OP_RMS_NORM && t->ne[1] >= 16 && i + 2 < n && nodes[i + 1]->op == MI355X_OP_MUL &&
                nodes[i + 1]->src[0] == t && elidable(t, readers[i]) && nodes[i + 1]->ne[0] == t->ne[0] &&
                nodes[i + 1]->ne[1] == t->ne[1] && nodes[i + 1]->src[1]->ne[0] == t->ne[0] &&
                nelem(nodes[i + 1]->src[1]) == t->ne[0] && t->nb[1] == (size_t)t->ne[0] * 4 &&
                t->src[0]->nb[1] == (size_t)t->ne[0] * 4 && ((uintptr_t)t->src[0]->data & 15u) == 0 &&
                !(nodes[i + 1]->flags & MI355X_TENSOR_FLAG_OUTPUT) && shares_run(i + 2, nodes[i + 1], cnt) &&
                readers[i + 1] == cnt) {
                l.kind = 2;
                l.pro = MI355X_PRO_RMS_NORM;
                l.x = (const float *)t->src[0]->data;
                l.x2 = (const float *)nodes[i + 1]->src[1]->data;
                l.eps = f_of(t->op_params[0]);
                l.q8_of = nodes[i + 1];
                l.count = 2;
                out.push_back(l);
                i += 2;
                continue;
            }
            if (t->op == MI355X_OP_SWIGLU && t->ne[1] >= 16 && t->ne[0] % MI355X_QK_K == 0 &&
                t->nb[1] == (size_t)t->ne[0] * 4 && t->src[0]->nb[1] == t->nb[1] && t->src[1]->nb[1] == t->nb[1] &&
                nelem(t->src[0]) == nelem(t) && nelem(t->src[1]) == nelem(t) && !(t->flags & MI355X_TENSOR_FLAG_OUTPUT) &&
                shares_run(i + 1, t, cnt) && readers[i] == cnt) {
                l.kind = 2;
                l.pro = MI355X_PRO_SWIGLU;
                l.x = (const float *)t->src[0]->data;
                l.x2 = (const float *)t->src[1]->data;
                l.q8_of = t;
                out.push_back(l);
                i += 1;
                continue;
            }
            if (t->op == MI355X_OP_MUL_MAT && t->src[1]->ne[1] >= 16 && batched_mm_shares(b, t) &&
                kq::mmq_tile64(t->src[0]->type, t->src[0]->ne[1], t->src[1]->ne[1])) {
                // (the f16 GEMM: one weight type per launch)
                int run = 1;
                while (i + run < n && run < 4) {
                    const mi355x_tensor *u = nodes[i + run];
                    if (u->op != MI355X_OP_MUL_MAT || u->src[1] != t->src[1] ||
                        !(mm_exact(t) ? multi_types_ok(t->src[0]->type, u->src[0]->type)
                                      : t->src[0]->type == u->src[0]->type) ||
                        u->src[0]->ne[0] != t->src[0]->ne[0] || !batched_mm_shares(b, u) ||
                        !kq::mmq_tile64(u->src[0]->type, u->src[0]->ne[1], u->src[1]->ne[1]))
                        break;
                    ++run;
                }
                if (run >= 2) {
                    l.kind = 4;
                    l.count = run;
                    out.push_back(l);
                    i += run;
                    continue;
                }
            }
            if (t->op == MI355X_OP_MUL_MAT && t->src[1]->ne[1] >= 16 && i + 1 < n && nodes[i + 1]->op == MI355X_OP_ADD &&
                elidable(t, readers[i]) && batched_mm_shares(b, t)) {
                const mi355x_tensor *ad = nodes[i + 1];
                const int s_mm = ad->src[0] == t ? 0 : ad->src[1] == t ? 1 : -1;
                const mi355x_tensor *other = s_mm >= 0 ? ad->src[1 - s_mm] : nullptr;
                if (other && ad->ne[0] == t->ne[0] && ad->ne[1] == t->ne[1] && other->ne[0] == t->ne[0] &&
                    other->ne[1] == t->ne[1] && other->nb[0] == 4 && ad->nb[0] == 4 && ad->type == MI355X_TYPE_F32 &&
                    other->type == MI355X_TYPE_F32) {
                    l.kind = 3;
                    l.res[0] = (const float *)other->data;
                    l.y[0] = (float *)ad->data;
                    l.count = 2;
                    out.push_back(l);
                    i += 2;
                    continue;
                }
            }
        }
        // single node (with RMS_NORM -> MUL fused when the norm output is only read by the MUL)
        if (fuse && t->op == MI355X_OP_RMS_NORM && i + 1 < n && nodes[i + 1]->op == MI355X_OP_MUL &&
            nodes[i + 1]->src[0] == t && elidable(t, readers[i]) && nodes[i + 1]->ne[0] == t->ne[0] &&
            nodes[i + 1]->src[1]->ne[0] == t->ne[0] && nodes[i + 1]->src[1]->ne[1] == 1) {
            l.norm_w = (const float *)nodes[i + 1]->src[1]->data;
            l.norm_y = (float *)nodes[i + 1]->data;
            l.count = 2;
        }
        out.push_back(l);
        i += l.count;
    }
    return out;
}


int enqueue_node(mi355x_backend *b, const Launch &l, const mi355x_tensor *t) {
    hipStream_t st = b->stream;
    switch (t->op) {
        case MI355X_OP_NONE:
            return 0;
        case MI355X_OP_MUL_MAT: {
            const mi355x_tensor *w = t->src[0], *x = t->src[1];
            return mi355x_mul_mat(w->type, w->data, w->ne[0], w->ne[1], w->nb[1], (const float *)x->data, x->ne[1],
                                  x->nb[1], (float *)t->data, t->nb[1], b->workspace, b->workspace_size, st);
        }
        case MI355X_OP_GET_ROWS:
            return mi355x_get_rows(t->src[0]->type, t->src[0]->data, t->src[0]->ne[0], t->src[0]->nb[1],
                                   t->src[0]->ne[1], (const int32_t *)t->src[1]->data, t->src[1]->ne[0],
                                   (float *)t->data, st);
        case MI355X_OP_RMS_NORM:
            if (l.norm_w)
                return mi355x_rms_norm((const float *)t->src[0]->data, l.norm_w, l.norm_y, t->ne[0], nelem(t) / t->ne[0],
                                       f_of(t->op_params[0]), st);
            return mi355x_rms_norm((const float *)t->src[0]->data, nullptr, (float *)t->data, t->ne[0],
                                   nelem(t) / t->ne[0], f_of(t->op_params[0]), st);
        case MI355X_OP_MUL:
        case MI355X_OP_ADD:  // src1 of one row is repeated over src0's rows (ggml broadcast)
            if (!kq::device_ok()) return MI355X_E_NODEVICE;
            return kq::launch_binary(t->op == MI355X_OP_ADD ? 0 : 1, (const float *)t->src[0]->data,
                                 (const float *)t->src[1]->data, (float *)t->data, nelem(t), st, nelem(t->src[1]));
        case MI355X_OP_SWIGLU:
            return mi355x_swiglu((const float *)t->src[0]->data, (const float *)t->src[1]->data, (float *)t->data,
                                 nelem(t), st);
        case MI355X_OP_ROPE:
            return mi355x_rope((const float *)t->src[0]->data, (float *)t->data, (int)t->ne[0], t->op_params[0],
                               (int)(nelem(t) / t->ne[0]), (const int32_t *)t->src[1]->data,
                               (const float *)t->src[2]->data, (int)t->src[2]->ne[1], st);
        case MI355X_OP_ALL_GATHER: {
            if (!b->comm && b->loop_world > 0) {  // emulated rank: own slice into place, the rest untouched
                if (nelem(t) != nelem(t->src[0]) * b->loop_world) return MI355X_E_COMM;
                if (b->loop_nocopy) return 0;  // (timing of a rank's compute alone: tools/split_budget.py)
                const size_t n = (size_t)nelem(t->src[0]) * 4;
                const hipError_t e = hipMemcpyAsync((char *)t->data + (size_t)b->loop_rank * n, t->src[0]->data, n,
                                                    hipMemcpyDeviceToDevice, st);
                return e == hipSuccess ? 0 : (int)e;
            }
            if (!b->comm || nelem(t) != nelem(t->src[0]) * b->world) return MI355X_E_COMM;
            const ncclResult_t r = rccl().all_gather(t->src[0]->data, t->data, (size_t)nelem(t->src[0]), ncclFloat32,
                                                     b->comm, st);
            if (r != ncclSuccess) {
                fprintf(stderr, "ggml_mi355x: ncclAllGather: %s\n", rccl().error_string(r));
                return MI355X_E_COMM;
            }
            return 0;
        }
        case MI355X_OP_ALL_REDUCE: {
            if (!b->comm && b->loop_world > 0) return 0;  // emulated rank: the caller's reduced vector stays
            if (!b->comm || nelem(t) != nelem(t->src[0])) return MI355X_E_COMM;
            const ncclResult_t r = rccl().all_reduce(t->src[0]->data, t->data, (size_t)nelem(t), ncclFloat32, ncclSum,
                                                     b->comm, st);
            if (r != ncclSuccess) {
                fprintf(stderr, "ggml_mi355x: ncclAllReduce: %s\n", rccl().error_string(r));
                return MI355X_E_COMM;
            }
            return 0;
        }
        case MI355X_OP_ATTN_DECODE: {
            mi355x_attn_desc a;
            attn_desc_of(t, a);
            const int64_t n_tok = t->src[0]->ne[1];
            if (n_tok > 1) {  // a prompt batch: all cells first, then every query (causal)
                a.rope_row = 0;
                return mi355x_attn_prompt(&a, (int)n_tok, st);
            }
            a.rope_row = t->src[6]->ne[1] == 1 ? 1 : 0;  // the position's row, staged with pos
            return mi355x_attn_decode(&a, st);
        }
        default:
            return MI355X_E_UNSUPPORTED;
    }
}

// A prompt ATTN_DECODE (>= 16 tokens, contiguous rows) whose output is the activation of the
// batched MUL_MAT the next launch starts with, on the group kernel that can write its Q8L rows.
bool attn_feeds_batched_mm(const mi355x_backend *b, const mi355x_tensor *t, const Launch &next,
                           mi355x_tensor *const *nodes) {
    if (t->src[0]->ne[1] < 16 || t->nb[1] != (size_t)t->ne[0] * 4) return false;
    if (next.kind != 0 && next.kind != 3 && next.kind != 4) return false;
    const mi355x_tensor *m = nodes[next.first];
    if (m->op == MI355X_OP_MUL_MAT && !mm_exact(m)) return false;  // kq_mmf reads an f16 image, not Q8L
    if (m->op != MI355X_OP_MUL_MAT || m->src[1] != t || m->src[0]->ne[0] != t->ne[0]) return false;
    if (next.kind == 0 && next.count != 1) return false;
    if (!batched_mm_shares(b, m)) return false;
    mi355x_attn_desc d;
    attn_desc_of(t, d);
    d.rope_row = 0;
    kq::AttnArgs a;
    return kq::attn_args_from(&d, a) == 0 && kq::attn_prompt_q8_ok(a);
}

// The kind-4 launch `l` holds the k and v MUL_MATs that the prompt ATTN_DECODE of `next`
// reads (src[1], src[2]): its KV-cache cells can be stored by the GEMM's epilogue.
bool kv_epilogue(mi355x_tensor *const *nodes, const Launch &l, const Launch &next, kq::MmqKv &kv) {
    const mi355x_tensor *t = nodes[next.first];
    if (next.kind != 0 || t->op != MI355X_OP_ATTN_DECODE || t->src[0]->ne[1] < 2) return false;
    const int hd = t->op_params[2], n_head_kv = t->op_params[1];
    if ((hd != 64 && hd != 128) || n_head_kv <= 0) return false;
    const mi355x_tensor *kc = t->src[4], *vc = t->src[5];
    if (((uintptr_t)kc->data & 15u) || ((uintptr_t)vc->data & 15u)) return false;
    memset(&kv, 0, sizeof(kv));
    int found = 0;
    for (int k = 0; k < l.count; ++k) {
        const mi355x_tensor *u = nodes[l.first + k];
        const int role = u == t->src[1] ? 1 : u == t->src[2] ? 2 : 0;
        if (!role) continue;
        if (u->ne[0] != (int64_t)n_head_kv * hd || u->ne[1] != t->src[0]->ne[1]) return false;
        kv.kind[k] = role;
        found |= role;
    }
    if (found != 3) return false;
    kv.pos = (const int32_t *)t->src[3]->data;
    kv.rope = (const float *)t->src[6]->data;
    kv.k_cache = (uint16_t *)kc->data;
    kv.v_cache = (uint16_t *)vc->data;
    kv.n_ctx = (int)kc->ne[1];
    kv.hd = hd;
    return true;
}

int enqueue(mi355x_backend *b, mi355x_tensor *const *nodes, const std::vector<Launch> &launches) {
    Q8State q8;
    const mi355x_tensor *kv_done = nullptr;  // prompt ATTN whose KV cells a GEMM epilogue stored
    if (!kq::device_ok()) return MI355X_E_NODEVICE;
    for (size_t li = 0; li < launches.size(); ++li) {
        const Launch &l = launches[li];
        const mi355x_tensor *t = nodes[l.first];
        int rc;
        const bool q8_fuse = l.kind == 0 && t->op == MI355X_OP_ATTN_DECODE && li + 1 < launches.size() &&
                             attn_feeds_batched_mm(b, t, launches[li + 1], nodes);
        if (q8_fuse || (l.kind == 0 && t == kv_done)) {
            // prompt attention: its KV cells already stored by the k/v GEMM's epilogue
            // (kv_done), and/or its output only read by the next launch's GEMM (the o-proj),
            // for which the group kernel also writes the Q8L blocks (no kq_quantize_q8L)
            mi355x_attn_desc d;
            attn_desc_of(t, d);
            d.rope_row = 0;
            kq::AttnArgs a;
            rc = kq::attn_args_from(&d, a);
            if (rc) return rc;
            a.no_store = t == kv_done;
            kv_done = nullptr;
            if (q8_fuse) a.q8_out = (uint8_t *)b->workspace;
            rc = kq::launch_attn_prompt(a, (int)t->src[0]->ne[1], b->stream);
            if (rc) return rc;
            q8 = Q8State();
            if (q8_fuse) {
                q8.src = t->data;
                q8.k = t->ne[0];
                q8.m = t->ne[1];
                q8.nb = t->nb[1];
            }
            continue;
        }
        if (l.kind == 2) {  // prefill prologue: the activation's Q8L blocks for the MUL_MATs after it
            const mi355x_tensor *m = l.q8_of;
            const int64_t K = m->ne[0], M = m->ne[1];
            rc = l.pro == MI355X_PRO_RMS_NORM
                     ? kq::launch_rms_norm_q8L(l.x, l.x2, b->workspace, K, M, l.eps, b->stream)
                     : kq::launch_swiglu_q8L(l.x, l.x2, b->workspace, K, M, b->stream);
            if (rc) return rc;
            q8 = Q8State();  // int8 Q8L blocks now (a preceding f16 GEMM may have left f16 = true)
            q8.src = m->data;
            q8.k = K;
            q8.m = M;
            q8.nb = m->nb[1];
            continue;
        }
        if (l.kind == 6) {  // a decode layer: one persistent launch
            kq::LayerArgs la = l.la;
            const int blk = find_ly_block(b, ly_block_key(l));
            if (!b->ly_sync || blk < 0 || blk >= b->ly_blocks) return MI355X_E_WORKSPACE;
            const mi355x_backend::LyTab *tb = find_ly_tab(b, ly_tab_key(la));
            if (!tb) return MI355X_E_WORKSPACE;
            la.tab = (const uint8_t *)tb->dev;
            la.tab_stride = tb->stride;
            la.sync = b->ly_sync + (size_t)blk * kq::LAYER_SYNC_U32;
            la.err = (int *)(b->ly_sync + (size_t)b->ly_blocks * kq::LAYER_SYNC_U32);
            rc = kq::launch_layer(la, b->stream);
            if (rc) return rc;
            q8 = Q8State();
            continue;
        }
        if (l.kind == 5) {  // decode attention + o-proj (+ residual): one launch
            const mi355x_tensor *mm = nodes[l.first + 1];
            mi355x_attn_desc d;
            attn_desc_of(t, d);
            d.rope_row = t->src[6]->ne[1] == 1 ? 1 : 0;  // the position's row, staged with pos
            kq::AttnArgs a;
            rc = kq::attn_args_from(&d, a);
            if (rc) return rc;
            const mi355x_tensor *w = mm->src[0];
            rc = kq::launch_attn_oproj(a, w->type, w->data, w->ne[1], w->nb[1], l.res[0], l.y[0], (uint8_t *)b->fx,
                                       b->fx_size, b->stream);
            if (rc) return rc;
            q8 = Q8State();
            continue;
        }
        bool f16_run = l.kind == 4 && kq::mmf_on();
        for (int k = 0; f16_run && k < l.count; ++k) {  // every matrix where the f16 kernel is the faster one
            const mi355x_tensor *u = nodes[l.first + k]->src[0];
            f16_run = kq::mmf_applies(u->type, u->data, u->ne[1], u->nb[1], nodes[l.first + k]->src[1]->ne[1], u->ne[0]);
        }
        if (f16_run) {  // the same on the f16 GEMM: the image once, one launch
            const mi355x_tensor *x = t->src[1];
            const int64_t K = t->src[0]->ne[0], M = x->ne[1];
            if (!(q8.src == x->data && q8.k == K && q8.m == M && q8.nb == x->nb[1] && q8.f16)) {
                q8 = Q8State();
                rc = kq::launch_f16img((const float *)x->data, (int64_t)(x->nb[1] / 4), (uint8_t *)b->workspace, K, M,
                                       b->stream);
                if (rc) return rc;
                q8.src = x->data, q8.k = K, q8.m = M, q8.nb = x->nb[1], q8.f16 = true;
            }
            const void *w[4];
            int64_t N[4], ycs[4];
            size_t rs[4];
            float *y[4];
            for (int k = 0; k < l.count; ++k) {
                const mi355x_tensor *u = nodes[l.first + k];
                w[k] = u->src[0]->data;
                N[k] = u->src[0]->ne[1];
                rs[k] = u->src[0]->nb[1];
                y[k] = (float *)u->data;
                ycs[k] = (int64_t)(u->nb[1] / 4);
            }
            rc = kq::launch_mmf_multi(t->src[0]->type, l.count, w, N, rs, y, ycs, K, (uint8_t *)b->workspace,
                                      b->workspace_size, M, b->stream);
            if (rc) return rc;
            const uintptr_t s0 = (uintptr_t)q8.src, s1 = s0 + q8.nb * (size_t)q8.m;
            for (int k = 0; k < l.count; ++k) {  // an output over the imaged activation invalidates it
                const uintptr_t o0 = (uintptr_t)y[k], o1 = o0 + (size_t)ycs[k] * 4 * (size_t)M;
                if (o0 < s1 && s0 < o1) q8 = Q8State();
            }
            continue;
        }
        if (l.kind == 4) {  // several batched MUL_MATs on one activation: one tile-GEMM launch
            const mi355x_tensor *x = t->src[1];
            const int64_t K = t->src[0]->ne[0], M = x->ne[1];
            if (!(q8.src == x->data && q8.k == K && q8.m == M && q8.nb == x->nb[1] && !q8.f16)) {
                q8 = Q8State();
                rc = kq::launch_quantize_q8L((const float *)x->data, (int64_t)(x->nb[1] / 4), b->workspace, K, M,
                                             b->stream, true);
                if (rc) return rc;
                q8.src = x->data;
                q8.k = K;
                q8.m = M;
                q8.nb = x->nb[1];
            }
            const void *w[4];
            int types[4];
            int64_t N[4], ycs[4];
            size_t rs[4];
            float *y[4];
            for (int k = 0; k < l.count; ++k) {
                const mi355x_tensor *u = nodes[l.first + k];
                w[k] = u->src[0]->data;
                types[k] = u->src[0]->type;
                N[k] = u->src[0]->ne[1];
                rs[k] = u->src[0]->nb[1];
                y[k] = (float *)u->data;
                ycs[k] = (int64_t)(u->nb[1] / 4);
            }
            // the prompt attention right after, reading k and v of this group: its KV cells
            // stored by this launch's epilogue (kq_kv_store's arithmetic), one launch fewer
            kq::MmqKv kv;
            const bool kv_fuse = li + 1 < launches.size() && kv_epilogue(nodes, l, launches[li + 1], kv);
            if (kv_fuse) {  // k and v first: their row tiles (and the cache stores) start first
                int order[4], no = 0;
                for (int k = 0; k < l.count; ++k)
                    if (kv.kind[k]) order[no++] = k;
                for (int k = 0; k < l.count; ++k)
                    if (!kv.kind[k]) order[no++] = k;
                const void *w2[4];
                int t2[4], kk2[4];
                int64_t N2[4], ycs2[4];
                size_t rs2[4];
                float *y2[4];
                for (int k = 0; k < l.count; ++k) {
                    const int o = order[k];
                    w2[k] = w[o], t2[k] = types[o], kk2[k] = kv.kind[o], N2[k] = N[o], ycs2[k] = ycs[o];
                    rs2[k] = rs[o], y2[k] = y[o];
                }
                for (int k = 0; k < l.count; ++k) {
                    w[k] = w2[k], types[k] = t2[k], kv.kind[k] = kk2[k], N[k] = N2[k], ycs[k] = ycs2[k];
                    rs[k] = rs2[k], y[k] = y2[k];
                }
            }
            rc = kq::launch_mmq_multi(types, l.count, w, N, rs, y, ycs, K, (const uint8_t *)b->workspace, M,
                                      b->stream, kv_fuse ? &kv : nullptr);
            if (!rc && kv_fuse) kv_done = nodes[launches[li + 1].first];
            if (rc) return rc;
            const uintptr_t s0 = (uintptr_t)q8.src, s1 = s0 + q8.nb * (size_t)q8.m;
            for (int k = 0; k < l.count; ++k) {  // an output over the quantized activation invalidates it
                const uintptr_t o0 = (uintptr_t)y[k], o1 = o0 + (size_t)ycs[k] * 4 * (size_t)M;
                if (o0 < s1 && s0 < o1) q8 = Q8State();
            }
            continue;
        }
        if (l.kind == 3) {  // batched MUL_MAT with the residual ADD as its epilogue
            const mi355x_tensor *ad = nodes[l.first + 1];
            const mi355x_tensor *other = ad->src[0] == t ? ad->src[1] : ad->src[0];
            rc = enqueue_batched_mm(b, t, q8, l.y[0], (int64_t)(ad->nb[1] / 4), l.res[0], (int64_t)(other->nb[1] / 4));
            if (rc) return rc;
            continue;
        }
        if (l.kind != 1 && l.count == 1 && batched_mm_shares(b, t)) {
            rc = enqueue_batched_mm(b, t, q8);
            if (rc) return rc;
            continue;
        }
        q8 = Q8State();  // any other launch may overwrite the workspace or the activation
        if (l.kind == 1) {
            const mi355x_tensor *w = t->src[0];
            mi355x_gemv_desc d[MI355X_MAX_FUSED];
            mi355x_gemv_ext ext;
            memset(&ext, 0, sizeof(ext));
            ext.prologue = l.pro;
            ext.x2 = l.x2;
            ext.eps = l.eps;
            for (int k = 0; k < l.count; ++k) {
                const mi355x_tensor *n = nodes[l.first + k];
                d[k].type = n->src[0]->type;
                d[k].w = n->src[0]->data;
                d[k].n_rows = n->src[0]->ne[1];
                d[k].row_stride = n->src[0]->nb[1];
                d[k].y = l.y[k];
                ext.residual[k] = l.res[k];
            }
            ext.epilogue = l.epi_y ? MI355X_EPI_SWIGLU : MI355X_EPI_NONE;
            ext.epi_y = l.epi_y;
            rc = mi355x_gemv_fused_ext(d, l.count, l.x, w->ne[0], &ext, b->workspace, b->workspace_size, b->stream);
        } else {
            rc = enqueue_node(b, l, t);
        }
        if (rc) return rc;
    }
    return 0;
}

std::vector<uint64_t> graph_key_of(mi355x_tensor *const *nodes, int n_nodes) {
    std::vector<uint64_t> key;
    key.reserve((size_t)n_nodes * 16 + 2);
    // the plan captured under this key also depends on the process-wide kernel selectors
    // (mmq_impl decides kind-4 batching and the KV-store epilogue, attn_prompt_impl the
    // attention's Q8L output, ...): a changed selector must not replay the old graph
    key.push_back(kq::api_selector_key());
    key.push_back(kq::ops_selector_key());
    for (int i = 0; i < n_nodes; ++i) {
        const mi355x_tensor *t = nodes[i];
        key.push_back((uint64_t)(uintptr_t)t->data);
        key.push_back((uint64_t)t->op);
        key.push_back((uint64_t)t->flags);
        for (int d = 0; d < 4; ++d) key.push_back((uint64_t)t->ne[d]);
        for (int d = 0; d < 8; ++d) key.push_back((uint64_t)(uint32_t)t->op_params[d]);
        for (int s = 0; s < MI355X_MAX_SRC; ++s) {
            const mi355x_tensor *u = t->src[s];
            if (!u) { key.push_back(0); continue; }
            key.push_back((uint64_t)(uintptr_t)u->data);
            key.push_back((uint64_t)u->type);
            for (int d = 0; d < 4; ++d) key.push_back((uint64_t)u->ne[d]);
            for (int d = 0; d < 4; ++d) key.push_back((uint64_t)u->nb[d]);
        }
        for (int d = 0; d < 4; ++d) key.push_back((uint64_t)t->nb[d]);
    }
    return key;
}

}  // namespace

extern "C" {

int mi355x_device_count(void) {
    int ndev = 0, n = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return 0;
    for (int d = 0; d < ndev; ++d) {
        DeviceGuard dg(d);
        n += kq::device_ok() ? 1 : 0;  // gfx950 with the library's code object
    }
    return n;
}

int mi355x_device_ordinal(int i) {
    int ndev = 0;
    if (i < 0 || hipGetDeviceCount(&ndev) != hipSuccess) return -1;
    for (int d = 0; d < ndev; ++d) {
        bool ok;
        {
            DeviceGuard dg(d);
            ok = kq::device_ok() != 0;
        }
        if (ok && i-- == 0) return d;
    }
    return -1;
}

int mi355x_device_memory(int device, size_t *free_bytes, size_t *total_bytes) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return MI355X_E_NODEVICE;
    DeviceGuard dg(device);
    size_t f = 0, t = 0;
    const hipError_t e = hipMemGetInfo(&f, &t);
    if (e != hipSuccess) return (int)e;
    if (free_bytes) *free_bytes = f;
    if (total_bytes) *total_bytes = t;
    return MI355X_OK;
}

mi355x_backend_t mi355x_backend_init(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return nullptr;
    DeviceGuard dg(device);
    if (!kq::device_ok()) return nullptr;
    mi355x_backend *b = new mi355x_backend();
    b->device = device;
    if (hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess) {
        delete b;
        return nullptr;
    }
    b->name = "MI355X" + std::to_string(device);
    return b;
}

void mi355x_backend_free(mi355x_backend_t b) {
    if (!b) return;
    {
    DeviceGuard dg(b->device);
    hipStreamSynchronize(b->stream);
    drop_graph(b);
    if (b->workspace) hipFree(b->workspace);
    if (b->fx) hipFree(b->fx);
    if (b->ly_sync) hipFree(b->ly_sync);
    for (auto &t : b->ly_tabs)
        if (t.dev) hipFree(t.dev);
    if (b->comm) rccl().comm_destroy(b->comm);
    hipStreamDestroy(b->stream);
    }
    delete b;
}

const char *mi355x_backend_name(mi355x_backend_t b) { return b ? b->name.c_str() : "MI355X"; }

void *mi355x_backend_stream(mi355x_backend_t b) { return b ? (void *)b->stream : nullptr; }

void *mi355x_backend_alloc(mi355x_backend_t b, size_t size) {
    if (!b) return nullptr;
    DeviceGuard dg(b->device);
    void *p = nullptr;
    if (hipMalloc(&p, size ? size : 1) != hipSuccess) return nullptr;
    return p;
}

void mi355x_backend_free_buffer(mi355x_backend_t b, void *ptr) {
    if (!b || !ptr) return;
    DeviceGuard dg(b->device);
    hipStreamSynchronize(b->stream);
    drop_graph(b);  // a captured graph may reference the buffer
    hipFree(ptr);
}

int mi355x_backend_memset(mi355x_backend_t b, void *dst, int value, size_t size) {
    if (!b || (!dst && size)) return MI355X_E_INVAL;
    if (!size) return MI355X_OK;
    DeviceGuard dg(b->device);
    const hipError_t e = hipMemsetAsync(dst, value & 0xff, size, b->stream);
    return e == hipSuccess ? MI355X_OK : (int)e;
}

int mi355x_backend_set_tensor(mi355x_backend_t b, void *dst, const void *host_src, size_t size) {
    if (!b || (!dst && size)) return MI355X_E_INVAL;
    DeviceGuard dg(b->device);
    // (hipStreamWriteValue32 per word for tiny inputs was measured 10 us/token slower
    // than this one copy of inp_tokens + inp_pos)
    const hipError_t e = hipMemcpyAsync(dst, host_src, size, hipMemcpyHostToDevice, b->stream);
    return e == hipSuccess ? 0 : (int)e;
}

int mi355x_backend_get_tensor(mi355x_backend_t b, void *host_dst, const void *src, size_t size) {
    if (!b || (!src && size)) return MI355X_E_INVAL;
    DeviceGuard dg(b->device);
    const hipError_t e = hipMemcpyAsync(host_dst, src, size, hipMemcpyDeviceToHost, b->stream);
    return e == hipSuccess ? 0 : (int)e;
}

int mi355x_backend_synchronize(mi355x_backend_t b) {
    if (!b) return MI355X_E_INVAL;
    DeviceGuard dg(b->device);
    const hipError_t e = hipStreamSynchronize(b->stream);
    if (e != hipSuccess) return (int)e;
    // a persistent-layer launch that gave up waiting left invalid outputs: report it here,
    // where every caller that reads results already stops (and re-arm the counters)
    if (b->layer_engine && b->ly_sync) {
        const int le = mi355x_backend_layer_error(b);
        if (le) return le > 0 ? MI355X_E_LAYER : le;
    }
    return 0;
}

// ggml_backend_device_i::supports_op for this device: MUL_MAT of a contiguous-row
// K-quant src0 with an f32 src1, 2-D (no broadcast over ne2/ne3), and the other
// nodes of a llama decode token on contiguous f32 (the op table in the header).
static bool contig_f32(const mi355x_tensor *t) { return t && t->type == MI355X_TYPE_F32 && t->nb[0] == 4 && t->data; }

int mi355x_backend_supports_op(const mi355x_tensor *op) {
    if (!op) return 0;
    switch (op->op) {
        case MI355X_OP_NONE:
            return 1;
        case MI355X_OP_MUL_MAT: {
            const mi355x_tensor *w = op->src[0], *x = op->src[1];
            if (!w || !x) return 0;
            if (!is_kquant(w->type) || x->type != MI355X_TYPE_F32 || op->type != MI355X_TYPE_F32) return 0;
            if (w->ne[0] % MI355X_QK_K || w->ne[0] != x->ne[0]) return 0;
            if (w->ne[2] != 1 || w->ne[3] != 1 || x->ne[2] != 1 || x->ne[3] != 1) return 0;
            if (op->ne[0] != w->ne[1] || op->ne[1] != x->ne[1]) return 0;
            if (x->nb[0] != 4 || op->nb[0] != 4) return 0;  // contiguous rows
            if (w->nb[0] != mi355x_row_size(w->type, MI355X_QK_K)) return 0;
            return 1;
        }
        case MI355X_OP_GET_ROWS: {
            const mi355x_tensor *w = op->src[0], *ids = op->src[1];
            if (!w || !ids || ids->type != MI355X_TYPE_I32 || !ids->data || ids->nb[0] != 4 || !contig_f32(op))
                return 0;
            if (w->type != MI355X_TYPE_F32 && !is_kquant(w->type)) return 0;
            if (op->ne[1] > 1 && op->nb[1] != (size_t)op->ne[0] * 4) return 0;  // dst rows packed (kernel: out + r*k)
            return op->ne[0] == w->ne[0] && op->ne[1] == ids->ne[0] && w->ne[0] % MI355X_QK_K == 0;
        }
        case MI355X_OP_RMS_NORM:
            // the kernel reads x + row*n with 16-B loads: src0 and dst packed rows, 16-B aligned
            return contig_f32(op) && contig_f32(op->src[0]) && op->ne[0] % MI355X_QK_K == 0 &&
                   op->nb[1] == (size_t)op->ne[0] * 4 && op->src[0]->nb[1] == (size_t)op->ne[0] * 4 &&
                   nelem(op->src[0]) == nelem(op) && ((uintptr_t)op->src[0]->data & 15u) == 0;
        case MI355X_OP_MUL:
        case MI355X_OP_ADD:
            // src1 the same shape, or one row repeated over the rows (ggml_mul by the norm weight)
            return contig_f32(op) && contig_f32(op->src[0]) && contig_f32(op->src[1]) && nelem(op->src[0]) == nelem(op) &&
                   (nelem(op->src[1]) == nelem(op) || (nelem(op->src[1]) == op->ne[0] && op->nb[1] == (size_t)op->ne[0] * 4));
        case MI355X_OP_SWIGLU:
            return contig_f32(op) && contig_f32(op->src[0]) && contig_f32(op->src[1]) &&
                   nelem(op->src[0]) == nelem(op) && nelem(op->src[1]) == nelem(op);
        case MI355X_OP_ROPE:
            return contig_f32(op) && contig_f32(op->src[0]) && op->src[1] && op->src[1]->type == MI355X_TYPE_I32 &&
                   contig_f32(op->src[2]) && op->op_params[0] > 0 && op->op_params[0] <= op->ne[0] &&
                   op->src[2]->ne[0] == op->op_params[0];
        case MI355X_OP_ALL_GATHER:
            // a packed f32 slice gathered into a packed f32 vector (world known at compute time)
            return contig_f32(op) && contig_f32(op->src[0]) && op->ne[1] == 1 && op->src[0]->ne[1] == 1 &&
                   op->src[0]->ne[0] > 0 && op->ne[0] % op->src[0]->ne[0] == 0;
        case MI355X_OP_ALL_REDUCE:
            // a packed f32 partial summed over the ranks into a packed f32 vector of the same length
            return contig_f32(op) && contig_f32(op->src[0]) && nelem(op) == nelem(op->src[0]) && nelem(op) > 0;
        case MI355X_OP_ATTN_DECODE: {
            for (int s = 0; s < 7; ++s)
                if (!op->src[s] || !op->src[s]->data) return 0;
            const int nh = op->op_params[0], nkv = op->op_params[1], hd = op->op_params[2];
            if ((hd != 64 && hd != 128) || nkv <= 0 || nh % nkv) return 0;
            if (op->src[4]->type != MI355X_TYPE_F16 || op->src[5]->type != MI355X_TYPE_F16) return 0;
            if (op->src[4]->ne[0] != (int64_t)nkv * hd || op->src[3]->type != MI355X_TYPE_I32) return 0;
            if (op->src[5]->ne[0] != op->src[4]->ne[1] || op->src[5]->ne[1] != op->src[4]->ne[0]) return 0;
            // caches exactly [n_ctx][kvw] and [kvw][n_ctx] f16, 16-B aligned (the kernel's addressing)
            if (op->src[4]->nb[0] != 2 || op->src[4]->nb[1] != (size_t)op->src[4]->ne[0] * 2) return 0;
            if (op->src[5]->nb[0] != 2 || op->src[5]->nb[1] != (size_t)op->src[5]->ne[0] * 2) return 0;
            if (((uintptr_t)op->src[4]->data & 15u) || ((uintptr_t)op->src[5]->data & 15u)) return 0;
            const int64_t n_ctx = op->src[4]->ne[1];
            if (n_ctx < 32 || n_ctx % 32 || n_ctx > 8192) return 0;
            for (int s = 0; s < 3; ++s)
                if (!contig_f32(op->src[s])) return 0;
            // T tokens (T > 1: a prompt batch, rows packed): q [nh*hd, T], k, v [kvw, T], pos [T]
            const int64_t T = op->src[0]->ne[1];
            if (T < 1 || T > 0x7fffffff || op->src[0]->ne[0] != (int64_t)nh * hd) return 0;
            if (nelem(op->src[0]) != (int64_t)nh * hd * T || nelem(op->src[1]) != (int64_t)nkv * hd * T ||
                nelem(op->src[2]) != (int64_t)nkv * hd * T || op->src[3]->ne[0] != T)
                return 0;
            if (T > 1 && (op->src[0]->nb[1] != (size_t)nh * hd * 4 || op->src[1]->nb[1] != (size_t)nkv * hd * 4 ||
                          op->src[2]->nb[1] != (size_t)nkv * hd * 4 || op->src[6]->ne[1] < n_ctx))
                return 0;  // packed rows; the whole rope table (one position per token)
            if (op->src[6]->ne[1] != 1 && op->src[6]->ne[1] < op->src[4]->ne[1]) return 0;  // row or table
            if (op->src[6]->ne[0] != hd) return 0;
            return contig_f32(op) && op->ne[0] == (int64_t)nh * hd && op->ne[1] == T &&
                   (T == 1 || op->nb[1] == (size_t)nh * hd * 4);
        }
        default:
            return 0;
    }
}

size_t mi355x_comm_id_size(void) { return sizeof(ncclUniqueId); }

int mi355x_comm_get_unique_id(void *id_out) {
    if (!id_out) return MI355X_E_INVAL;
    Rccl &r = rccl();
    if (!r.ok) return MI355X_E_COMM;
    ncclUniqueId id;
    const ncclResult_t e = r.get_unique_id(&id);
    if (e != ncclSuccess) {
        fprintf(stderr, "ggml_mi355x: ncclGetUniqueId: %s\n", r.error_string(e));
        return MI355X_E_COMM;
    }
    memcpy(id_out, &id, sizeof(id));
    return MI355X_OK;
}

int mi355x_backend_set_comm(mi355x_backend_t b, int rank, int world, const void *unique_id) {
    if (!b || world < 1 || rank < 0 || rank >= world || !unique_id) return MI355X_E_INVAL;
    Rccl &r = rccl();
    if (!r.ok) return MI355X_E_COMM;
    DeviceGuard dg(b->device);
    hipStreamSynchronize(b->stream);
    drop_graph(b);  // a captured graph holds the old communicator's collectives
    if (b->comm) {
        r.comm_destroy(b->comm);
        b->comm = nullptr;
        b->world = 0;
    }
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    ncclComm_t c = nullptr;
    const ncclResult_t e = r.comm_init_rank(&c, world, id, rank);
    if (e != ncclSuccess) {
        fprintf(stderr, "ggml_mi355x: ncclCommInitRank(rank %d of %d): %s\n", rank, world, r.error_string(e));
        return MI355X_E_COMM;
    }
    b->comm = c;
    b->rank = rank;
    b->world = world;
    return MI355X_OK;
}

int mi355x_backend_comm_world(mi355x_backend_t b) {
    return b && b->comm ? b->world : (b && b->loop_world ? b->loop_world : 0);
}

int mi355x_backend_set_comm_loopback(mi355x_backend_t b, int rank, int world) {
    if (!b || world < 0 || (world > 0 && (rank < 0 || rank >= world))) return MI355X_E_INVAL;
    DeviceGuard dg(b->device);
    hipStreamSynchronize(b->stream);
    drop_graph(b);
    b->loop_rank = world > 0 ? rank : -1;
    b->loop_world = world;
    // timing only: emulated ALL_GATHERs skip their own-slice copy, so a token's time is the
    // rank's compute alone (the gathered vectors are then stale: never for parity runs)
    b->loop_nocopy = kq::knob(kq::KNOB_LOOPBACK_NOCOPY) != 0;  // mi355x_debug_knob("LOOPBACK_NOCOPY")
    return MI355X_OK;
}

int mi355x_backend_set_attn_oproj(mi355x_backend_t b, int enable) {
    if (!b) return MI355X_E_INVAL;
    DeviceGuard dg(b->device);
    const int prev = b->attn_oproj ? 1 : 0;
    if ((enable != 0) != b->attn_oproj) {
        hipStreamSynchronize(b->stream);
        drop_graph(b);
        b->attn_oproj = enable != 0;
    }
    return prev;
}

int mi355x_backend_set_layer_engine(mi355x_backend_t b, int enable) {
    if (!b) return MI355X_E_INVAL;
    DeviceGuard dg(b->device);
    const int prev = b->layer_engine ? 1 : 0;
    if ((enable != 0) != b->layer_engine) {
        hipStreamSynchronize(b->stream);
        drop_graph(b);
        b->layer_engine = enable != 0;
    }
    return prev;
}

int mi355x_backend_layer_error(mi355x_backend_t b) {
    if (!b) return MI355X_E_INVAL;
    if (!b->ly_sync) return 0;
    DeviceGuard dg(b->device);
    if (hipStreamSynchronize(b->stream) != hipSuccess) return MI355X_E_NODEVICE;
    int err = 0;
    const size_t words = (size_t)b->ly_blocks * kq::LAYER_SYNC_U32 + 64;
    if (hipMemcpy(&err, b->ly_sync + (size_t)b->ly_blocks * kq::LAYER_SYNC_U32, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return MI355X_E_NODEVICE;
    if (err) {  // the counters of an abandoned launch are out of step: start every block again
        if (hipMemsetAsync(b->ly_sync, 0, words * 4, b->stream) != hipSuccess ||
            hipStreamSynchronize(b->stream) != hipSuccess)
            return MI355X_E_NODEVICE;
    }
    return err ? 1 : 0;
}

int mi355x_backend_set_fusion(mi355x_backend_t b, int enable) {
    if (!b) return MI355X_E_INVAL;
    DeviceGuard dg(b->device);
    const int prev = b->fuse ? 1 : 0;
    if ((enable != 0) != b->fuse) {
        hipStreamSynchronize(b->stream);
        drop_graph(b);
        b->fuse = enable != 0;
    }
    return prev;
}

int mi355x_backend_graph_compute(mi355x_backend_t b, mi355x_tensor *const *nodes, int n_nodes, int use_graph) {
    if (!b || (n_nodes > 0 && !nodes) || n_nodes < 0) return MI355X_E_INVAL;
    DeviceGuard dg(b->device);
    // replay fast path: the node list of the captured graph (every decode step after
    // the first) was validated, planned and captured under this key already
    if (use_graph && !b->graphs.empty()) {
        const std::vector<uint64_t> key = graph_key_of(nodes, n_nodes);
        if (mi355x_backend::Captured *c = find_graph(b, key)) {
            const hipError_t e = hipGraphLaunch(c->exec, b->stream);
            return e == hipSuccess ? 0 : (int)e;
        }
    }
    size_t ws = 0;
    for (int i = 0; i < n_nodes; ++i) {
        if (!mi355x_backend_supports_op(nodes[i])) return MI355X_E_UNSUPPORTED;
        if (nodes[i]->op == MI355X_OP_MUL_MAT) {
            const mi355x_tensor *w = nodes[i]->src[0];
            size_t need = mi355x_mul_mat_workspace_size(w->type, w->ne[0], w->ne[1], nodes[i]->src[1]->ne[1]);
            const size_t nf = mi355x_gemv_ext_workspace_size(w->ne[0]);
            need = need > nf ? need : nf;
            if (nodes[i]->src[1]->ne[1] == 1 && ((uintptr_t)nodes[i]->src[1]->data & 15u))
                need = need > (size_t)(w->ne[0] / 256) * kq::Q8L_STRIDE ? need : (size_t)(w->ne[0] / 256) * kq::Q8L_STRIDE;
            ws = need > ws ? need : ws;
        }
    }
    if (ws > b->workspace_size) {  // grow outside any capture
        hipStreamSynchronize(b->stream);
        drop_graph(b);
        if (b->workspace) hipFree(b->workspace);
        b->workspace = nullptr;
        b->workspace_size = 0;
        if (hipMalloc(&b->workspace, ws) != hipSuccess) return MI355X_E_WORKSPACE;
        b->workspace_size = ws;
    }
    const std::vector<Launch> launches = plan_launches(b, nodes, n_nodes, b->fuse);
    {  // the fused attention + o-proj launches' buffer: sized and zeroed outside any capture
        size_t need = 0;
        int nsb = 0;
        bool mixed = false;
        for (const Launch &l : launches) {
            if (l.kind != 5) continue;
            const mi355x_tensor *t = nodes[l.first], *w = nodes[l.first + 1]->src[0];
            int k = 0;
            const size_t sz = kq::attn_oproj_buffer(t->op_params[2], t->op_params[0], t->op_params[1],
                                                    (int)t->src[4]->ne[1], w->type, w->ne[0], w->ne[1], &k);
            need = sz > need ? sz : need;
            mixed |= nsb && k != nsb;
            nsb = k;
        }
        if (mixed) return MI355X_E_UNSUPPORTED;  // (never built by plan_launches' callers: one o-proj shape per graph)
        if (need && (need > b->fx_size || nsb != b->fx_nsb)) {
            hipStreamSynchronize(b->stream);
            drop_graph(b);
            if (need > b->fx_size) {
                if (b->fx) hipFree(b->fx);
                b->fx = nullptr;
                b->fx_size = 0;
                if (hipMalloc(&b->fx, need) != hipSuccess) return MI355X_E_WORKSPACE;
                b->fx_size = need;
            }
            // on the backend stream (non-blocking: a legacy-stream memset is not ordered
            // before its next launch), then waited for
            if (hipMemsetAsync(b->fx, 0, kq::kAttnOprojCounterBytes, b->stream) != hipSuccess ||
                hipStreamSynchronize(b->stream) != hipSuccess)
                return MI355X_E_WORKSPACE;
            b->fx_nsb = nsb;
        }
    }
    {  // the persistent layers' counter blocks: one per kind-6 launch, zeroed outside any capture
       // whenever they are (re)allocated or their producer counts change
        // A launch's counters are monotonic over its launches with ITS producer counts, so a
        // block is keyed by (layer index in the graph, producers per edge and shard): graphs
        // with other counts (another cache size or model on this backend) get blocks of their
        // own instead of inheriting counters stepped by other counts.
        size_t need = b->ly_keys.size();
        std::vector<std::vector<uint32_t>> fresh;
        for (const Launch &l : launches) {
            if (l.kind != 6) continue;
            const std::vector<uint32_t> k = ly_block_key(l);
            if (find_ly_block(b, k) < 0 && std::find(fresh.begin(), fresh.end(), k) == fresh.end())
                fresh.push_back(k);
        }
        need += fresh.size();
        if (!fresh.empty()) {
            hipStreamSynchronize(b->stream);
            if ((int)need > b->ly_blocks) {  // grow (capacity doubles): every counter restarts at 0
                drop_graph(b);
                int cap = b->ly_blocks ? b->ly_blocks : 8;
                while (cap < (int)need) cap *= 2;
                if (b->ly_sync) hipFree(b->ly_sync);
                b->ly_sync = nullptr;
                b->ly_blocks = 0;
                if (hipMalloc(&b->ly_sync, ((size_t)cap * kq::LAYER_SYNC_U32 + 64) * 4) != hipSuccess) {
                    b->ly_keys.clear();
                    return MI355X_E_WORKSPACE;
                }
                b->ly_blocks = cap;
                if (hipMemsetAsync(b->ly_sync, 0, ((size_t)cap * kq::LAYER_SYNC_U32 + 64) * 4, b->stream) !=
                        hipSuccess ||
                    hipStreamSynchronize(b->stream) != hipSuccess)
                    return MI355X_E_WORKSPACE;
            }
            // new blocks are still zero: blocks past ly_keys.size() were zeroed when allocated
            // and never launched on
            for (auto &k : fresh) b->ly_keys.push_back(std::move(k));
        }
        // the step tables: built on the host once per full geometry (weights, shape, ring depth,
        // attention placement, LDS layout) and kept; a table is never rebuilt in place, so a
        // captured graph never reads a table that changed under it
        for (const Launch &l : launches) {
            if (l.kind != 6) continue;
            std::vector<uint64_t> key = ly_tab_key(l.la);
            if (find_ly_tab(b, key)) continue;
            if (b->ly_tabs.size() >= kMaxLyTabs) {  // bound the cache: start over (graphs may read them)
                hipStreamSynchronize(b->stream);
                drop_graph(b);
                for (auto &t : b->ly_tabs)
                    if (t.dev) hipFree(t.dev);
                b->ly_tabs.clear();
            }
            const int64_t stride = kq::layer_table_stride(l.la);
            if (stride <= 0) return MI355X_E_UNSUPPORTED;
            std::vector<uint8_t> host((size_t)(stride * l.la.G));
            kq::layer_table_fill(l.la, host.data(), stride);
            mi355x_backend::LyTab tb;
            if (hipMalloc(&tb.dev, host.size()) != hipSuccess) return MI355X_E_WORKSPACE;
            if (hipMemcpy(tb.dev, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) {
                hipFree(tb.dev);
                return MI355X_E_WORKSPACE;
            }
            tb.stride = stride;
            tb.key.swap(key);
            b->ly_tabs.push_back(std::move(tb));
        }
    }
    for (const Launch &l : launches) {  // long-cache decode attention: its score workspace, outside any capture
        const mi355x_tensor *t = nodes[l.first];
        if (l.kind != 0 || t->op != MI355X_OP_ATTN_DECODE || t->src[0]->ne[1] != 1) continue;
        mi355x_attn_desc d = {};
        attn_desc_of(t, d);
        kq::AttnArgs a = {};
        if (kq::attn_args_from(&d, a) == MI355X_OK && kq::attn_cells_reserve(a, b->stream) != MI355X_OK) return MI355X_E_WORKSPACE;
    }
    if (!use_graph) return enqueue(b, nodes, launches);
    std::vector<uint64_t> key = graph_key_of(nodes, n_nodes);
    mi355x_backend::Captured *c = find_graph(b, key);
    if (!c) {
        if (hipStreamBeginCapture(b->stream, hipStreamCaptureModeThreadLocal) != hipSuccess)
            return MI355X_E_UNSUPPORTED;
        const int rc = enqueue(b, nodes, launches);
        hipGraph_t g = nullptr;
        const hipError_t ec = hipStreamEndCapture(b->stream, &g);
        if (rc || ec != hipSuccess) {
            if (g) hipGraphDestroy(g);
            return rc ? rc : (int)ec;
        }
        hipGraphExec_t ge = nullptr;
        if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) {
            hipGraphDestroy(g);
            return MI355X_E_UNSUPPORTED;
        }
        if (b->graphs.size() == kMaxGraphs) {  // the least recently used goes
            hipStreamSynchronize(b->stream);
            destroy_captured(b->graphs.front());
            b->graphs.erase(b->graphs.begin());
        }
        mi355x_backend::Captured nc;
        nc.key.swap(key);
        nc.graph = g;
        nc.exec = ge;
        b->graphs.push_back(nc);
        c = &b->graphs.back();
    }
    const hipError_t e = hipGraphLaunch(c->exec, b->stream);
    return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"
