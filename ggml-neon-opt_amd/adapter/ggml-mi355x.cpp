// ggml-mi355x.cpp — the ggml-backend registration of the MI355X K-quant backend:
// registry -> device -> buffer type / buffer -> backend, the sibling of the CPU backend
// that the reference's decode runs on (ggml_backend_cpu_graph_compute, ggml-cpu.cpp:186,
// called from ggml_backend_sched_compute_splits, ggml-backend.cpp:1553 / :1753,
// README.md:162-164). Built inside llama.cpp's tree as ggml/src/ggml-mi355x/ (INTEGRATION.md
// §2) against ggml-backend-impl.h [U] and linked with libggml_mi355x.so; here
// tests/test_adapter.py compiles it with -Werror against a restated subset of those
// headers (tests/adapter/ggml/) and drives reg -> device -> backend -> buffer ->
// graph_compute through the real library.
//
// What each slot does:
//  * reg: one device per gfx950 GPU the library runs on (mi355x_device_count);
//    GGML_BACKEND_DL_IMPL / _SCORE_IMPL for a dynamically loaded backend.
//  * device: name / description / memory / props, init_backend (one HIP stream per
//    backend), the device buffer type, supports_op (the ops the lowering takes: K-quant
//    MUL_MAT, GET_ROWS, RMS_NORM, MUL, ADD, GLU(SWIGLU), the non-flash attention block
//    ROPE / SET_ROWS / f16 MUL_MAT / SOFT_MAX / CONT and the views), offload_op (prompt
//    batches, as ggml-cuda does), supports_buft (its own buffer type).
//  * buffer type / buffer: device memory (hipMalloc through the library), GGUF block bytes
//    copied unchanged (no repack), memset / clear, synchronous set / get as ggml expects.
//  * backend: graph_compute = mirror the ggml_cgraph into mi355x_gtensors, check the
//    cells == positions promise from the graph's own inputs (k_idxs, inp_pos, the KQ
//    mask), lower (mi355x_lower_ggml_graph) and run (mi355x_backend_graph_compute with
//    hipGraph replay); async set / get on the backend stream; synchronize.
// A graph the lowering cannot take (flash attention, a mask that is not causal over
// [0, pos], an op outside the list) returns GGML_STATUS_FAILED rather than a wrong result.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "ggml-backend-impl.h"
#include "ggml-mi355x.h"
#include "ggml_mi355x.h"
#include "mi355x_ggml_mirror.hpp"

namespace {

constexpr size_t kAlign = 256;          // tensor alignment of the device buffers
constexpr size_t kTailPad = 4096;       // slack after a buffer: 16-B DMA granules never leave the allocation
constexpr size_t kShadowMax = 1 << 20;  // host copies kept of inputs set through set_tensor

ggml_guid g_guid = {0x6d, 0x69, 0x33, 0x35, 0x35, 0x78, 0x2d, 0x6b, 0x71, 0x75, 0x61, 0x6e, 0x74, 0x2d, 0x67, 0x31};

struct Device;

// ------------------------------------------------------------------ devices
struct Device {
    int index = 0;
    std::string name, description;
    mi355x_backend_t mem = nullptr;  // memory operations of the device's buffers (own stream)
    std::mutex mu;
    // host copies of small inputs written by set_tensor since the last graph_compute
    // (ggml sets every graph input that way before computing): the cells == positions
    // check reads them instead of the device; keyed by device address
    struct Shadow {
        std::vector<uint8_t> bytes;
        uint64_t epoch;
    };
    std::map<uintptr_t, Shadow> shadows;
    uint64_t epoch = 1;
    ggml_backend_buffer_type buft;
    ggml_backend_device dev;
};

mi355x_backend_t device_mem(Device *d) {
    std::lock_guard<std::mutex> lk(d->mu);
    if (!d->mem) d->mem = mi355x_backend_init(d->index);
    return d->mem;
}

void shadow_store(Device *d, const void *dst, const void *src, size_t n) {
    if (n == 0 || n > kShadowMax) return;
    std::lock_guard<std::mutex> lk(d->mu);
    auto &s = d->shadows[(uintptr_t)dst];
    s.bytes.assign((const uint8_t *)src, (const uint8_t *)src + n);
    s.epoch = d->epoch;
}

void shadow_drop(Device *d, uintptr_t lo, uintptr_t hi) {
    std::lock_guard<std::mutex> lk(d->mu);
    for (auto it = d->shadows.lower_bound(lo); it != d->shadows.end() && it->first < hi;) it = d->shadows.erase(it);
}

// ------------------------------------------------------------------ buffers
struct Buffer {
    Device *dev;
    void *base;
    size_t size;
};

void buf_free(ggml_backend_buffer_t b) {
    auto *ctx = (Buffer *)b->context;
    shadow_drop(ctx->dev, (uintptr_t)ctx->base, (uintptr_t)ctx->base + ctx->size);
    mi355x_backend_free_buffer(device_mem(ctx->dev), ctx->base);
    delete ctx;
}

void *buf_base(ggml_backend_buffer_t b) { return ((Buffer *)b->context)->base; }

enum ggml_status buf_init_tensor(ggml_backend_buffer_t, struct ggml_tensor *) { return GGML_STATUS_SUCCESS; }

void buf_memset(ggml_backend_buffer_t b, struct ggml_tensor *t, uint8_t value, size_t off, size_t n) {
    auto *ctx = (Buffer *)b->context;
    char *p = (char *)t->data + off;
    shadow_drop(ctx->dev, (uintptr_t)p, (uintptr_t)p + n);
    mi355x_backend_t m = device_mem(ctx->dev);
    mi355x_backend_memset(m, p, value, n);
    mi355x_backend_synchronize(m);
}

void buf_set(ggml_backend_buffer_t b, struct ggml_tensor *t, const void *data, size_t off, size_t n) {
    auto *ctx = (Buffer *)b->context;
    char *p = (char *)t->data + off;
    mi355x_backend_t m = device_mem(ctx->dev);
    mi355x_backend_set_tensor(m, p, data, n);
    mi355x_backend_synchronize(m);  // ggml_backend_tensor_set is synchronous
    shadow_store(ctx->dev, p, data, n);
}

void buf_get(ggml_backend_buffer_t b, const struct ggml_tensor *t, void *data, size_t off, size_t n) {
    auto *ctx = (Buffer *)b->context;
    mi355x_backend_t m = device_mem(ctx->dev);
    mi355x_backend_get_tensor(m, data, (const char *)t->data + off, n);
    mi355x_backend_synchronize(m);
}

void buf_clear(ggml_backend_buffer_t b, uint8_t value) {
    auto *ctx = (Buffer *)b->context;
    shadow_drop(ctx->dev, (uintptr_t)ctx->base, (uintptr_t)ctx->base + ctx->size);
    mi355x_backend_t m = device_mem(ctx->dev);
    mi355x_backend_memset(m, ctx->base, value, ctx->size);
    mi355x_backend_synchronize(m);
}

const struct ggml_backend_buffer_i kBufferIface = {
    /* .free_buffer   = */ buf_free,
    /* .get_base      = */ buf_base,
    /* .init_tensor   = */ buf_init_tensor,
    /* .memset_tensor = */ buf_memset,
    /* .set_tensor    = */ buf_set,
    /* .get_tensor    = */ buf_get,
    /* .cpy_tensor    = */ nullptr,  // the scheduler copies through the host
    /* .clear         = */ buf_clear,
    /* .reset         = */ nullptr,
};

const char *buft_name(ggml_backend_buffer_type_t buft) { return ((Device *)buft->context)->name.c_str(); }

ggml_backend_buffer_t buft_alloc(ggml_backend_buffer_type_t buft, size_t size) {
    auto *d = (Device *)buft->context;
    mi355x_backend_t m = device_mem(d);
    if (!m) return nullptr;
    void *p = mi355x_backend_alloc(m, size + kTailPad);
    if (!p) return nullptr;
    auto *ctx = new Buffer{d, p, size};
    return ggml_backend_buffer_init(buft, kBufferIface, ctx, size);
}

size_t buft_alignment(ggml_backend_buffer_type_t) { return kAlign; }

bool buft_is_host(ggml_backend_buffer_type_t) { return false; }

// ------------------------------------------------------------------ backend
struct Backend : mi355x_adapter::Context {
    Device *dev = nullptr;
    size_t rope_bytes = 0;
    int rope_dims = 0;
    std::vector<uint8_t> host_in;  // read-back of the inputs when no fresh shadow holds them
};

const char *be_name(ggml_backend_t backend) { return ((Backend *)backend->context)->dev->name.c_str(); }

void be_free(ggml_backend_t backend) {
    auto *ctx = (Backend *)backend->context;
    if (ctx->rope_table) mi355x_backend_free_buffer(ctx->be, ctx->rope_table);
    mi355x_backend_free(ctx->be);
    delete ctx;
    delete backend;
}

void be_set_async(ggml_backend_t backend, struct ggml_tensor *t, const void *data, size_t off, size_t n) {
    auto *ctx = (Backend *)backend->context;
    char *p = (char *)t->data + off;
    mi355x_backend_set_tensor(ctx->be, p, data, n);
    shadow_store(ctx->dev, p, data, n);
}

void be_get_async(ggml_backend_t backend, const struct ggml_tensor *t, void *data, size_t off, size_t n) {
    auto *ctx = (Backend *)backend->context;
    mi355x_backend_get_tensor(ctx->be, data, (const char *)t->data + off, n);
}

// ggml's synchronize returns nothing: like ggml-cuda's CUDA_CHECK, a failed wait aborts
// (a persistent-layer launch that lost co-residency left invalid outputs: MI355X_E_LAYER)
void be_synchronize(ggml_backend_t backend) {
    const int rc = mi355x_backend_synchronize(((Backend *)backend->context)->be);
    if (rc != 0) {
        std::fprintf(stderr, "ggml-mi355x: synchronize failed (%d)%s\n", rc,
                     rc == MI355X_E_LAYER ? ": persistent layer lost co-residency, outputs invalid" : "");
        std::abort();
    }
}

const char *op_name(const ggml_tensor *t) { return ggml_op_name(t->op); }

bool is_op(const ggml_tensor *t, const char *name) { return t && std::strcmp(ggml_op_name(t->op), name) == 0; }

// `n` bytes of input tensor t on the host: the fresh shadow of a set_tensor, or a
// read-back on the backend stream (after the work queued before it).
const uint8_t *read_input(Backend *ctx, const ggml_tensor *t, size_t n, size_t at) {
    Device *d = ctx->dev;
    {
        std::lock_guard<std::mutex> lk(d->mu);
        auto it = d->shadows.find((uintptr_t)t->data);
        if (it != d->shadows.end() && it->second.epoch == d->epoch && it->second.bytes.size() >= n) {
            std::memcpy(ctx->host_in.data() + at, it->second.bytes.data(), n);
            return ctx->host_in.data() + at;
        }
    }
    if (mi355x_backend_get_tensor(ctx->be, ctx->host_in.data() + at, t->data, n) != 0) return nullptr;
    if (mi355x_backend_synchronize(ctx->be) != 0) return nullptr;
    return ctx->host_in.data() + at;
}

// The lowering's cells == positions promise (mi355x_lower_opts.cells_eq_pos), from the
// graph's inputs: the first K-cache store's cell indices equal inp_pos, and the KQ mask
// rows are causal over [0, pos] (mi355x_ggml_mirror.hpp).
bool cells_checked(Backend *ctx, const std::vector<ggml_tensor *> &nodes) {
    const ggml_tensor *k_idxs = nullptr, *pos = nullptr, *mask = nullptr;
    for (const ggml_tensor *t : nodes) {
        if (!k_idxs && is_op(t, "SET_ROWS")) k_idxs = t->src[1];
        if (!pos && is_op(t, "ROPE")) pos = t->src[1];
        if (!mask && is_op(t, "SOFT_MAX")) mask = t->src[1];
    }
    if (!k_idxs || !pos || !mask || !k_idxs->data || !pos->data || !mask->data) return false;
    if (pos->type != GGML_TYPE_I32 || (k_idxs->type != GGML_TYPE_I64 && k_idxs->type != GGML_TYPE_I32)) return false;
    if (mask->type != GGML_TYPE_F32 && mask->type != GGML_TYPE_F16) return false;
    const int64_t T = ggml_nelements(pos);
    if (T <= 0 || ggml_nelements(k_idxs) != T || mask->ne[1] < T) return false;
    const size_t eb = k_idxs->type == GGML_TYPE_I64 ? 8 : 4;
    const size_t mb = (size_t)(T - 1) * mask->nb[1] + (size_t)mask->ne[0] * mask->nb[0];
    ctx->host_in.resize((size_t)T * 4 + (size_t)T * 8 + mb + 64);
    const uint8_t *hp = read_input(ctx, pos, (size_t)T * 4, 0);
    const uint8_t *hk = hp ? read_input(ctx, k_idxs, (size_t)T * eb, (size_t)T * 4) : nullptr;
    const uint8_t *hm = hk ? read_input(ctx, mask, mb, (size_t)T * 12) : nullptr;
    if (!hm) return false;
    std::vector<int64_t> kid((size_t)T);
    std::vector<int32_t> pv((size_t)T);
    std::memcpy(pv.data(), hp, (size_t)T * 4);
    for (int64_t i = 0; i < T; ++i) {
        if (eb == 8) {
            std::memcpy(&kid[(size_t)i], hk + 8 * i, 8);
        } else {
            int32_t v;
            std::memcpy(&v, hk + 4 * i, 4);
            kid[(size_t)i] = v;
        }
    }
    return mi355x_adapter::cells_eq_pos(kid.data(), pv.data(), T) &&
           mi355x_adapter::kq_mask_causal(hm, mask->type == GGML_TYPE_F16 ? 1 : 0, mask->ne[0], mask->nb[1], pv.data(),
                                          T);
}

// The rope table the lowering's ROPE nodes are checked against: created on the backend
// for the graph's (n_dims, freq_base, freq_scale) and at least as many positions as the
// K cache has cells (every SET_ROWS destination's storage), kept while those hold.
bool rope_table_for(Backend *ctx, const std::vector<ggml_tensor *> &nodes) {
    const ggml_tensor *rope = nullptr;
    int64_t cells = 0;
    for (const ggml_tensor *t : nodes) {
        if (!rope && is_op(t, "ROPE")) rope = t;
        if (is_op(t, "SET_ROWS")) {
            const ggml_tensor *root = t;
            while (root->view_src) root = root->view_src;
            for (int d = 0; d < 2; ++d) cells = root->ne[d] > cells ? root->ne[d] : cells;
        }
    }
    if (!rope) return true;  // nothing to rotate: no table needed
    mi355x_adapter::RopeParams p;
    if (!mi355x_adapter::rope_params_of(rope, p)) return false;
    const int n_pos = (int)((cells + 255) / 256 * 256);
    if (ctx->rope_table && ctx->rope_dims == p.n_dims && ctx->freq_base == p.freq_base &&
        ctx->freq_scale == p.freq_scale && ctx->rope_n_pos >= n_pos)
        return true;
    if (ctx->rope_table) mi355x_backend_free_buffer(ctx->be, ctx->rope_table);
    ctx->rope_table = nullptr;
    const size_t bytes = mi355x_rope_table_size(n_pos, p.n_dims);
    void *tab = bytes ? mi355x_backend_alloc(ctx->be, bytes) : nullptr;
    if (!tab) return false;
    if (mi355x_rope_table((float *)tab, n_pos, p.n_dims, p.freq_base, p.freq_scale, mi355x_backend_stream(ctx->be))) {
        mi355x_backend_free_buffer(ctx->be, tab);
        return false;
    }
    ctx->rope_table = tab;
    ctx->rope_bytes = bytes;
    ctx->rope_n_pos = n_pos;
    ctx->rope_dims = p.n_dims;
    ctx->freq_base = p.freq_base;
    ctx->freq_scale = p.freq_scale;
    return true;
}

enum ggml_status be_graph_compute(ggml_backend_t backend, struct ggml_cgraph *cgraph) {
    auto *ctx = (Backend *)backend->context;
    const int n = ggml_graph_n_nodes(cgraph);
    std::vector<ggml_tensor *> nodes((size_t)n);
    for (int i = 0; i < n; ++i) nodes[(size_t)i] = ggml_graph_node(cgraph, i);
    if (!rope_table_for(ctx, nodes)) return GGML_STATUS_FAILED;
    const bool cells_ok = cells_checked(ctx, nodes);
    {
        std::lock_guard<std::mutex> lk(ctx->dev->mu);
        ++ctx->dev->epoch;  // inputs set after this point are fresh for the next graph
    }
    mi355x_adapter::Mirror<ggml_tensor> mir;
    mir.op_name = op_name;
    mir.output_flag = GGML_TENSOR_FLAG_OUTPUT;
    mir.max_src = GGML_MAX_SRC;
    const int rc = mi355x_adapter::graph_compute(*ctx, mir, nodes.data(), n, cells_ok);
    return rc == 0 ? GGML_STATUS_SUCCESS : GGML_STATUS_FAILED;
}

const struct ggml_backend_i kBackendIface = {
    /* .get_name           = */ be_name,
    /* .free               = */ be_free,
    /* .set_tensor_async   = */ be_set_async,
    /* .get_tensor_async   = */ be_get_async,
    /* .cpy_tensor_async   = */ nullptr,
    /* .synchronize        = */ be_synchronize,
    /* .graph_plan_create  = */ nullptr,
    /* .graph_plan_free    = */ nullptr,
    /* .graph_plan_update  = */ nullptr,
    /* .graph_plan_compute = */ nullptr,
    /* .graph_compute      = */ be_graph_compute,
    /* .event_record       = */ nullptr,
    /* .event_wait         = */ nullptr,
    /* .graph_optimize     = */ nullptr,
};

// ------------------------------------------------------------------ device interface
const char *dev_name(ggml_backend_dev_t dev) { return ((Device *)dev->context)->name.c_str(); }
const char *dev_description(ggml_backend_dev_t dev) { return ((Device *)dev->context)->description.c_str(); }

void dev_memory(ggml_backend_dev_t dev, size_t *free, size_t *total) {
    *free = *total = 0;
    mi355x_device_memory(((Device *)dev->context)->index, free, total);
}

enum ggml_backend_dev_type dev_type(ggml_backend_dev_t) { return GGML_BACKEND_DEVICE_TYPE_GPU; }

void dev_props(ggml_backend_dev_t dev, struct ggml_backend_dev_props *props) {
    props->name = dev_name(dev);
    props->description = dev_description(dev);
    props->type = dev_type(dev);
    props->device_id = nullptr;
    dev_memory(dev, &props->memory_free, &props->memory_total);
    props->caps.async = true;
    props->caps.host_buffer = false;
    props->caps.buffer_from_host_ptr = false;
    props->caps.events = false;
}

ggml_backend_t dev_init_backend(ggml_backend_dev_t dev, const char *) {
    auto *d = (Device *)dev->context;
    mi355x_backend_t be = mi355x_backend_init(d->index);
    if (!be) return nullptr;
    auto *ctx = new Backend();
    ctx->be = be;
    ctx->dev = d;
    return new ggml_backend{&g_guid, kBackendIface, dev, ctx};
}

ggml_backend_buffer_type_t dev_buft(ggml_backend_dev_t dev) { return &((Device *)dev->context)->buft; }

bool is_kquant(int type) { return type == GGML_TYPE_Q4_K || type == GGML_TYPE_Q5_K || type == GGML_TYPE_Q6_K; }
bool f32_rows(const ggml_tensor *t) { return t && t->type == GGML_TYPE_F32 && t->nb[0] == 4; }

// mi355x_tensor of a ggml tensor's shape for the library's own supports_op
void shape_of(const ggml_tensor *t, mi355x_tensor &m) {
    std::memset(&m, 0, sizeof(m));
    m.type = (int)t->type;
    for (int d = 0; d < 4; ++d) {
        m.ne[d] = t->ne[d];
        m.nb[d] = t->nb[d];
    }
}

// Through views / reshapes / permutes / transposes to the tensor that owns the bytes, or
// to the op that computed them.
const ggml_tensor *alias_root(const ggml_tensor *t) {
    for (int hop = 0; t && hop < 64; ++hop) {
        if (t->view_src) {
            t = t->view_src;
            continue;
        }
        if ((is_op(t, "RESHAPE") || is_op(t, "PERMUTE") || is_op(t, "TRANSPOSE") || is_op(t, "VIEW")) && t->src[0]) {
            t = t->src[0];
            continue;
        }
        break;
    }
    return t;
}

// The f16 MUL_MATs the lowering takes are the non-flash attention's KQ and KQV only
// (kq_lower.cpp attention()): src0 a view from cell 0 of an f16 KV-cache leaf, src1 the
// rope'd query (KQ) or the soft_max output (KQV). Any other f16 MUL_MAT (an f16 lm_head,
// a tied embedding) stays with the CPU backend: claiming it would fail graph_compute.
bool attn_f16_mul_mat(const ggml_tensor *op) {
    const ggml_tensor *a = op->src[0], *b = op->src[1];
    if (!a || !b || a->type != GGML_TYPE_F16 || b->type != GGML_TYPE_F32) return false;
    if (!a->view_src || a->view_offs != 0) return false;
    const ggml_tensor *cache = alias_root(a);
    if (!cache || !is_op(cache, "NONE") || cache->type != GGML_TYPE_F16) return false;
    const ggml_tensor *rb = alias_root(b);
    return is_op(rb, "ROPE") || is_op(rb, "SOFT_MAX");
}

// What the lowering takes (mi355x_lower_ggml_graph): the scheduler places these nodes
// here; a graph whose attention block is not the non-flash llm_build_llama pattern
// fails in graph_compute (GGML_STATUS_FAILED), it is never computed wrongly.
bool dev_supports_op(ggml_backend_dev_t, const struct ggml_tensor *op) {
    const char *name = ggml_op_name(op->op);
    const int gop = mi355x_adapter::gop_of_name(name);
    if (gop < 0) return false;
    const ggml_tensor *a = op->src[0], *b = op->src[1];
    switch (gop) {
        case MI355X_GOP_NONE:
        case MI355X_GOP_RESHAPE:
        case MI355X_GOP_VIEW:
        case MI355X_GOP_PERMUTE:
        case MI355X_GOP_TRANSPOSE:
            return true;
        case MI355X_GOP_MUL_MAT: {
            if (!a || !b) return false;
            if (a->type == GGML_TYPE_F16) return attn_f16_mul_mat(op);  // KQ / KQV on the f16 cache only
            if (!is_kquant(a->type)) return false;
            mi355x_tensor w, x, y;
            shape_of(a, w);
            shape_of(b, x);
            shape_of(op, y);
            y.op = MI355X_OP_MUL_MAT;
            y.src[0] = &w;
            y.src[1] = &x;
            return mi355x_backend_supports_op(&y) != 0;
        }
        case MI355X_GOP_GET_ROWS:
            return a && b && (a->type == GGML_TYPE_F32 || is_kquant(a->type)) && b->type == GGML_TYPE_I32 &&
                   f32_rows(op) && op->ne[0] == a->ne[0] && a->ne[0] % 256 == 0;
        case MI355X_GOP_RMS_NORM:
            return f32_rows(op) && f32_rows(a) && op->ne[0] % 256 == 0;
        case MI355X_GOP_MUL:
        case MI355X_GOP_ADD:
            return f32_rows(op) && f32_rows(a) && f32_rows(b);
        case MI355X_GOP_GLU:  // SWIGLU with separate gate and up (ggml_swiglu_split)
            return op->op_params[0] == GGML_GLU_OP_SWIGLU && op->op_params[1] == 0 && f32_rows(a) && f32_rows(b) &&
                   f32_rows(op);
        case MI355X_GOP_ROPE:
            return op->op_params[2] == 0 && f32_rows(a) && b && b->type == GGML_TYPE_I32;  // mode NORMAL
        case MI355X_GOP_SET_ROWS:
            return op->type == GGML_TYPE_F16 && f32_rows(a) && b &&
                   (b->type == GGML_TYPE_I64 || b->type == GGML_TYPE_I32);
        case MI355X_GOP_SOFT_MAX: {
            float max_bias;
            std::memcpy(&max_bias, &op->op_params[1], 4);
            return f32_rows(a) && max_bias == 0.0f &&
                   (!b || b->type == GGML_TYPE_F16 || b->type == GGML_TYPE_F32);
        }
        case MI355X_GOP_CONT: {  // only the attention block's last node: CONT(PERMUTE(KQV))
            if (!a || a->type != GGML_TYPE_F32 || op->type != GGML_TYPE_F32 || !is_op(a, "PERMUTE")) return false;
            const ggml_tensor *kqv = alias_root(a);
            return is_op(kqv, "MUL_MAT") && attn_f16_mul_mat(kqv);
        }
        case MI355X_GOP_CPY:  // never lowered (the KV store is SET_ROWS)
        default:
            return false;
    }
}

bool dev_supports_buft(ggml_backend_dev_t dev, ggml_backend_buffer_type_t buft) {
    return buft == &((Device *)dev->context)->buft;
}

// Weights in a host buffer: offload a prompt batch's K-quant MUL_MAT (the weights are
// copied over for it), as ggml-cuda does from batch 32; decode stays where the weights are.
bool dev_offload_op(ggml_backend_dev_t dev, const struct ggml_tensor *op) {
    return is_op(op, "MUL_MAT") && op->src[0] && is_kquant(op->src[0]->type) && op->ne[1] >= 32 &&
           dev_supports_op(dev, op);
}

const struct ggml_backend_device_i kDeviceIface = {
    /* .get_name             = */ dev_name,
    /* .get_description      = */ dev_description,
    /* .get_memory           = */ dev_memory,
    /* .get_type             = */ dev_type,
    /* .get_props            = */ dev_props,
    /* .init_backend         = */ dev_init_backend,
    /* .get_buffer_type      = */ dev_buft,
    /* .get_host_buffer_type = */ nullptr,
    /* .buffer_from_host_ptr = */ nullptr,
    /* .supports_op          = */ dev_supports_op,
    /* .supports_buft        = */ dev_supports_buft,
    /* .offload_op           = */ dev_offload_op,
    /* .event_new            = */ nullptr,
    /* .event_free           = */ nullptr,
    /* .event_synchronize    = */ nullptr,
};

const struct ggml_backend_buffer_type_i kBuftIface = {
    /* .get_name       = */ buft_name,
    /* .alloc_buffer   = */ buft_alloc,
    /* .get_alignment  = */ buft_alignment,
    /* .get_max_size   = */ nullptr,  // SIZE_MAX
    /* .get_alloc_size = */ nullptr,  // ggml_nbytes
    /* .is_host        = */ buft_is_host,
};

// ------------------------------------------------------------------ registry
struct Registry {
    std::vector<Device *> devices;
    ggml_backend_reg reg;
};

const char *reg_name(ggml_backend_reg_t) { return "MI355X"; }
size_t reg_count(ggml_backend_reg_t reg) { return ((Registry *)reg->context)->devices.size(); }
ggml_backend_dev_t reg_device(ggml_backend_reg_t reg, size_t i) {
    auto *r = (Registry *)reg->context;
    return i < r->devices.size() ? &r->devices[i]->dev : nullptr;
}
void *reg_proc(ggml_backend_reg_t, const char *) { return nullptr; }

const struct ggml_backend_reg_i kRegIface = {
    /* .get_name         = */ reg_name,
    /* .get_device_count = */ reg_count,
    /* .get_device       = */ reg_device,
    /* .get_proc_address = */ reg_proc,
};

Registry *registry() {
    static Registry *r = [] {
        auto *reg = new Registry();
        const int n = mi355x_device_count();
        for (int i = 0; i < n; ++i) {
            auto *d = new Device();
            d->index = mi355x_device_ordinal(i);  // the HIP ordinal, not the position in the list
            d->name = "MI355X" + std::to_string(i);
            d->description = "AMD Instinct MI355X (gfx950): K-quant MUL_MAT + llama decode ops, libggml_mi355x";
            d->buft = ggml_backend_buffer_type{kBuftIface, &d->dev, d};
            d->dev = ggml_backend_device{kDeviceIface, &reg->reg, d};
            reg->devices.push_back(d);
        }
        reg->reg = ggml_backend_reg{GGML_BACKEND_API_VERSION, kRegIface, reg};
        return reg;
    }();
    return r;
}

int mi355x_score() { return mi355x_device_count() > 0 ? 10 : 0; }

}  // namespace

ggml_backend_reg_t ggml_backend_mi355x_reg(void) { return &registry()->reg; }

ggml_backend_t ggml_backend_mi355x_init(int device) {
    ggml_backend_reg_t reg = ggml_backend_mi355x_reg();
    ggml_backend_dev_t dev = device >= 0 ? reg_device(reg, (size_t)device) : nullptr;
    return dev ? dev_init_backend(dev, nullptr) : nullptr;
}

bool ggml_backend_is_mi355x(ggml_backend_t backend) {
    return backend && backend->guid && std::memcmp(*backend->guid, g_guid, sizeof(ggml_guid)) == 0;
}

ggml_backend_buffer_type_t ggml_backend_mi355x_buffer_type(int device) {
    ggml_backend_dev_t dev = device >= 0 ? reg_device(ggml_backend_mi355x_reg(), (size_t)device) : nullptr;
    return dev ? dev_buft(dev) : nullptr;
}

int ggml_backend_mi355x_get_device_count(void) { return (int)registry()->devices.size(); }

GGML_BACKEND_DL_IMPL(ggml_backend_mi355x_reg)
GGML_BACKEND_DL_SCORE_IMPL(mi355x_score)
