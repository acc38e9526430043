// mi355x_ggml_mirror.hpp — the ggml-backend adapter's core, header-only and compiled.
//
// A ggml backend built on libggml_mi355x receives the ggml_cgraph that
// ggml_backend_sched_compute_splits hands to iface.graph_compute (ggml-backend.cpp:1553,
// CPU sibling ggml-cpu.cpp:186, README.md:162-163). This header does everything between
// that call and the library: it mirrors each ggml_tensor field for field into an
// mi355x_gtensor (memoised, so views and shared sources stay shared), maps GGML_OP_*
// to the lowering's op numbering by name, checks the cells == positions promise the
// attention lowering needs, lowers the graph (mi355x_lower_ggml_graph) and runs it
// (mi355x_backend_graph_compute, hipGraph replay).
//
// It is a template over the tensor struct: `Tensor` is ggml's `struct ggml_tensor` in the
// real adapter (adapter/ggml-mi355x.cpp, built inside llama.cpp's tree), and the test
// struct of tests/adapter_test.cpp here, which has upstream's field names [U]. So the
// code a maintainer builds is the code tests/test_adapter.py compiles against
// include/ggml_mi355x.h and runs through the lowering (host only, no device).
#pragma once

#include <cstdint>
#include <cstring>
#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

#include "ggml_mi355x.h"

namespace mi355x_adapter {

// ggml op -> the lowering's op numbering, by the op's name (the enums differ between
// ggml versions; ggml_op_name() gives e.g. "MUL_MAT"): -1 = not taken by this backend.
inline int gop_of_name(const char *name) {
    static const struct {
        const char *n;
        int op;
    } table[] = {{"NONE", MI355X_GOP_NONE},       {"GET_ROWS", MI355X_GOP_GET_ROWS}, {"RMS_NORM", MI355X_GOP_RMS_NORM},
                 {"MUL", MI355X_GOP_MUL},         {"ADD", MI355X_GOP_ADD},           {"MUL_MAT", MI355X_GOP_MUL_MAT},
                 {"ROPE", MI355X_GOP_ROPE},       {"SET_ROWS", MI355X_GOP_SET_ROWS}, {"SOFT_MAX", MI355X_GOP_SOFT_MAX},
                 {"GLU", MI355X_GOP_GLU},         {"RESHAPE", MI355X_GOP_RESHAPE},   {"VIEW", MI355X_GOP_VIEW},
                 {"PERMUTE", MI355X_GOP_PERMUTE}, {"TRANSPOSE", MI355X_GOP_TRANSPOSE}, {"CONT", MI355X_GOP_CONT},
                 {"CPY", MI355X_GOP_CPY}};
    for (const auto &e : table)
        if (std::strcmp(e.n, name) == 0) return e.op;
    return -1;
}

// One mirror per ggml tensor, fields copied as they are.
template <typename Tensor>
struct Mirror {
    std::unordered_map<const Tensor *, mi355x_gtensor *> m;
    std::deque<mi355x_gtensor> store;
    const char *(*op_name)(const Tensor *);  // ggml_op_name(t->op) in the real adapter
    int output_flag;                         // GGML_TENSOR_FLAG_OUTPUT
    int max_src;                             // GGML_MAX_SRC

    mi355x_gtensor *of(const Tensor *t) {
        if (!t) return nullptr;
        auto it = m.find(t);
        if (it != m.end()) return it->second;
        mi355x_gtensor &g = store.emplace_back();
        std::memset(&g, 0, sizeof(g));
        m[t] = &g;
        g.type = (int)t->type;
        g.op = gop_of_name(op_name(t));
        for (int i = 0; i < 4; ++i) {
            g.ne[i] = t->ne[i];
            g.nb[i] = t->nb[i];
        }
        std::memcpy(g.op_params, t->op_params, sizeof(g.op_params) < sizeof(t->op_params) ? sizeof(g.op_params)
                                                                                         : sizeof(t->op_params));
        g.flags = (t->flags & output_flag) ? MI355X_TENSOR_FLAG_OUTPUT : 0;
        for (int s = 0; s < 10; ++s) g.src[s] = s < max_src ? of(t->src[s]) : nullptr;
        g.view_src = of(t->view_src);
        g.view_offs = t->view_offs;
        g.data = t->data;
        std::strncpy(g.name, t->name, sizeof(g.name) - 1);
        return &g;
    }
};

// Per-context state of the adapter: the backend, the rope table of the context and the
// lowering's arena.
struct Context {
    mi355x_backend_t be = nullptr;
    void *rope_table = nullptr;
    int rope_n_pos = 0;
    float freq_base = 10000.f, freq_scale = 1.f;
    std::vector<mi355x_tensor> arena;
    std::vector<mi355x_tensor *> nodes;
};

// The cells == positions promise of mi355x_lower_opts, established from the graph's own
// inputs (host copies, T tokens): every token's K cell index (SET_ROWS k_idxs) equals its
// position (inp_pos), and its KQ mask row (SOFT_MAX src[1], n_kv entries per row, row
// stride `mask_row_bytes`, f32 or f16) is the causal mask over cells [0, pos]: 0 there and
// -INFINITY after. ATTN_DECODE stores cell pos and attends over [0, pos], so that is
// exactly what the graph asks for -- whatever the number of sequences in the cache: cells
// of another sequence, a removed or shifted cell inside [0, pos] shows up as a -INF entry
// there (or a k_idx that is not the position) and the promise is refused (the ADVICE r3
// gap: a one_sequence flag nobody could check).
inline bool cells_eq_pos(const int64_t *k_idxs, const int32_t *pos, int64_t n_tokens) {
    if (n_tokens <= 0 || !k_idxs || !pos) return false;
    for (int64_t i = 0; i < n_tokens; ++i)
        if (k_idxs[i] != (int64_t)pos[i] || pos[i] < 0) return false;
    return true;
}

// mask_type: 0 = f32, 1 = f16 (ggml type numbers)
inline bool kq_mask_causal(const void *mask, int mask_type, int64_t n_kv, size_t mask_row_bytes,
                           const int32_t *pos, int64_t n_tokens) {
    if (!mask || !pos || n_kv <= 0 || n_tokens <= 0 || (mask_type != 0 && mask_type != 1)) return false;
    for (int64_t t = 0; t < n_tokens; ++t) {
        if (pos[t] < 0 || pos[t] >= n_kv) return false;
        const unsigned char *row = (const unsigned char *)mask + (size_t)t * mask_row_bytes;
        for (int64_t j = 0; j < n_kv; ++j) {
            bool zero, ninf;
            if (mask_type == 0) {
                uint32_t u;
                std::memcpy(&u, row + 4 * j, 4);
                zero = (u & 0x7fffffffu) == 0;
                ninf = u == 0xff800000u;
            } else {
                uint16_t h;
                std::memcpy(&h, row + 2 * j, 2);
                zero = (h & 0x7fffu) == 0;
                ninf = h == 0xfc00u;
            }
            if (j <= pos[t] ? !zero : !ninf) return false;
        }
    }
    return true;
}

// Rope table parameters the lowering checks a ROPE node against (ggml rope op_params:
// [1] n_dims, [2] mode, [5] freq_base, [6] freq_scale as float bits).
struct RopeParams {
    int n_dims = 0;
    float freq_base = 0.f, freq_scale = 0.f;
};
template <typename Tensor>
inline bool rope_params_of(const Tensor *rope, RopeParams &p) {
    if (!rope) return false;
    p.n_dims = rope->op_params[1];
    std::memcpy(&p.freq_base, &rope->op_params[5], 4);
    std::memcpy(&p.freq_scale, &rope->op_params[6], 4);
    return p.n_dims > 0 && (p.n_dims % 2) == 0;
}

// Lower `n` graph nodes; 0 and the backend node list, or the lowering's status.
template <typename Tensor>
int lower(Context &ctx, Mirror<Tensor> &mir, Tensor *const *graph_nodes, int n, bool cells_ok, int *n_out) {
    std::vector<mi355x_gtensor *> g((size_t)n);
    for (int i = 0; i < n; ++i) g[(size_t)i] = mir.of(graph_nodes[i]);
    ctx.arena.resize(4 * (size_t)n + 64);
    ctx.nodes.resize(ctx.arena.size());
    mi355x_lower_opts opts;
    std::memset(&opts, 0, sizeof(opts));
    opts.rope_table = ctx.rope_table;
    opts.rope_n_pos = ctx.rope_n_pos;
    opts.rope_freq_base = ctx.freq_base;
    opts.rope_freq_scale = ctx.freq_scale;
    opts.cells_eq_pos = cells_ok ? 1 : 0;
    return mi355x_lower_ggml_graph(g.data(), n, &opts, ctx.arena.data(), (int)ctx.arena.size(), ctx.nodes.data(),
                                   (int)ctx.nodes.size(), n_out);
}

// graph_compute: lower, then run with hipGraph replay (decode steps repeat the graph).
template <typename Tensor>
int graph_compute(Context &ctx, Mirror<Tensor> &mir, Tensor *const *graph_nodes, int n, bool cells_ok) {
    int nn = 0;
    const int rc = lower(ctx, mir, graph_nodes, n, cells_ok, &nn);
    if (rc) return rc;
    return mi355x_backend_graph_compute(ctx.be, ctx.nodes.data(), nn, /*use_graph=*/1);
}

}  // namespace mi355x_adapter
