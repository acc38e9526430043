// kq_lower.cpp — lowering of a ggml decode graph (llm_build_llama, one token,
// non-flash attention) onto this backend's node list (host only, no device calls).
//
// The reference runs the graph node by node on ggml-cpu (ggml_graph_compute_thread ->
// ggml_compute_forward, artifacts/perf/out.folded:91-234; CPU backend entry
// ggml-cpu.cpp:186, README.md:162). A ggml backend built on this library receives the
// same ggml_cgraph in its graph_compute; its adapter mirrors each ggml_tensor as an
// mi355x_gtensor (same fields) and calls mi355x_lower_ggml_graph, then
// mi355x_backend_graph_compute on the result. What the lowering does:
//  * view-like ops (RESHAPE, VIEW, PERMUTE, TRANSPOSE) are aliases of their source;
//  * GET_ROWS / RMS_NORM / MUL / ADD / MUL_MAT / GLU(SWIGLU) become one node each;
//  * the attention block of llama-graph.cpp's build_attn (non-flash: ROPE(Q), ROPE(K),
//    SET_ROWS into the K and V caches, MUL_MAT(K cache, Q), SOFT_MAX_EXT(kq, mask,
//    scale), MUL_MAT(V cache, kq), PERMUTE, CONT [U]) becomes one ATTN_DECODE node with
//    the pre-rope q/k/v, the position, both caches and the caller's rope table;
//  * the [up, gate] MUL_MAT pair build_ffn emits before SWIGLU(gate, up) [U] is put in
//    [gate, up] order (the two nodes are independent) so the gate/up launch fuses.
// Anything else returns MI355X_E_UNSUPPORTED: the caller hands the graph to another
// backend, as ggml's scheduler does for supports_op == false.
#include <stdint.h>
#include <string.h>

#include <unordered_map>
#include <vector>

#include "ggml_mi355x.h"

namespace {

constexpr int kTypeF32 = MI355X_TYPE_F32, kTypeF16 = 1, kTypeI32 = 26, kTypeI64 = 27;

float f_of(int32_t bits) {
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

bool is_alias(int op) {
    return op == MI355X_GOP_RESHAPE || op == MI355X_GOP_VIEW || op == MI355X_GOP_PERMUTE ||
           op == MI355X_GOP_TRANSPOSE;
}
bool is_kquant(int t) { return t == MI355X_TYPE_Q4_K || t == MI355X_TYPE_Q5_K || t == MI355X_TYPE_Q6_K; }

// Follow alias ops (and SET_ROWS's destination view) down to the producing node or leaf.
const mi355x_gtensor *root(const mi355x_gtensor *t) {
    while (t && is_alias(t->op) && t->src[0]) t = t->src[0];
    return t;
}
const mi355x_gtensor *dest_root(const mi355x_gtensor *t) {  // the buffer a SET_ROWS writes
    const mi355x_gtensor *d = t->view_src;
    while (d && (is_alias(d->op) || d->view_src)) d = is_alias(d->op) && d->src[0] ? d->src[0] : d->view_src;
    return d;
}

struct Lower {
    mi355x_gtensor *const *g;
    int n;
    const mi355x_lower_opts *opts;
    mi355x_tensor *arena;
    int cap, used = 0;
    std::unordered_map<const mi355x_gtensor *, mi355x_tensor *> val;  // lowered node / leaf mirror
    std::unordered_map<const mi355x_gtensor *, int> uses;             // reads by graph nodes (through aliases)
    std::vector<mi355x_tensor *> out;
    int err = MI355X_OK;

    mi355x_tensor *alloc() {
        if (used >= cap) {
            err = MI355X_E_WORKSPACE;
            return nullptr;
        }
        mi355x_tensor *t = &arena[used++];
        memset(t, 0, sizeof(*t));
        return t;
    }

    // Mirror of a ggml leaf (weights, norms, inputs, caches; views of them keep their own
    // data pointer, ne and nb, as ggml sets them).
    mi355x_tensor *leaf(const mi355x_gtensor *t) {
        auto it = val.find(t);
        if (it != val.end()) return it->second;
        mi355x_tensor *m = alloc();
        if (!m) return nullptr;
        m->type = t->type;
        m->op = MI355X_OP_NONE;
        for (int d = 0; d < 4; ++d) {
            m->ne[d] = t->ne[d];
            m->nb[d] = t->nb[d];
        }
        m->data = t->data;
        val[t] = m;
        return m;
    }

    // The value a node operand reads: the lowered producer, or a leaf mirror.
    mi355x_tensor *value(const mi355x_gtensor *t) {
        if (!t) {
            err = MI355X_E_INVAL;
            return nullptr;
        }
        const mi355x_gtensor *r = root(t);
        auto it = val.find(r);
        if (it != val.end()) return it->second;
        if (r->op == MI355X_GOP_NONE) return leaf(t);  // (a view of a leaf: its own data/shape)
        err = MI355X_E_UNSUPPORTED;                       // a producer this lowering skipped
        return nullptr;
    }

    mi355x_tensor *emit(const mi355x_gtensor *t, int op, std::initializer_list<mi355x_tensor *> srcs) {
        mi355x_tensor *m = alloc();
        if (!m) return nullptr;
        m->type = kTypeF32;
        m->op = op;
        for (int d = 0; d < 4; ++d) {
            m->ne[d] = t->ne[d];
            m->nb[d] = t->nb[d];
        }
        int s = 0;
        for (mi355x_tensor *x : srcs) {
            if (!x) {
                if (err == MI355X_OK) err = MI355X_E_UNSUPPORTED;
                return nullptr;
            }
            m->src[s++] = x;
        }
        m->data = t->data;
        m->flags = t->flags & MI355X_TENSOR_FLAG_OUTPUT;
        val[t] = m;
        out.push_back(m);
        return m;
    }

    bool rope_ok(const mi355x_gtensor *r, int hd) const {
        if (!r || r->op != MI355X_GOP_ROPE || r->ne[2] < 1 || r->ne[3] != 1) return false;  // [hd, heads, tokens]
        // freq_factors (src[2], Llama-3.1+ rope_freqs): the caller's table carries none
        if (r->src[2]) return false;
        if (r->op_params[1] != hd || r->op_params[2] != 0) return false;   // n_dims, mode NORMAL
        if (f_of(r->op_params[5]) != opts->rope_freq_base || f_of(r->op_params[6]) != opts->rope_freq_scale)
            return false;
        return f_of(r->op_params[7]) == 0.0f && f_of(r->op_params[8]) == 1.0f;  // ext_factor, attn_factor
    }

    // A SET_ROWS index operand: an I32/I64 leaf of `n` entries (its contents live on the
    // device; what they hold is the adapter's cells_eq_pos promise).
    static bool idx_ok(const mi355x_gtensor *t, int64_t n) {
        const mi355x_gtensor *r = root(t);
        return r && r->op == MI355X_GOP_NONE && (t->type == kTypeI32 || t->type == kTypeI64) && t->ne[0] == n &&
               t->ne[1] == 1 && t->ne[2] == 1 && t->ne[3] == 1;
    }

    // The attention block ending at CONT node `c` -> one ATTN_DECODE. ATTN_DECODE writes
    // each token's K/V at cell == its position and attends causally over [0, pos]; that
    // is the block's meaning only under the adapter's cells_eq_pos promise (one sequence,
    // k_idxs == v_idxs cells == inp_pos, causal mask, views from cell 0), so without it
    // the block is not lowered.
    bool attention(const mi355x_gtensor *c) {
        if (!opts->cells_eq_pos) return false;
        const mi355x_gtensor *p = c->src[0];
        if (!p || p->op != MI355X_GOP_PERMUTE) return false;
        const mi355x_gtensor *kqv = root(p->src[0]);
        if (!kqv || kqv->op != MI355X_GOP_MUL_MAT || !kqv->src[0] || kqv->src[0]->type != kTypeF16) return false;
        const mi355x_gtensor *sm = root(kqv->src[1]);
        if (!sm || sm->op != MI355X_GOP_SOFT_MAX || !sm->src[1] || sm->src[2]) return false;  // mask, no sinks
        if (f_of(sm->op_params[1]) != 0.0f) return false;                                      // max_bias
        const mi355x_gtensor *kq = root(sm->src[0]);
        if (!kq || kq->op != MI355X_GOP_MUL_MAT || !kq->src[0] || kq->src[0]->type != kTypeF16) return false;
        const mi355x_gtensor *rq = root(kq->src[1]);
        const mi355x_gtensor *kcache = root(kq->src[0]), *vcache = root(kqv->src[0]);
        if (!rq || rq->op != MI355X_GOP_ROPE) return false;
        const int hd = (int)rq->ne[0], nh = (int)rq->ne[1];
        if (!rope_ok(rq, hd)) return false;
        // the SET_ROWS writing the K and V caches
        const mi355x_gtensor *sk = nullptr, *sv = nullptr;
        for (int i = 0; i < n; ++i) {
            const mi355x_gtensor *t = g[i];
            if (t->op != MI355X_GOP_SET_ROWS) continue;
            const mi355x_gtensor *d = dest_root(t);
            if (d == kcache) sk = t;
            if (d == vcache) sv = t;
        }
        if (!sk || !sv) return false;
        const mi355x_gtensor *rk = root(sk->src[0]);
        if (!rk || rk->op != MI355X_GOP_ROPE || !rope_ok(rk, hd) || rk->ne[0] != hd) return false;
        const int nkv = (int)rk->ne[1];
        if (nkv <= 0 || nh % nkv) return false;
        const int64_t T = rq->ne[2];  // tokens of the batch (1: a decode token; > 1: a prompt)
        if (rk->ne[2] != T) return false;
        // one K row per token; the transposed V store scatters one index per element
        if (!idx_ok(sk->src[1], T) || !idx_ok(sv->src[1], (int64_t)nkv * hd * T)) return false;
        // the KQ / KQV operands are views of the caches from cell 0
        if (kq->src[0]->view_offs != 0 || kqv->src[0]->view_offs != 0) return false;
        const mi355x_gtensor *qmm = root(rq->src[0]), *kmm = root(rk->src[0]), *vmm = root(sv->src[0]);
        if (!qmm || !kmm || !vmm || qmm->op != MI355X_GOP_MUL_MAT || kmm->op != MI355X_GOP_MUL_MAT ||
            vmm->op != MI355X_GOP_MUL_MAT)
            return false;
        // the block's inner values feed nothing outside it
        if (uses[rq] != 1 || uses[rk] != 1 || uses[sm] != 1 || uses[kq] != 1 || uses[kqv] != 1) return false;
        const mi355x_gtensor *pos = rq->src[1];
        if (!pos || root(rk->src[1]) != root(pos) || pos->type != kTypeI32 || pos->ne[0] != T) return false;
        if (kcache->type != kTypeF16 || vcache->type != kTypeF16 || kcache->ne[0] != (int64_t)nkv * hd ||
            vcache->ne[1] != (int64_t)nkv * hd || vcache->ne[0] != kcache->ne[1])
            return false;
        if (!opts->rope_table || opts->rope_n_pos < kcache->ne[1]) return false;
        mi355x_tensor *tab = alloc();
        if (!tab) return false;
        tab->type = kTypeF32;
        tab->ne[0] = hd;
        tab->ne[1] = opts->rope_n_pos;
        tab->ne[2] = tab->ne[3] = 1;
        tab->nb[0] = 4;
        tab->nb[1] = (size_t)hd * 4;
        tab->nb[2] = tab->nb[3] = tab->nb[1] * (size_t)opts->rope_n_pos;
        tab->data = opts->rope_table;
        mi355x_tensor *a = emit(c, MI355X_OP_ATTN_DECODE,
                                {value(qmm), value(kmm), value(vmm), leaf(root(pos)), leaf(kcache), leaf(vcache), tab});
        if (!a) return false;
        a->ne[0] = (int64_t)nh * hd;
        a->ne[1] = T;
        a->ne[2] = a->ne[3] = 1;
        a->nb[0] = 4;
        a->nb[1] = (size_t)nh * hd * 4;
        a->nb[2] = a->nb[3] = (size_t)nh * hd * 4 * (size_t)T;
        a->op_params[0] = nh;
        a->op_params[1] = nkv;
        a->op_params[2] = hd;
        a->op_params[3] = sm->op_params[0];  // kq_scale (float bits)
        return true;
    }

    int run() {
        for (int i = 0; i < n; ++i) {  // reads through aliases count once, at the real reader
            if (is_alias(g[i]->op)) continue;
            for (int s = 0; s < 10; ++s)
                if (g[i]->src[s]) ++uses[root(g[i]->src[s])];
        }
        for (int i = 0; i < n && err == MI355X_OK; ++i) {
            const mi355x_gtensor *t = g[i];
            switch (t->op) {
                case MI355X_GOP_NONE:
                case MI355X_GOP_RESHAPE:
                case MI355X_GOP_VIEW:
                case MI355X_GOP_PERMUTE:
                case MI355X_GOP_TRANSPOSE:
                    break;  // aliases (and leaves listed among the nodes)
                case MI355X_GOP_ROPE:
                case MI355X_GOP_SET_ROWS:
                case MI355X_GOP_SOFT_MAX:
                    break;  // members of an attention block, lowered at its CONT
                case MI355X_GOP_GET_ROWS:
                    if (t->type != kTypeF32) return MI355X_E_UNSUPPORTED;
                    emit(t, MI355X_OP_GET_ROWS, {leaf(root(t->src[0])), value(t->src[1])});
                    break;
                case MI355X_GOP_RMS_NORM: {
                    mi355x_tensor *m = emit(t, MI355X_OP_RMS_NORM, {value(t->src[0])});
                    if (m) m->op_params[0] = t->op_params[0];  // eps (float bits)
                    break;
                }
                case MI355X_GOP_MUL:
                    emit(t, MI355X_OP_MUL, {value(t->src[0]), value(t->src[1])});
                    break;
                case MI355X_GOP_ADD:
                    emit(t, MI355X_OP_ADD, {value(t->src[0]), value(t->src[1])});
                    break;
                case MI355X_GOP_MUL_MAT: {
                    const mi355x_gtensor *w = root(t->src[0]);
                    if (w && w->type == kTypeF16) break;  // the attention's KQ / KQV: at CONT
                    if (!w || !is_kquant(w->type) || w->op != MI355X_GOP_NONE) return MI355X_E_UNSUPPORTED;
                    emit(t, MI355X_OP_MUL_MAT, {leaf(t->src[0]), value(t->src[1])});
                    break;
                }
                case MI355X_GOP_GLU:
                    if (t->op_params[0] != MI355X_GLU_SWIGLU || !t->src[1] || t->op_params[1] != 0)
                        return MI355X_E_UNSUPPORTED;  // split SWIGLU, not swapped
                    emit(t, MI355X_OP_SWIGLU, {value(t->src[0]), value(t->src[1])});
                    break;
                case MI355X_GOP_CONT:
                case MI355X_GOP_CPY:
                    if (t->op == MI355X_GOP_CONT && attention(t)) break;
                    if (err != MI355X_OK) return err;
                    return MI355X_E_UNSUPPORTED;
                default:
                    return MI355X_E_UNSUPPORTED;
            }
        }
        if (err != MI355X_OK) return err;
        // [up, gate] -> [gate, up] ahead of SWIGLU(gate, up): independent MUL_MATs on one input
        for (size_t j = 2; j < out.size(); ++j) {
            mi355x_tensor *sg = out[j];
            if (sg->op != MI355X_OP_SWIGLU) continue;
            mi355x_tensor *a = out[j - 2], *b = out[j - 1];
            if (a->op == MI355X_OP_MUL_MAT && b->op == MI355X_OP_MUL_MAT && a->src[1] == b->src[1] &&
                sg->src[0] == b && sg->src[1] == a) {
                out[j - 2] = b;
                out[j - 1] = a;
            }
        }
        return MI355X_OK;
    }
};

}  // namespace

extern "C" int mi355x_lower_ggml_graph(mi355x_gtensor *const *gnodes, int n, const mi355x_lower_opts *opts,
                                       mi355x_tensor *arena, int arena_cap, mi355x_tensor **nodes_out, int nodes_cap,
                                       int *n_nodes) {
    if (!gnodes || n < 0 || !opts || !arena || arena_cap <= 0 || !nodes_out || !n_nodes) return MI355X_E_INVAL;
    for (int i = 0; i < n; ++i)
        if (!gnodes[i]) return MI355X_E_INVAL;
    Lower L{gnodes, n, opts, arena, arena_cap};
    const int rc = L.run();
    *n_nodes = 0;
    if (rc) return rc;
    if ((int)L.out.size() > nodes_cap) return MI355X_E_WORKSPACE;
    for (size_t i = 0; i < L.out.size(); ++i) nodes_out[i] = L.out[i];
    *n_nodes = (int)L.out.size();
    return MI355X_OK;
}
