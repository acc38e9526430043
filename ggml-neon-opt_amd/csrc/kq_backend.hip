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
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "kq_common.h"
#include "kq_internal.h"

// A node list planned as one persistent kq_chain launch (kq_chain.hip).
struct ChainCache {
    std::vector<uint64_t> key;
    bool ok = false;  // key planned; false: not eligible, use per-stage launches
    uint8_t *d_stages = nullptr;  // stage table, kq::kChainSlotBytes per stage
    uint32_t *sync = nullptr;  // epoch, finished workgroups, timeout flag
    std::vector<void *> bus;
    kq::ChainArgs args{};
    size_t lds = 0;
    double bytes = 0;
};

struct mi355x_backend {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string name;
    void *workspace = nullptr;
    size_t workspace_size = 0;
    std::vector<uint64_t> graph_key;
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    ChainCache chain;
    std::vector<uint32_t *> old_sync;
};

namespace {

bool is_kquant(int t) { return t == MI355X_TYPE_Q4_K || t == MI355X_TYPE_Q5_K || t == MI355X_TYPE_Q6_K; }

void drop_graph(mi355x_backend *b) {
    if (b->graph_exec) hipGraphExecDestroy(b->graph_exec);
    if (b->graph) hipGraphDestroy(b->graph);
    b->graph_exec = nullptr;
    b->graph = nullptr;
    b->graph_key.clear();
}

// One launch: a MUL_MAT node, or a run of ne11 == 1 MUL_MAT nodes sharing src1.
struct Launch {
    int first, count;
};

std::vector<Launch> plan_launches(mi355x_tensor *const *nodes, int n) {
    std::vector<Launch> out;
    int i = 0;
    while (i < n) {
        const mi355x_tensor *t = nodes[i];
        int cnt = 1;
        if (t->op == MI355X_OP_MUL_MAT && t->src[1]->ne[1] == 1) {
            while (i + cnt < n && cnt < MI355X_MAX_FUSED) {
                const mi355x_tensor *u = nodes[i + cnt];
                if (u->op != MI355X_OP_MUL_MAT || u->src[1]->ne[1] != 1) break;
                if (u->src[1]->data != t->src[1]->data || u->src[0]->ne[0] != t->src[0]->ne[0]) break;
                ++cnt;
            }
        }
        out.push_back({i, cnt});
        i += cnt;
    }
    return out;
}

int enqueue(mi355x_backend *b, mi355x_tensor *const *nodes, const std::vector<Launch> &launches) {
    for (const Launch &l : launches) {
        const mi355x_tensor *t = nodes[l.first];
        if (t->op == MI355X_OP_NONE) continue;
        const mi355x_tensor *w = t->src[0], *x = t->src[1];
        int rc;
        if (l.count > 1 || x->ne[1] == 1) {
            mi355x_gemv_desc d[MI355X_MAX_FUSED];
            for (int k = 0; k < l.count; ++k) {
                const mi355x_tensor *n = nodes[l.first + k];
                d[k].type = n->src[0]->type;
                d[k].w = n->src[0]->data;
                d[k].n_rows = n->src[0]->ne[1];
                d[k].row_stride = n->src[0]->nb[1];
                d[k].y = (float *)n->data;
            }
            rc = mi355x_gemv_fused(d, l.count, (const float *)x->data, w->ne[0], b->workspace, b->workspace_size,
                                   b->stream);
        } else {
            rc = mi355x_mul_mat(w->type, w->data, w->ne[0], w->ne[1], w->nb[1], (const float *)x->data, x->ne[1],
                                x->nb[1], (float *)t->data, t->nb[1], b->workspace, b->workspace_size,
                                b->stream);
        }
        if (rc) return rc;
    }
    return 0;
}

void drop_chain(mi355x_backend *b) {
    ChainCache &c = b->chain;
    if (c.d_stages) hipFree(c.d_stages);
    for (void *p : c.bus) hipFree(p);
    if (c.sync) b->old_sync.push_back(c.sync);  // its timeout flag is still reported once
    c = ChainCache();
}

std::vector<uint64_t> graph_key_of(mi355x_tensor *const *nodes, int n_nodes) {
    std::vector<uint64_t> key;
    key.reserve((size_t)n_nodes * 16);
    for (int i = 0; i < n_nodes; ++i) {
        const mi355x_tensor *t = nodes[i];
        key.push_back((uint64_t)(uintptr_t)t->data);
        key.push_back((uint64_t)t->op);
        for (int s = 0; s < 2; ++s) {
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

bool overlaps(uintptr_t a0, uintptr_t a1, uintptr_t b0, uintptr_t b1) { return a0 < b1 && b0 < a1; }

// Plan the node list as one kq_chain launch. Eligible: >= 2 launches, every one a
// decode stage (ne11 == 1) that kq_rows takes with the fused quantizer; each
// stage's activation is either exactly an earlier node's output (read from that
// node's bus: a true RAW dependency, honoured by the hand-off) or memory that no
// node of the list writes; outputs pairwise disjoint. Anything else keeps the
// per-stage launches, which are stream-ordered.
int plan_chain(mi355x_backend *b, mi355x_tensor *const *nodes, int n_nodes, const std::vector<Launch> &launches) {
    ChainCache &c = b->chain;
    if (launches.size() < 2) return MI355X_E_UNSUPPORTED;
    struct Range {
        uintptr_t a0, a1;
    };
    std::vector<Range> dst;
    for (int i = 0; i < n_nodes; ++i) {
        const mi355x_tensor *t = nodes[i];
        if (t->op != MI355X_OP_MUL_MAT || t->src[1]->ne[1] != 1) return MI355X_E_UNSUPPORTED;
        dst.push_back({(uintptr_t)t->data, (uintptr_t)t->data + (uintptr_t)t->ne[0] * 4});
    }
    for (size_t i = 0; i < dst.size(); ++i)
        for (size_t j = i + 1; j < dst.size(); ++j)
            if (overlaps(dst[i].a0, dst[i].a1, dst[j].a0, dst[j].a1)) return MI355X_E_UNSUPPORTED;
    std::vector<kq::ChainStage> st(launches.size());
    std::vector<int> node_stage(n_nodes, -1), node_desc(n_nodes, -1);
    std::vector<int> producer(launches.size(), -1);
    kq::ChainFit fit;
    for (size_t li = 0; li < launches.size(); ++li) {
        const Launch &l = launches[li];
        const mi355x_tensor *t = nodes[l.first];
        const mi355x_tensor *w = t->src[0], *x = t->src[1];
        const int64_t K = w->ne[0];
        mi355x_gemv_desc d[MI355X_MAX_FUSED];
        for (int k = 0; k < l.count; ++k) {
            const mi355x_tensor *n = nodes[l.first + k];
            d[k].type = n->src[0]->type;
            d[k].w = n->src[0]->data;
            d[k].n_rows = n->src[0]->ne[1];
            d[k].row_stride = n->src[0]->nb[1];
            d[k].y = (float *)n->data;
            node_stage[l.first + k] = (int)li;
            node_desc[l.first + k] = k;
        }
        int rc = kq::plan_chain_stage(d, l.count, K, st[li], fit);
        if (rc) return rc;
        const uintptr_t x0 = (uintptr_t)x->data, x1 = x0 + (uintptr_t)K * 4;
        for (int j = 0; j < l.first; ++j)
            if ((uintptr_t)nodes[j]->data == x0 && nodes[j]->ne[0] >= K) producer[li] = j;
        if (producer[li] < 0) {
            if (x0 & 15u) return MI355X_E_UNSUPPORTED;
            for (const Range &r : dst)
                if (overlaps(x0, x1, r.a0, r.a1)) return MI355X_E_UNSUPPORTED;
            st[li].x = (const float *)x->data;
        }
    }
    size_t lds = 0;
    kq::ChainArgs a{};
    int rc = kq::chain_layout(fit, a, lds);
    if (rc) return rc;
    // buses of the nodes some stage reads
    for (size_t li = 0; li < launches.size(); ++li) {
        const int j = producer[li];
        if (j < 0) continue;
        kq::ChainStage &ps = st[node_stage[j]];
        const int k = node_desc[j];
        if (!ps.bus[k]) {
            void *p = nullptr;
            const size_t bytes = (size_t)nodes[j]->ne[0] * 8;
            if (hipMalloc(&p, bytes) != hipSuccess) return MI355X_E_WORKSPACE;
            c.bus.push_back(p);
            if (hipMemsetAsync(p, 0, bytes, b->stream) != hipSuccess) return MI355X_E_WORKSPACE;  // tag 0 never matches
            ps.bus[k] = (uint32_t *)p;
        }
        st[li].xbus = ps.bus[k];
    }
    std::vector<uint8_t> table(st.size() * kq::kChainSlotBytes, 0);
    for (size_t i = 0; i < st.size(); ++i) memcpy(table.data() + i * kq::kChainSlotBytes, &st[i], sizeof(kq::ChainStage));
    if (hipMalloc(&c.d_stages, table.size()) != hipSuccess) return MI355X_E_WORKSPACE;
    if (hipMalloc(&c.sync, 64) != hipSuccess) return MI355X_E_WORKSPACE;
    if (hipMemcpyAsync(c.d_stages, table.data(), table.size(), hipMemcpyHostToDevice, b->stream) != hipSuccess ||
        hipMemsetAsync(c.sync, 0, 64, b->stream) != hipSuccess || hipStreamSynchronize(b->stream) != hipSuccess)
        return MI355X_E_WORKSPACE;
    a.st = c.d_stages;
    a.n_stages = (int)st.size();
    a.sync = c.sync;
    c.args = a;
    c.lds = lds;
    c.bytes = fit.bytes;
    c.ok = true;
    return MI355X_OK;
}

// Report (once) a hand-off timeout of any chain launched on this backend.
int chain_status(mi355x_backend *b) {
    std::vector<uint32_t *> syncs = b->old_sync;
    if (b->chain.sync) syncs.push_back(b->chain.sync);
    int rc = MI355X_OK;
    for (uint32_t *s : syncs) {
        uint32_t w[8] = {0};
        if (hipMemcpy(w, s + 2, sizeof(w), hipMemcpyDeviceToHost) != hipSuccess) continue;
        if (w[0]) {
            fprintf(stderr, "ggml_mi355x: kq_chain hand-off timed out: stage %u, workgroup %u, superblock %u, tag seen %u, expected %u\n",
                    w[1], w[2], w[3], w[4], w[5]);
            rc = MI355X_E_TIMEOUT;
            hipMemset(s + 2, 0, sizeof(w));
        }
    }
    for (uint32_t *s : b->old_sync) hipFree(s);
    b->old_sync.clear();
    return rc;
}

}  // namespace

extern "C" {

mi355x_backend_t mi355x_backend_init(int device) {
    if (!kq::device_ok()) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
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
    hipStreamSynchronize(b->stream);
    drop_graph(b);
    drop_chain(b);
    for (uint32_t *s : b->old_sync) hipFree(s);
    if (b->workspace) hipFree(b->workspace);
    hipStreamDestroy(b->stream);
    delete b;
}

const char *mi355x_backend_name(mi355x_backend_t b) { return b ? b->name.c_str() : "MI355X"; }

void *mi355x_backend_stream(mi355x_backend_t b) { return b ? (void *)b->stream : nullptr; }

void *mi355x_backend_alloc(mi355x_backend_t b, size_t size) {
    if (!b) return nullptr;
    void *p = nullptr;
    if (hipMalloc(&p, size ? size : 1) != hipSuccess) return nullptr;
    return p;
}

void mi355x_backend_free_buffer(mi355x_backend_t b, void *ptr) {
    if (!b || !ptr) return;
    hipStreamSynchronize(b->stream);
    drop_graph(b);  // a captured graph or a chain plan may reference the buffer
    drop_chain(b);
    hipFree(ptr);
}

int mi355x_backend_set_tensor(mi355x_backend_t b, void *dst, const void *host_src, size_t size) {
    if (!b || (!dst && size)) return MI355X_E_INVAL;
    const hipError_t e = hipMemcpyAsync(dst, host_src, size, hipMemcpyHostToDevice, b->stream);
    return e == hipSuccess ? 0 : (int)e;
}

int mi355x_backend_get_tensor(mi355x_backend_t b, void *host_dst, const void *src, size_t size) {
    if (!b || (!src && size)) return MI355X_E_INVAL;
    const hipError_t e = hipMemcpyAsync(host_dst, src, size, hipMemcpyDeviceToHost, b->stream);
    return e == hipSuccess ? 0 : (int)e;
}

int mi355x_backend_synchronize(mi355x_backend_t b) {
    if (!b) return MI355X_E_INVAL;
    const hipError_t e = hipStreamSynchronize(b->stream);
    if (e != hipSuccess) return (int)e;
    return chain_status(b);
}

// ggml_backend_device_i::supports_op for this device: MUL_MAT of a contiguous-row
// K-quant src0 with an f32 src1, 2-D (no broadcast over ne2/ne3).
int mi355x_backend_supports_op(const mi355x_tensor *op) {
    if (!op) return 0;
    if (op->op == MI355X_OP_NONE) return 1;
    if (op->op != MI355X_OP_MUL_MAT) return 0;
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

int mi355x_backend_graph_compute(mi355x_backend_t b, mi355x_tensor *const *nodes, int n_nodes, int use_graph) {
    if (!b || (n_nodes > 0 && !nodes) || n_nodes < 0) return MI355X_E_INVAL;
    size_t ws = 0;
    for (int i = 0; i < n_nodes; ++i) {
        if (!mi355x_backend_supports_op(nodes[i])) return MI355X_E_UNSUPPORTED;
        if (nodes[i]->op == MI355X_OP_MUL_MAT) {
            const mi355x_tensor *w = nodes[i]->src[0];
            size_t need = mi355x_mul_mat_workspace_size(w->type, w->ne[0], w->ne[1], nodes[i]->src[1]->ne[1]);
            const size_t nf = mi355x_gemv_fused_workspace_size(w->ne[0]);
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
    const std::vector<Launch> launches = plan_launches(nodes, n_nodes);
    const bool try_chain = kq::chain_enabled() && launches.size() >= 2;
    if (!use_graph && !try_chain) return enqueue(b, nodes, launches);
    std::vector<uint64_t> key = graph_key_of(nodes, n_nodes);
    if (try_chain) {
        if (b->chain.key != key) {
            hipStreamSynchronize(b->stream);  // a running chain may still use the old plan
            drop_chain(b);
            b->chain.key = key;
            if (plan_chain(b, nodes, n_nodes, launches) != MI355X_OK) {
                drop_chain(b);
                b->chain.key = key;  // remembered as not eligible
            }
        }
        if (b->chain.ok) return kq::launch_chain(b->chain.args, b->chain.lds, b->chain.bytes, b->stream);
        if (!use_graph) return enqueue(b, nodes, launches);
    }
    if (!b->graph_exec || key != b->graph_key) {
        drop_graph(b);
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
        b->graph = g;
        b->graph_exec = ge;
        b->graph_key.swap(key);
    }
    const hipError_t e = hipGraphLaunch(b->graph_exec, b->stream);
    return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"
