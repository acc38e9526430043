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

struct mi355x_backend {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string name;
    void *workspace = nullptr;
    size_t workspace_size = 0;
    std::vector<uint64_t> graph_key;
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
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
    drop_graph(b);  // a captured graph may reference the buffer
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
    return e == hipSuccess ? 0 : (int)e;
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
    if (!use_graph) return enqueue(b, nodes, launches);

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
