// ggml-mi355x.cpp — the ggml backend glue, built inside llama.cpp's tree as
// ggml/src/ggml-mi355x/ggml-mi355x.cpp, linked with libggml_mi355x.so.
//
// Everything with logic lives in mi355x_ggml_mirror.hpp, which tests/test_adapter.py
// compiles and runs against include/ggml_mi355x.h here. This file only binds it to
// ggml's backend interface (ggml-backend-impl.h [U]; the reference pins llama.cpp
// a3cb0474, README.md:195, and does not vendor it, so it is not compiled in this repo).
#include <vector>

#include "ggml-backend-impl.h"
#include "ggml_mi355x.h"
#include "mi355x_ggml_mirror.hpp"

namespace {

const char *op_name(const ggml_tensor *t) { return ggml_op_name(t->op); }

struct mi355x_context : mi355x_adapter::Context {
    std::vector<int64_t> k_idxs;  // host copies for the cells == positions check
    std::vector<int32_t> pos;
};

// The promise mi355x_lower_opts.cells_eq_pos makes: the first SET_ROWS K index vector and
// inp_pos, read back (T entries each, small), are equal, and the batch is one sequence
// (the caller's ubatch: n_seqs == 1, no seq_rm / defrag / shift since the cache started).
bool cells_eq_pos_checked(mi355x_context *ctx, const ggml_cgraph *cg, bool one_sequence) {
    const ggml_tensor *k_idxs = nullptr, *pos = nullptr;
    for (int i = 0; i < cg->n_nodes && !(k_idxs && pos); ++i) {
        const ggml_tensor *t = cg->nodes[i];
        if (t->op == GGML_OP_SET_ROWS && !k_idxs) k_idxs = t->src[1];
        if (t->op == GGML_OP_ROPE && !pos) pos = t->src[1];
    }
    if (!k_idxs || !pos || k_idxs->type != GGML_TYPE_I64 || pos->type != GGML_TYPE_I32) return false;
    const int64_t T = ggml_nelements(pos);
    if (ggml_nelements(k_idxs) != T) return false;
    ctx->k_idxs.resize((size_t)T);
    ctx->pos.resize((size_t)T);
    mi355x_backend_get_tensor(ctx->be, ctx->k_idxs.data(), k_idxs->data, (size_t)T * sizeof(int64_t));
    mi355x_backend_get_tensor(ctx->be, ctx->pos.data(), pos->data, (size_t)T * sizeof(int32_t));
    mi355x_backend_synchronize(ctx->be);
    return mi355x_adapter::cells_eq_pos(ctx->k_idxs.data(), ctx->pos.data(), T, one_sequence);
}

enum ggml_status mi355x_graph_compute(ggml_backend_t backend, ggml_cgraph *cgraph) {
    auto *ctx = (mi355x_context *)backend->context;
    mi355x_adapter::Mirror<ggml_tensor> mir;
    mir.op_name = op_name;
    mir.output_flag = GGML_TENSOR_FLAG_OUTPUT;
    mir.max_src = GGML_MAX_SRC;
    const bool cells_ok = cells_eq_pos_checked(ctx, cgraph, /*one_sequence=*/true);
    const int rc = mi355x_adapter::graph_compute(*ctx, mir, cgraph->nodes, cgraph->n_nodes, cells_ok);
    return rc == 0 ? GGML_STATUS_SUCCESS : GGML_STATUS_FAILED;
}

// buffer interface: device memory, GGUF bytes copied unchanged (no repack)
void mi355x_buf_set_tensor(ggml_backend_buffer_t b, ggml_tensor *t, const void *data, size_t off, size_t n) {
    mi355x_backend_set_tensor((mi355x_backend_t)b->context, (char *)t->data + off, data, n);
}
void mi355x_buf_get_tensor(ggml_backend_buffer_t b, const ggml_tensor *t, void *data, size_t off, size_t n) {
    mi355x_backend_get_tensor((mi355x_backend_t)b->context, data, (const char *)t->data + off, n);
    mi355x_backend_synchronize((mi355x_backend_t)b->context);
}

}  // namespace

// The remaining slots are one-line forwards: alloc_buffer -> mi355x_backend_alloc,
// free_buffer -> mi355x_backend_free_buffer, synchronize -> mi355x_backend_synchronize,
// get_name -> mi355x_backend_name; supports_op accepts the K-quant MUL_MAT and the
// decode ops (the lowering's output nodes pass mi355x_backend_supports_op) and the
// attention members (ROPE, SET_ROWS, f16 MUL_MAT, SOFT_MAX, CONT) so the scheduler keeps
// the block on this backend, where the lowering fuses it.
ggml_backend_reg_t ggml_backend_mi355x_reg(void);  // + GGML_BACKEND_DL_IMPL(ggml_backend_mi355x_reg)
