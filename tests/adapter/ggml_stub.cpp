// ggml_stub.cpp — minimal implementations of the ggml calls the backend glue makes
// (ggml_op_name, ggml_nelements, ggml_nbytes, ggml_graph_n_nodes / _node,
// ggml_backend_buffer_init / _get_base / _get_size), for tests/adapter/glue_test.cpp.
// Semantics restated from ggml.c / ggml-backend.cpp [U]; test infrastructure only.
#include <cstring>

#include "ggml_stub.h"

struct ggml_cgraph {
    int n_nodes;
    struct ggml_tensor **nodes;
};

static const char *const kOpNames[GGML_OP_COUNT] = {
    "NONE",     "DUP",     "ADD",     "MUL",       "RMS_NORM", "MUL_MAT",  "MUL_MAT_ID",
    "SCALE",    "CPY",     "CONT",    "RESHAPE",   "VIEW",     "PERMUTE",  "TRANSPOSE",
    "GET_ROWS", "SET_ROWS", "SOFT_MAX", "ROPE",    "FLASH_ATTN_EXT", "UNARY", "GLU",
};

extern "C" {

const char *ggml_op_name(enum ggml_op op) { return (int)op >= 0 && op < GGML_OP_COUNT ? kOpNames[op] : "?"; }

const char *ggml_type_name(enum ggml_type type) {
    switch (type) {
        case GGML_TYPE_F32: return "f32";
        case GGML_TYPE_F16: return "f16";
        case GGML_TYPE_Q4_K: return "q4_K";
        case GGML_TYPE_Q5_K: return "q5_K";
        case GGML_TYPE_Q6_K: return "q6_K";
        case GGML_TYPE_I32: return "i32";
        case GGML_TYPE_I64: return "i64";
        default: return "?";
    }
}

int64_t ggml_nelements(const struct ggml_tensor *t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }

// ggml_nbytes: blck_size == 1 -> sum of (ne-1)*nb + type size; blocks -> ne0/blck*nb0 + ...
size_t ggml_nbytes(const struct ggml_tensor *t) {
    size_t blck = 1, tsize = 0;
    switch (t->type) {
        case GGML_TYPE_F32: case GGML_TYPE_I32: tsize = 4; break;
        case GGML_TYPE_F16: tsize = 2; break;
        case GGML_TYPE_I64: tsize = 8; break;
        case GGML_TYPE_Q4_K: blck = 256; tsize = 144; break;
        case GGML_TYPE_Q5_K: blck = 256; tsize = 176; break;
        case GGML_TYPE_Q6_K: blck = 256; tsize = 210; break;
        default: return 0;
    }
    size_t n;
    if (blck == 1) {
        n = tsize;
        for (int i = 0; i < GGML_MAX_DIMS; ++i) n += (size_t)(t->ne[i] - 1) * t->nb[i];
    } else {
        n = (size_t)t->ne[0] * t->nb[0] / blck;
        for (int i = 1; i < GGML_MAX_DIMS; ++i) n += (size_t)(t->ne[i] - 1) * t->nb[i];
    }
    return n;
}

bool ggml_guid_matches(ggml_guid_t a, ggml_guid_t b) { return std::memcmp(a, b, sizeof(ggml_guid)) == 0; }

int ggml_graph_n_nodes(struct ggml_cgraph *g) { return g->n_nodes; }

struct ggml_tensor *ggml_graph_node(struct ggml_cgraph *g, int i) {
    return i < 0 ? g->nodes[g->n_nodes + i] : g->nodes[i];
}

ggml_backend_buffer_t ggml_backend_buffer_init(ggml_backend_buffer_type_t buft, struct ggml_backend_buffer_i iface,
                                               void *context, size_t size) {
    return new ggml_backend_buffer{iface, buft, context, size, GGML_BACKEND_BUFFER_USAGE_ANY};
}

void *ggml_backend_buffer_get_base(ggml_backend_buffer_t b) { return b->iface.get_base(b); }
size_t ggml_backend_buffer_get_size(ggml_backend_buffer_t b) { return b->size; }

}  // extern "C"

struct ggml_cgraph *stub_graph_new(struct ggml_tensor **nodes, int n) { return new ggml_cgraph{n, nodes}; }
void stub_graph_free(struct ggml_cgraph *g) { delete g; }

enum ggml_op stub_op_of_name(const char *name) {
    for (int i = 0; i < GGML_OP_COUNT; ++i)
        if (std::strcmp(kOpNames[i], name) == 0) return (enum ggml_op)i;
    return GGML_OP_COUNT;
}
