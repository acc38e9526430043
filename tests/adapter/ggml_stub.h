// ggml_stub.h — the few ggml functions the backend glue calls, implemented for the glue
// test (tests/adapter/ggml_stub.cpp); test infrastructure, not part of the product.
#pragma once

#include "ggml-backend-impl.h"

// a cgraph over `n` nodes (ggml_graph_n_nodes / ggml_graph_node read it)
struct ggml_cgraph *stub_graph_new(struct ggml_tensor **nodes, int n);
void stub_graph_free(struct ggml_cgraph *g);
// ggml_op by its ggml_op_name() string (GGML_OP_COUNT if unknown)
enum ggml_op stub_op_of_name(const char *name);
