// Restated SUBSET of ggml/include/ggml.h at llama.cpp a3cb0474 (build 6735, the
// reference's pin, README.md:195) [U]: only what adapter/ggml-mi355x.cpp and
// adapter/mi355x_ggml_mirror.hpp use, with upstream's names, field order and array
// sizes, so that the glue compiles here exactly as inside llama.cpp's tree. Test
// infrastructure: the reference does not vendor llama.cpp, so this is
// a from-memory restatement, not a copy. Enum VALUES of ggml_op are not upstream's
// (the list is abridged); the glue never depends on them (ops are matched by name).
#pragma once

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_API
#define GGML_MAX_DIMS 4
#define GGML_MAX_SRC 10
#define GGML_MAX_NAME 64
#define GGML_MAX_OP_PARAMS 64

enum ggml_status {
    GGML_STATUS_ALLOC_FAILED = -2,
    GGML_STATUS_FAILED = -1,
    GGML_STATUS_SUCCESS = 0,
    GGML_STATUS_ABORTED = 1,
};

typedef uint16_t ggml_fp16_t;

enum ggml_type {
    GGML_TYPE_F32 = 0,
    GGML_TYPE_F16 = 1,
    GGML_TYPE_Q4_0 = 2,
    GGML_TYPE_Q4_1 = 3,
    GGML_TYPE_Q5_0 = 6,
    GGML_TYPE_Q5_1 = 7,
    GGML_TYPE_Q8_0 = 8,
    GGML_TYPE_Q8_1 = 9,
    GGML_TYPE_Q2_K = 10,
    GGML_TYPE_Q3_K = 11,
    GGML_TYPE_Q4_K = 12,
    GGML_TYPE_Q5_K = 13,
    GGML_TYPE_Q6_K = 14,
    GGML_TYPE_Q8_K = 15,
    GGML_TYPE_I8 = 24,
    GGML_TYPE_I16 = 25,
    GGML_TYPE_I32 = 26,
    GGML_TYPE_I64 = 27,
    GGML_TYPE_F64 = 28,
    GGML_TYPE_BF16 = 30,
    GGML_TYPE_COUNT = 39,
};

// abridged, upstream order (values differ)
enum ggml_op {
    GGML_OP_NONE = 0,
    GGML_OP_DUP,
    GGML_OP_ADD,
    GGML_OP_MUL,
    GGML_OP_RMS_NORM,
    GGML_OP_MUL_MAT,
    GGML_OP_MUL_MAT_ID,
    GGML_OP_SCALE,
    GGML_OP_CPY,
    GGML_OP_CONT,
    GGML_OP_RESHAPE,
    GGML_OP_VIEW,
    GGML_OP_PERMUTE,
    GGML_OP_TRANSPOSE,
    GGML_OP_GET_ROWS,
    GGML_OP_SET_ROWS,
    GGML_OP_SOFT_MAX,
    GGML_OP_ROPE,
    GGML_OP_FLASH_ATTN_EXT,
    GGML_OP_UNARY,
    GGML_OP_GLU,
    GGML_OP_COUNT,
};

enum ggml_glu_op {
    GGML_GLU_OP_REGLU,
    GGML_GLU_OP_GEGLU,
    GGML_GLU_OP_SWIGLU,
    GGML_GLU_OP_COUNT,
};

enum ggml_tensor_flag {
    GGML_TENSOR_FLAG_INPUT = 1,
    GGML_TENSOR_FLAG_OUTPUT = 2,
    GGML_TENSOR_FLAG_PARAM = 4,
    GGML_TENSOR_FLAG_LOSS = 8,
};

typedef uint8_t ggml_guid[16];
typedef ggml_guid *ggml_guid_t;

struct ggml_backend_buffer;
struct ggml_cgraph;

struct ggml_tensor {
    enum ggml_type type;
    struct ggml_backend_buffer *buffer;
    int64_t ne[GGML_MAX_DIMS];
    size_t nb[GGML_MAX_DIMS];
    enum ggml_op op;
    int32_t op_params[GGML_MAX_OP_PARAMS / sizeof(int32_t)];
    int32_t flags;
    struct ggml_tensor *src[GGML_MAX_SRC];
    struct ggml_tensor *view_src;
    size_t view_offs;
    void *data;
    char name[GGML_MAX_NAME];
    void *extra;
    char padding[8];
};

GGML_API const char *ggml_op_name(enum ggml_op op);
GGML_API const char *ggml_type_name(enum ggml_type type);
GGML_API int64_t ggml_nelements(const struct ggml_tensor *tensor);
GGML_API size_t ggml_nbytes(const struct ggml_tensor *tensor);
GGML_API bool ggml_guid_matches(ggml_guid_t guid_a, ggml_guid_t guid_b);
GGML_API int ggml_graph_n_nodes(struct ggml_cgraph *cgraph);
GGML_API struct ggml_tensor *ggml_graph_node(struct ggml_cgraph *cgraph, int i);

#ifdef __cplusplus
}
#endif
