// Restated SUBSET of ggml/include/ggml-backend.h at llama.cpp a3cb0474 [U] (test
// infrastructure; see ggml.h here): the handle types, device type / props and the
// few public calls adapter/ggml-mi355x.cpp makes.
#pragma once

#include "ggml.h"

#define GGML_BACKEND_API __attribute__((visibility("default")))

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ggml_backend_buffer_type *ggml_backend_buffer_type_t;
typedef struct ggml_backend_buffer *ggml_backend_buffer_t;
typedef struct ggml_backend_event *ggml_backend_event_t;
typedef struct ggml_backend *ggml_backend_t;
typedef void *ggml_backend_graph_plan_t;
typedef struct ggml_backend_reg *ggml_backend_reg_t;
typedef struct ggml_backend_device *ggml_backend_dev_t;

enum ggml_backend_buffer_usage {
    GGML_BACKEND_BUFFER_USAGE_ANY = 0,
    GGML_BACKEND_BUFFER_USAGE_WEIGHTS = 1,
    GGML_BACKEND_BUFFER_USAGE_COMPUTE = 2,
};

enum ggml_backend_dev_type {
    GGML_BACKEND_DEVICE_TYPE_CPU,
    GGML_BACKEND_DEVICE_TYPE_GPU,
    GGML_BACKEND_DEVICE_TYPE_IGPU,
    GGML_BACKEND_DEVICE_TYPE_ACCEL,
};

struct ggml_backend_dev_caps {
    bool async;
    bool host_buffer;
    bool buffer_from_host_ptr;
    bool events;
};

struct ggml_backend_dev_props {
    const char *name;
    const char *description;
    size_t memory_free;
    size_t memory_total;
    enum ggml_backend_dev_type type;
    const char *device_id;
    struct ggml_backend_dev_caps caps;
};

GGML_API void *ggml_backend_buffer_get_base(ggml_backend_buffer_t buffer);
GGML_API size_t ggml_backend_buffer_get_size(ggml_backend_buffer_t buffer);

#ifdef __cplusplus
}
#endif
