// ggml-mi355x.h — public header of the MI355X K-quant ggml backend, the sibling of
// ggml/include/ggml-cpu.h / ggml-cuda.h [U] in llama.cpp's tree.
//
// The backend is registered like every ggml backend: ggml_backend_mi355x_reg() is added
// to ggml-backend-reg.cpp's registry (or the library is loaded dynamically through
// GGML_BACKEND_DL_IMPL's ggml_backend_init), and llama.cpp's scheduler then hands it the
// graph splits whose nodes its device's supports_op accepts (ggml-backend.cpp:1553 ->
// iface.graph_compute, README.md:162-163).
#pragma once

#include "ggml-backend.h"

#ifdef __cplusplus
extern "C" {
#endif

// the registry entry: one device per gfx950 GPU the library runs on
GGML_BACKEND_API ggml_backend_reg_t ggml_backend_mi355x_reg(void);
// a backend (one HIP stream) on device `device`; NULL when it does not exist
GGML_BACKEND_API ggml_backend_t ggml_backend_mi355x_init(int device);
GGML_BACKEND_API bool ggml_backend_is_mi355x(ggml_backend_t backend);
// device buffer type (weights and compute buffers live in device memory, GGUF bytes
// unchanged: no repack)
GGML_BACKEND_API ggml_backend_buffer_type_t ggml_backend_mi355x_buffer_type(int device);
GGML_BACKEND_API int ggml_backend_mi355x_get_device_count(void);

#ifdef __cplusplus
}
#endif
