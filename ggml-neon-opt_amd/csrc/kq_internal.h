// kq_internal.h — host-side helpers shared by the C-ABI (kq_api.hip) and the
// backend mirror (kq_backend.hip). Not part of the public ABI.
#pragma once

#include "kq_common.h"

namespace kq {

int device_ok();
int num_cus();
int choose_ncol(int64_t M, int nb);
int plan_gemv(const mi355x_gemv_desc *d, int n_desc, int64_t K, int64_t M, int ncol, GemvArgs &a, dim3 &grid,
              size_t &lds, int &tmask);
int launch_gemv(const GemvArgs &a, dim3 grid, size_t lds, int ncol, bool fusedq, bool debug, int tmask,
                hipStream_t stream);
int launch_quantize(const float *x, int64_t x_stride_floats, void *y, int64_t k, int64_t nrows,
                    hipStream_t stream);

}  // namespace kq
