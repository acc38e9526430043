// kq_internal.h — host-side helpers shared by the C-ABI (kq_api.hip) and the
// backend mirror (kq_backend.hip). Not part of the public ABI.
#pragma once

#include <string>

#include "kq_common.h"

namespace kq {

int device_ok();
bool timing_slot(hipStream_t s, hipEvent_t &a, hipEvent_t &b);
void timing_log(const std::string &kernel, double bytes, hipEvent_t a, hipEvent_t b);
int num_cus();
int choose_ncol(int64_t M, int nb);
typedef void (*gemv_fn)(const GemvArgs);
struct GemvPlan {
    GemvArgs a;
    dim3 grid;
    size_t lds;
    gemv_fn fn;
    int ncol, tmask;
    bool fusedq, debug;
};
int plan_gemv(const mi355x_gemv_desc *d, int n_desc, int64_t K, int64_t M, int ncol, bool fusedq, bool debug,
              GemvPlan &pl);
int launch_gemv(const GemvPlan &pl, hipStream_t stream);
typedef void (*rows_fn)(const RowsArgs);
struct RowsPlan {
    RowsArgs a;
    dim3 grid;
    size_t lds;
    rows_fn fn;
    int tmask;
    bool fusedq;
    int nwv;  // waves per workgroup (one workgroup per CU): ROWS_WAVES, or ROWS_WAVES_SMALL
    bool dyn = false;  // kq_rows_dyn: rows claimed from a per-workgroup counter
};
// Row-stream decode GEMV (kq_rows): returns MI355X_E_UNSUPPORTED when the rows are
// not contiguous or not aligned for it (callers then use kq_gemv). waves_per_cu = 0:
// ROWS_WAVES_SMALL waves per workgroup for launches under kRowsSmallBytes of weights,
// ROWS_WAVES otherwise.
int plan_rows(const mi355x_gemv_desc *d, int n_desc, int64_t K, bool fusedq, RowsPlan &pl,
              int waves_per_cu = 0);
int launch_rows(const RowsPlan &pl, hipStream_t stream);
bool rows_enabled();
int launch_quantize(const float *x, int64_t x_stride_floats, void *y, int64_t k, int64_t nrows,
                    hipStream_t stream);
int gemv_m1(const mi355x_gemv_desc *d, int n, const float *x, int64_t k, void *ws, size_t ws_size,
            hipStream_t stream, const mi355x_gemv_ext *ext = nullptr);
// kq_ops.hip
int launch_rms_norm(const float *x, const float *w, float *y, int64_t n, int64_t nrows, float eps, hipStream_t s);
int launch_binary(int op, const float *a, const float *b, float *y, int64_t n, hipStream_t s,
                  int64_t nb = 0);  // 0 add, 1 mul; b of nb elements repeated (0: nb = n)
int launch_attn_prompt(const AttnArgs &a, int n_tok, hipStream_t s);
int attn_cells_reserve(const AttnArgs &a, hipStream_t stream);  // long-cache attention workspace (per stream), before any capture
bool attn_prompt_q8_ok(const AttnArgs &a);  // the group kernel can write a.q8_out
// prefill (ne11 >= 16) pieces, for the backend's shared-activation runs
bool mmq_applies(int type, const void *w, int64_t N, size_t row_stride, int64_t M);
int launch_quantize_q8L(const float *x, int64_t x_stride_floats, void *y, int64_t k, int64_t nrows,
                        hipStream_t stream, bool mmq = false);  // mmq: the prefill GEMMs' Q8L/mmq layout
int launch_mmq(int type, const void *w, int64_t K, int64_t N, size_t row_stride, const uint8_t *xq, int64_t M,
               float *y, int64_t y_col_stride, hipStream_t stream, const float *res = nullptr,
               int64_t res_col_stride = 0);  // res: ADD epilogue
bool mmq_tile64(int type, int64_t N, int64_t M);  // launch_mmq would use the 64 x 64 tile kernel
// f16 prefill path (mi355x_prefill_precision F16, csrc/kq_mmf.hip): the activation image
// (kq_quantize_f16img) at the workspace start, then the GEMM (its split-K slabs after the
// image); res: ADD epilogue
bool mmf_on();
bool mmf_applies(int type, const void *w, int64_t N, size_t row_stride, int64_t M, int64_t K);  // + mmf_prefers
bool mmf_prefers(int type, int64_t N, int64_t K);  // the f16 kernel is the faster one at this shape
int launch_f16img(const float *x, int64_t x_stride_floats, uint8_t *ws, int64_t K, int64_t M, hipStream_t stream);
int launch_mmf_gemm(int type, const void *w, int64_t K, int64_t N, size_t row_stride, uint8_t *ws, int64_t M,
                    float *y, int64_t y_col_stride, hipStream_t stream, const float *res = nullptr,
                    int64_t res_col_stride = 0);
// up to 4 matrices of one type on the image in one launch (split-K slabs only where they
// fit ws_size)
int launch_mmf_multi(int type, int n_mat, const void *const *w, const int64_t *N, const size_t *row_stride,
                     float *const *y, const int64_t *y_col_stride, int64_t K, uint8_t *ws, size_t ws_size, int64_t M,
                     hipStream_t stream, const float *res = nullptr, int64_t res_col_stride = 0);
// KV-cache store epilogue of launch_mmq_multi (a prompt's k / v projections): kind[d] 1 k,
// 2 v, 0 none; the cells of kq_kv_store (rope(k) -> f16 rows, v -> f16 transposed)
struct MmqKv {
    int kind[4];
    const int32_t *pos;
    const float *rope;
    uint16_t *k_cache, *v_cache;
    int n_ctx, hd;
};
int launch_mmq_multi(const int *types, int n_mat, const void *const *w, const int64_t *N, const size_t *row_stride,
                     float *const *y, const int64_t *y_col_stride, int64_t K, const uint8_t *xq, int64_t M,
                     hipStream_t stream, const MmqKv *kv = nullptr);  // types: Q4_K/Q6_K may mix (kq_mmq_mixed)
// prefill prologues: rms_norm(x) * w -> Q8L, swiglu(g, u) -> Q8L (nrows rows of n)
int launch_rms_norm_q8L(const float *x, const float *w, void *yq, int64_t n, int64_t nrows, float eps, hipStream_t s);
int launch_swiglu_q8L(const float *g, const float *u, void *yq, int64_t n, int64_t nrows, hipStream_t s);
int launch_swiglu(const float *g, const float *u, float *y, int64_t n, hipStream_t s);
int attn_args_from(const mi355x_attn_desc *d, AttnArgs &a);  // + check_attn
int launch_attn(const AttnArgs &a, hipStream_t s);
bool attn_group_ok(const AttnArgs &a, int nwaves);      // the one-workgroup-per-kv-group path applies
size_t attn_group_bytes(const AttnArgs &a, int nwaves);  // its LDS
// kq_attn_oproj.hip: decode attention + the o-proj GEMV (+ residual ADD) in one launch.
// attn_oproj_buffer: bytes of the device buffer it needs (arrival counters, zeroed once,
// then the records), 0 when the shape is not supported; *nsb: the superblocks of K.
constexpr size_t kAttnOprojCounterBytes = 1024;
constexpr int kAttnOprojMaxCtx = 256;  // kq_attn_oproj fuses caches of at most this many cells
size_t attn_oproj_buffer(int hd, int n_head, int n_head_kv, int n_ctx, int type, int64_t K, int64_t n_rows, int *nsb);
int launch_attn_oproj(const AttnArgs &a, int type, const void *w, int64_t n_rows, size_t row_stride, const float *res,
                      float *y, uint8_t *buf, size_t buf_size, hipStream_t stream);
int attn_impl();  // mi355x_attn_impl (kq_ops.hip)
size_t attn_lds16(int hd, int n_ctx);  // attn_head's LDS per head, 16-B multiple (kq_attn_oproj.hip)
// kq_layer.hip: one decode layer as one persistent launch. The caller fills E, F, nq, nkv,
// type / w, y, x, the norms, eps, att / x1 / h / x2, at (rope_row 1), sync, err; layer_plan
// checks the shape and fills the rest (grid, attention placement, ring depth, LDS layout).
int layer_plan(LayerArgs &a, int hd, int n_head);
int launch_layer(const LayerArgs &a, hipStream_t stream);
int64_t layer_table_stride(const LayerArgs &a);                  // bytes per workgroup's step lists (-1: too long)
void layer_table_fill(const LayerArgs &a, uint8_t *buf, int64_t stride);  // G tables (host memory)
uint64_t *diag_stamps(int64_t *cap);  // mi355x_diag_stamps' buffer (diagnostic builds)
// kq_api.hip
void allow_lds(const void *fn, size_t lds);
// Experiment / diagnostic knobs of A/B runs. The product reads no environment: a knob
// holds its product default until mi355x_debug_knob() sets it (tools only), and every
// knob that changes a launch plan bumps knob_generation() (part of the graph key).
enum Knob {
    KNOB_GEMV_DIAG,        // timing stops of the KQ_ROWS_DIAG / KQ_GEMV_DIAG builds
    KNOB_GEMV_RING,        // kq_gemv ring depth override (0: by LDS)
    KNOB_GEMV_PRE0,        // kq_rows weight steps issued before the activation (1)
    KNOB_GEMV_PF,          // kq_rows L2 prefetch of the stream (experiment builds)
    KNOB_GEMV_XMODE,       // kq_rows prologue variants (experiment builds)
    KNOB_GEMV_SMALL_MB,    // launches below this many MB of weights: ROWS_WAVES_SMALL waves
    KNOB_GEMV_WPC,         // cap on active waves per CU (0: none)
    KNOB_GEMV_SMALL_WG,    // cap on workgroups of small launches (0: one per CU)
    KNOB_GEMV_FQMAX,       // most superblocks quantized inside kq_rows
    KNOB_MMF_WAVES,        // kq_mmf waves per workgroup (0: by K)
    KNOB_MMF_ORDER,        // kq_mmf tile order
    KNOB_ATTN_DIAG,        // timing stops of the KQ_ATTN_DIAG build
    KNOB_LOOPBACK_NOCOPY,  // emulated ALL_GATHERs skip their own-slice copy (timing only)
    KNOB_ATTN_OPROJ,       // attention + o-proj fusion: 1 per backend (set_attn_oproj), 0 never, 2 always (A/B)
    KNOB_AO_NRB,           // kq_attn_oproj row blocks (0: by shape)
    KNOB_GEMV_DYN,         // kq_rows_dyn when a wave gets at least this many units (and 16 steps) on average (0: never)
    KNOB_GEMV_DYN_P,       // kq_rows_dyn: static units per wave (0: a ring's worth; A/B only)
    KNOB_GEMV_DYN_STEPS,   // kq_rows_dyn AUTO: 16-superblock steps per wave at least (with GEMV_DYN units)
    KNOB_COUNT
};
double knob(Knob k);
uint32_t knob_generation();
// Process-wide kernel selectors a captured launch plan depends on (gemv impl / waves,
// mmq impl; attention decode / prompt impl), packed for the backend's graph key.
uint64_t api_selector_key();
uint64_t ops_selector_key();

}  // namespace kq
