/*
 * ggml_mi355x.h — C-ABI of the MI355X (gfx950) K-quant mat-vec / mat-mat hot path.
 *
 * This is the drop-in boundary for ggml's quantized MUL_MAT path
 * (ggml_compute_forward_mul_mat -> type_traits_cpu[src0].vec_dot, here
 * ggml_vec_dot_q4_K_q8_K). Every entry point is plain C: pointers, sizes,
 * an opaque HIP stream handle (hipStream_t passed as void*, NULL = default
 * stream). No torch or C++ types cross this boundary.
 *
 * Reference interfaces replaced (file:line in /root/reference, which quotes the
 * un-vendored llama.cpp @ a3cb0474):
 *   - ggml_vec_dot_t               README.md:449, :686  (ggml-cpu/arch/arm/quants.c:2059)
 *   - quantize_row_q8_K(_ref)      artifacts/perf/out.folded:184-186
 *   - ggml_compute_forward_mul_mat README.md:137, :157  (ggml-cpu.c:1389, one_chunk :1194)
 *   - ggml_backend_cpu_graph_compute README.md:162      (ggml-cpu.cpp:186) -> mi355x_backend_graph_compute
 *
 * Memory: every data pointer below is DEVICE memory (hipMalloc / torch cuda
 * tensor) unless stated otherwise. Weight blocks are stored exactly as GGUF /
 * ggml stores them (no repack): rows of contiguous superblocks.
 *
 * Errors: functions returning int return 0 on success, a negative
 * MI355X_E* code for argument errors, or a positive hipError_t value. The
 * ggml-surface mirrors that return void (vec_dot, from_float) abort with a
 * message on invalid arguments, as GGML_ASSERT does upstream.
 */
#ifndef GGML_MI355X_H
#define GGML_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ formats */
/* Super-block size and block layouts: identical to ggml-common.h. Offsets
 * are proven by the reference disassembly: block_q4_K stride 0x90
 * (README.md:460, :611), d @0 (:529 "[x7,#-144]"), dmin @2 (:507), scales @4
 * (:472 "#-140", :488 "#-132"), qs @16 (:480 "x7-0x80"); block_q8_K stride 0x124
 * (:610), d @0 (:522), qs @4 (:459), bsums @260 (:492 "[x11,#256]"). */
#define MI355X_QK_K 256
#define MI355X_K_SCALE_SIZE 12

typedef uint16_t mi355x_half; /* IEEE binary16 bits (ggml_half) */

typedef struct {
    mi355x_half d;                       /* super-block scale for quantized scales */
    mi355x_half dmin;                    /* super-block scale for quantized mins   */
    uint8_t scales[MI355X_K_SCALE_SIZE]; /* 8 x 6-bit scales + 8 x 6-bit mins      */
    uint8_t qs[MI355X_QK_K / 2];         /* 4-bit quants                           */
} mi355x_block_q4_K;                     /* 144 bytes, 4.5 bpw */

typedef struct {
    mi355x_half d;
    mi355x_half dmin;
    uint8_t scales[MI355X_K_SCALE_SIZE];
    uint8_t qh[MI355X_QK_K / 8];         /* 5th bit of each quant */
    uint8_t qs[MI355X_QK_K / 2];         /* low 4 bits            */
} mi355x_block_q5_K;                     /* 176 bytes, 5.5 bpw */

typedef struct {
    uint8_t ql[MI355X_QK_K / 2];         /* low 4 bits             */
    uint8_t qh[MI355X_QK_K / 4];         /* high 2 bits            */
    int8_t scales[MI355X_QK_K / 16];     /* 8-bit sub-block scales */
    mi355x_half d;                       /* super-block scale      */
} mi355x_block_q6_K;                     /* 210 bytes, 6.5625 bpw */

typedef struct {
    float d;                             /* delta (negative when the block max is positive) */
    int8_t qs[MI355X_QK_K];              /* quants                                          */
    int16_t bsums[MI355X_QK_K / 16];     /* sums of 16 consecutive quants                    */
} mi355x_block_q8_K;                     /* 292 bytes */

/* ggml_type values (ggml.h enum ggml_type) for the types this path handles. */
enum mi355x_type {
    MI355X_TYPE_F32  = 0,
    MI355X_TYPE_F16  = 1,
    MI355X_TYPE_Q4_K = 12,
    MI355X_TYPE_Q5_K = 13,
    MI355X_TYPE_Q6_K = 14,
    MI355X_TYPE_Q8_K = 15,
    MI355X_TYPE_I32  = 26,
};

enum mi355x_status {
    MI355X_OK           = 0,
    MI355X_E_INVAL      = -1,  /* bad shape / stride / type                    */
    MI355X_E_UNSUPPORTED = -2, /* combination not implemented on this device   */
    MI355X_E_WORKSPACE  = -3,  /* workspace missing or too small               */
    MI355X_E_NODEVICE   = -4,  /* no gfx950 device / HIP runtime unavailable   */
    MI355X_E_COMM       = -6,  /* RCCL missing / communicator error            */
    MI355X_E_LAYER      = -7,  /* a persistent-layer launch lost co-residency:
                                  that step's outputs are invalid (re-armed)   */
};

/* Bytes of one row of `type` with `k` elements (ggml_row_size). k % 256 == 0. */
size_t mi355x_row_size(int type, int64_t k);

/* Library / kernel-object identification (for logs and tests). */
const char *mi355x_version(void);
/* 1 when a gfx950 device is visible and the code object loads, else 0. */
int mi355x_device_available(void);

/* ------------------------------------------------ ggml operator surface */
/* Device mirror of ggml_from_float_t for GGML_TYPE_Q8_K
 * (type_traits_cpu[Q8_K].from_float = quantize_row_q8_K -> quantize_row_q8_K_ref).
 * x: k floats, y: k/256 block_q8_K. Bit-exact with the reference
 * (aarch64 build: iscale*x + 12582912.f contracted to one fma). x and y may be host
 * or device pointers (ggml-cpu passes src1 rows and params->wdata); runs on the
 * calling thread's own stream and returns after it completes (reentrant, see the
 * vec_dot entries below). Aborts if k % 256 != 0, as GGML_ASSERT does. */
void mi355x_quantize_row_q8_K(const float *x, void *y, int64_t k);

/* Device mirror of ggml_vec_dot_t for Q4_K x Q8_K / Q5_K x Q8_K / Q6_K x Q8_K
 * (README.md:449: void (int n, float *s, size_t bs, const void *vx, size_t bx,
 * const void *vy, size_t by, int nrc)). n % 256 == 0, nrc == 1 (the measured
 * reference configuration: no I8MM, README.md:677, so nrows == 1); bs/bx/by are
 * unused exactly as upstream. s, vx, vy may be host pointers (ggml-cpu's src0 rows and
 * params->wdata, as type_traits_cpu[type].vec_dot is called from mul_mat_one_chunk)
 * or device pointers, in any mix. Reentrant: every calling thread uses its own HIP
 * stream and staging buffer on its current device (ggml's nth threads call it at once,
 * README.md:125-131), and the call returns after that stream completes (no default-
 * stream synchronization). The Q4_K result is bit-identical to the reference NEON
 * function's fp32 output (README.md:725-777, fmsub :551, fmadd :614). */
void mi355x_vec_dot_q4_K_q8_K(int n, float *s, size_t bs, const void *vx, size_t bx,
                              const void *vy, size_t by, int nrc);
void mi355x_vec_dot_q5_K_q8_K(int n, float *s, size_t bs, const void *vx, size_t bx,
                              const void *vy, size_t by, int nrc);
void mi355x_vec_dot_q6_K_q8_K(int n, float *s, size_t bs, const void *vx, size_t bx,
                              const void *vy, size_t by, int nrc);

/* ----------------------------------------------------- stream-level API */
/* Quantize `nrows` f32 rows of k elements (row stride x_stride bytes) into
 * contiguous Q8_K rows (k/256 blocks each). Async on `stream`. */
int mi355x_quantize_q8_K(const float *x, size_t x_stride, void *y, int64_t k, int64_t nrows,
                         void *stream);

/* MUL_MAT for src0 in {Q4_K, Q5_K, Q6_K}: dst[N x M] = src0[N x K] . src1[K x M]
 * with ggml conventions: src0 row i at src0 + i*nb01 (ne00 = K, ne01 = N);
 * src1 column j (ggml row j of src1) at src1 + j*nb11, K floats; dst column j at
 * dst + j*nb1, N floats. Semantics = ggml_compute_forward_mul_mat: src1 is first
 * quantized to Q8_K (bit-exact), then every dst element is vec_dot(row, col).
 * M == 1 with K <= 8192 quantizes inside the GEMV kernel (no workspace); other
 * shapes need a workspace of mi355x_mul_mat_workspace_size() bytes (the Q8_K
 * copy of src1). Async on `stream`. */
size_t mi355x_mul_mat_workspace_size(int src0_type, int64_t ne00, int64_t ne01, int64_t ne11);
int mi355x_mul_mat(int src0_type, const void *src0, int64_t ne00, int64_t ne01, size_t nb01,
                   const float *src1, int64_t ne11, size_t nb11,
                   float *dst, size_t nb1,
                   void *workspace, size_t workspace_size, void *stream);

/* Same, with src1 already quantized to Q8_K rows (vec_dot_type), each
 * ne00/256 blocks, column j at src1_q8 + j*nb11. No workspace. */
int mi355x_mul_mat_q8(int src0_type, const void *src0, int64_t ne00, int64_t ne01, size_t nb01,
                      const void *src1_q8, int64_t ne11, size_t nb11,
                      float *dst, size_t nb1, void *stream);

/* Fused decode GEMV over up to MI355X_MAX_FUSED matrices that share one f32
 * input vector x (K floats): e.g. attn_q/attn_k/attn_v, or ffn_gate/ffn_up.
 * Each matrix may have its own K-quant type. Equivalent to n separate
 * mi355x_mul_mat calls with ne11 == 1 (bit-identical results). For K <= 8192
 * x is quantized inside the GEMV (each wave quantizes its own K-range into LDS,
 * one launch, no workspace); above that x is first quantized into `workspace`
 * (mi355x_gemv_fused_workspace_size(k) bytes; 0 means none needed). */
#define MI355X_MAX_FUSED 4
typedef struct {
    int type;            /* MI355X_TYPE_Q4_K / Q5_K / Q6_K */
    const void *w;       /* device: N rows of K/256 blocks  */
    int64_t n_rows;      /* N                                */
    size_t row_stride;   /* nb01 in bytes                    */
    float *y;            /* device: N floats                 */
} mi355x_gemv_desc;
size_t mi355x_gemv_fused_workspace_size(int64_t k);
int mi355x_gemv_fused(const mi355x_gemv_desc *descs, int n_desc, const float *x, int64_t k,
                      void *workspace, size_t workspace_size, void *stream);

/* mi355x_gemv_fused with the decode graph's neighbours of the MUL_MATs fused in
 * (the backend's node fusion uses this): `prologue` transforms x before its Q8_K
 * quantization exactly as the separate node would (MI355X_PRO_RMS_NORM: ggml_rms_norm
 * then ggml_mul by x2 = the norm weight; MI355X_PRO_SWIGLU: x = gate, x2 = up), and
 * descs[i].y receives mul_mat + residual[i] when residual[i] != NULL (ggml_add).
 * Bit-identical to the separate ops. Workspace: mi355x_gemv_ext_workspace_size(k)
 * (used only when the kernel cannot fuse, e.g. rows not contiguous). */
#define MI355X_PRO_NONE 0
#define MI355X_PRO_RMS_NORM 1
#define MI355X_PRO_SWIGLU 2
/* `epilogue` MI355X_EPI_SWIGLU: descs[0] = gate, descs[1] = up (n_desc == 2, equal
 * n_rows, no residual); epi_y[r] = ggml_vec_swiglu_f32(gate, up)[r] is written besides
 * descs[i].y — the GGML_GLU(SWIGLU) node that follows the gate/up MUL_MATs. */
#define MI355X_EPI_NONE 0
#define MI355X_EPI_SWIGLU 1
typedef struct {
    int prologue;
    const float *x2;
    float eps;
    const float *residual[MI355X_MAX_FUSED];
    int epilogue;
    float *epi_y;
} mi355x_gemv_ext;
size_t mi355x_gemv_ext_workspace_size(int64_t k);
int mi355x_gemv_fused_ext(const mi355x_gemv_desc *descs, int n_desc, const float *x, int64_t k,
                          const mi355x_gemv_ext *ext, void *workspace, size_t workspace_size, void *stream);

/* Debug/parity hook: per-superblock integer partials of a Q4_K/Q5_K/Q6_K x Q8_K
 * dot, as the GEMV kernel computes them. For each row r and superblock b:
 * out[2*(r*nb+b)+0] = sumi (sum_j sc_j * dot_j), out[...+1] = summins
 * (sum_g bsums_g * m_{g/2}; for Q6_K: sum_g bsums_g * sc_g). Device pointers. */
/* Diagnostic (no reference counterpart): the streaming ceiling of one launch -- the
 * buffer's first `bytes` (rounded down to whole 2-KB steps of 12 waves per CU) pulled into
 * LDS by non-temporal LDS-DMA, no arithmetic, on `stream`. The time a decode GEMV of that
 * many weight bytes could approach; bench.py's gemv_large "stream_us". buf 16-B aligned,
 * sink >= 4 device bytes. */
int mi355x_debug_stream(const void *buf, size_t bytes, void *sink, void *stream);
int mi355x_debug_block_partials(int src0_type, const void *src0, int64_t ne00, int64_t ne01,
                                size_t nb01, const void *src1_q8, int32_t *out, void *stream);

/* ------------------------------------------------------------ profiling */
/* Per-launch kernel timing. While enabled, every GEMV/quantize launch made
 * outside a stream capture goes through hipExtLaunchKernelGGL with a start and
 * a stop event (the kernel's own begin/end timestamps, as rocprofv3's kernel
 * trace reports them) and is logged with its kernel name and ALGORITHMIC bytes
 * (weights + f32/Q8_K activations read + f32 outputs written).
 * mi355x_timing_enable(1) clears the log; mi355x_timing_read synchronizes the
 * device and copies up to `max` entries, returning the number logged. */
typedef struct {
    char kernel[96];
    double bytes;
    float ms;
} mi355x_launch_timing;
int mi355x_timing_enable(int enable);
int mi355x_timing_read(mi355x_launch_timing *out, int max);
/* Diagnostics: while `buf` (device memory, `bytes` long) is set, GEMV launches
 * record per-wave s_memrealtime stamps (100 MHz) at kernel entry, after the
 * activation prologue, after the main loop and at exit, then after the first
 * task lookup, after the prologue DMAs are issued and after their wait:
 * 8 x uint64 per wave, [(blockIdx.x * 4 + wave) * 8 + i]. NULL disables. */
int mi355x_diag_stamps(void *buf, size_t bytes);
/* Decode-GEMV implementation selector (A/B runs, parity of every path):
 * MI355X_GEMV_AUTO (row-stream kq_rows when rows are contiguous, else kq_gemv; the
 * claimed-row form kq_rows_dyn for one-type launches with enough rows per wave),
 * MI355X_GEMV_TASKS (always the 8-row-task kq_gemv), MI355X_GEMV_ROWS (kq_rows, one
 * launch per stage; as AUTO) or MI355X_GEMV_DYN (kq_rows_dyn for every one-type
 * launch: rows claimed per workgroup from an LDS counter). Same numerics in all.
 * Returns the previous value, or MI355X_E_INVAL. */
#define MI355X_GEMV_AUTO 0
#define MI355X_GEMV_TASKS 1
#define MI355X_GEMV_ROWS 2
#define MI355X_GEMV_DYN 3
int mi355x_gemv_impl(int impl);
/* Prefill (ne11 >= 16) GEMM selector for the int8-MFMA tile kernel: MI355X_MMQ_TILE64
 * (64 weight rows x 64 activation columns per workgroup), MI355X_MMQ_TILE128 (128 rows x
 * 64 columns, 8 waves: the activation tile fetched once per 128 rows), MI355X_MMQ_TILE128W
 * (128 rows x 128 columns: each wave's weight operands feed two MFMA column tiles) or
 * MI355X_MMQ_AUTO (the library's choice by shape). Same numerics in all. Returns the
 * previous value, or MI355X_E_INVAL. */
#define MI355X_MMQ_AUTO 0
#define MI355X_MMQ_TILE64 1
#define MI355X_MMQ_TILE128 2
#define MI355X_MMQ_TILE128W 3
#define MI355X_MMQ_TILE64W 4 /* 64 rows x 128 columns, 4 waves (two column tiles per wave) */
#define MI355X_MMQ_TILE128X 5 /* 128 rows x 128 columns, 4 waves (each wave 32 rows x all 128 columns,
                                 one wave per SIMD); Q4_K / Q5_K (Q6_K takes TILE128W) */
#define MI355X_MMQ_TILE192 6 /* 192 rows x 64 columns, 12 waves (three per SIMD); Q4_K / Q5_K (Q6_K takes TILE128) */
int mi355x_mmq_impl(int impl);
/* Prefill (ne11 >= 16) precision: MI355X_PREFILL_EXACT (kq_mmq, int8 MFMA, bit-exact
 * against ggml's per-(row, column) vec_dot loop; the default), MI355X_PREFILL_F16 (within
 * a stated tolerance: kq_mmf -- the same Q8_K activation quantization and integer
 * unpacking, the accumulated dot on the f16 matrix core, csrc/kq_mmf.hip -- on the shapes
 * where it is the faster kernel, kq_mmq elsewhere) or MI355X_PREFILL_F16_ALL (kq_mmf on
 * every shape; A/B and tests). The north_star's "within a stated fp32 tolerance on the
 * accumulated dot". Replaces no reference interface (ggml-cpu has one precision); a
 * backend option like llama.cpp's GGML_CUDA_FORCE_MMQ / cuBLAS choice. A negative value
 * queries. The library reads no environment: the precision changes only through this
 * call (process-wide; a graph captured before it is re-planned, and a caller sizing its
 * workspace with mi355x_mul_mat_workspace_size must query it again after switching to
 * F16). Returns the previous value, or MI355X_E_INVAL. */
#define MI355X_PREFILL_EXACT 0
#define MI355X_PREFILL_F16 1
#define MI355X_PREFILL_F16_ALL 2
int mi355x_prefill_precision(int precision);
/* Decode GEMV (kq_rows) waves per workgroup (A/B runs, parity of both launch shapes):
 * 0 = by launch size (6 waves under 10 MB of weights, else 12; the debug knob
 * "GEMV_SMALL_MB" moves the threshold), or a fixed count 1..12 where the launch allows it (the in-kernel
 * quantization covers 12 superblocks per wave). Returns the previous value, or
 * MI355X_E_INVAL. */
int mi355x_gemv_waves(int waves);
/* Experiment / diagnostic knobs of A/B runs and timing tools (replaces no reference
 * interface). The library reads no environment variable; every knob holds its product
 * default until set here, process-wide: "GEMV_DIAG", "GEMV_RING", "GEMV_PRE0",
 * "GEMV_PF", "GEMV_XMODE", "GEMV_SMALL_MB", "GEMV_WPC", "GEMV_SMALL_WG", "GEMV_FQMAX",
 * "MMF_WAVES", "MMF_ORDER", "ATTN_DIAG", "LOOPBACK_NOCOPY", "ATTN_OPROJ", "AO_NRB"
 * (csrc/kq_internal.h). None changes numerics: the DIAG knobs act only in the diagnostic
 * builds (make variant), the others move launch shapes of bit-exact kernels (ATTN_OPROJ: 1
 * each backend's mi355x_backend_set_attn_oproj, 0 never, 2 in every backend), and LOOPBACK_NOCOPY (timing only)
 * leaves emulated all-gathers stale. value NaN restores the default; *previous (may be
 * NULL) receives the value in force before. 0, or MI355X_E_INVAL for an unknown name. */
int mi355x_debug_knob(const char *name, double value, double *previous);

/* --------------------------------------- decode ops of the llama graph (§8f) */
/* The non-matmul nodes of one llama decode token (llm_build_llama, out.folded:249),
 * each bit-compatible with the ggml-cpu function the reference profile shows
 * (artifacts/perf/out.folded; restatement and [U] notes: the CPU checker under the tests).
 * Device pointers, async on `stream`, 0 / MI355X_E* / hipError_t like the GEMVs. */

/* GGML_OP_GET_ROWS (ggml_compute_forward_get_rows_q -> dequantize_row_q4_K,
 * out.folded:103-104): dst[r][0..ne0) = row ids[r] of `table` as f32. type F32 /
 * Q4_K / Q5_K / Q6_K; `n_rows` rows (ne01) of `row_stride` bytes; ids: device int32[n_ids].
 * An id outside [0, n_rows) (ggml: GGML_ASSERT(i01 >= 0 && i01 < ne01)) reads nothing
 * and writes a NaN row. */
int mi355x_get_rows(int type, const void *table, int64_t ne0, size_t row_stride, int64_t n_rows,
                    const int32_t *ids, int64_t n_ids, float *dst, void *stream);
/* GGML_OP_RMS_NORM (ggml_compute_forward_rms_norm_f32, out.folded:189-193) over
 * `nrows` rows of n floats, y = x * (1/sqrtf(mean(x^2) + eps)); when w != NULL the
 * following GGML_OP_MUL by the norm weight is fused: y = (x*scale) * w (two roundings,
 * as the two ops). n % 256 == 0. */
int mi355x_rms_norm(const float *x, const float *w, float *y, int64_t n, int64_t nrows, float eps, void *stream);
/* GGML_OP_ADD / GGML_OP_MUL on contiguous f32 (binary_op<op_add/op_mul>, out.folded:91-99, 115-121). */
int mi355x_add(const float *a, const float *b, float *y, int64_t n, void *stream);
int mi355x_mul(const float *a, const float *b, float *y, int64_t n, void *stream);
/* GGML_OP_GLU / GLU_OP_SWIGLU split form (ggml_vec_swiglu_f32, out.folded:107-113):
 * y = silu(gate) * up with ggml_v_silu/ggml_v_expf arithmetic. */
int mi355x_swiglu(const float *gate, const float *up, float *y, int64_t n, void *stream);
/* GGML_OP_ROPE, mode NORMAL, ext_factor 0, attn_factor 1 (ggml_compute_forward_rope_f32,
 * ggml_rope_cache_init, rope_yarn; out.folded:196-208). The per-position cos/sin cache
 * ggml builds on every call is built once for positions [0, n_pos) by the host C
 * library (powf, cosf, sinf: the calls of the CPU path) into a device table of
 * mi355x_rope_table_size() bytes. pos: device int32 (one token). */
size_t mi355x_rope_table_size(int n_pos, int n_dims);
int mi355x_rope_table(float *table, int n_pos, int n_dims, float freq_base, float freq_scale, void *stream);
int mi355x_rope(const float *x, float *y, int head_dim, int n_dims, int n_heads, const int32_t *pos,
                const float *table, int n_pos, void *stream);
/* The non-flash attention block of a decode token, one launch: rope(q), rope(k) at
 * *pos, f16 K/V cache cell write (set_rows, out.folded:209-215; V transposed),
 * KQ = mul_mat(k_cache f16, q->f16) via ggml_vec_dot_f16 (NEON FP16 accumulation,
 * out.folded:140-144), soft_max_ext(scale, causal mask) (out.folded:216-234), KQV =
 * mul_mat(v_cache, kq->f16), permute + cont -> out[n_head*head_dim]. n_kv =
 * min(n_ctx, max(32, pad32(pos+1))). head_dim 64 or 128; n_ctx % 32 == 0, <= 8192;
 * caches zero-initialised by the caller, 16-B aligned. */
typedef struct {
    const float *q, *k, *v;    /* this token's projections, before rope */
    const int32_t *pos;        /* device int32 */
    const float *rope_table;   /* mi355x_rope_table(n_pos >= n_ctx, n_dims = head_dim) */
    uint16_t *k_cache;         /* f16 [n_ctx][n_head_kv*head_dim] */
    uint16_t *v_cache;         /* f16 [n_head_kv*head_dim][n_ctx] */
    float *out;                /* [n_head*head_dim] */
    int n_ctx, n_head, n_head_kv, head_dim;
    float scale;               /* kq_scale = 1/sqrtf(head_dim) */
    int rope_row;              /* 0: rope_table is the whole table, row *pos read on device;
                                  1: rope_table is already the row of this token's position
                                  (staged by the caller with *pos), read without waiting for pos */
} mi355x_attn_desc;
int mi355x_attn_decode(const mi355x_attn_desc *a, void *stream);
/* Which decode attention kernel mi355x_attn_decode (and the ATTN_DECODE graph node) runs for
 * this descriptor under the current selectors: no launch, no device access (the pointers are
 * only checked and their alignment read). Returns one of the paths below, or a negative
 * MI355X_E_* for a descriptor attn_decode would reject. A captured launch whose workspace was
 * not reserved runs MI355X_ATTN_PATH_HEAD_BATCH in place of MI355X_ATTN_PATH_CELLS. */
#define MI355X_ATTN_PATH_HEAD 0       /* one workgroup per query head, register path (<= 256 cells) */
#define MI355X_ATTN_PATH_HEAD_BATCH 1 /* one workgroup per query head, batched cache loads */
#define MI355X_ATTN_PATH_SPLIT4 2     /* each head split by output over 4 workgroups */
#define MI355X_ATTN_PATH_SPLIT8 3     /* ... over 8 */
#define MI355X_ATTN_PATH_CELLS 4      /* KQ split over cells: kq_attn_cells + kq_attn_cells_kqv */
#define MI355X_ATTN_PATH_GROUP 5      /* one workgroup per KV group (MI355X_ATTN_GROUP) */
#define MI355X_ATTN_PATH_KD1 6        /* experiment builds (KQ_ATTN_KDMA1) */
int mi355x_attn_path(const mi355x_attn_desc *a);
/* The same block for a prompt of n_tokens tokens in one graph (llama-bench pp: ggml's
 * batched non-flash path — SET_ROWS of the batch's cells, then KQ / soft_max with the
 * causal mask / KQV per query): q [n_tokens][n_head*head_dim], k, v [n_tokens][kvw],
 * pos device int32 [n_tokens], out [n_tokens][n_head*head_dim]; rope_row must be 0 (the
 * whole table). All cells are written first, then every query attends to the cells at or
 * before its position: each output row equals mi355x_attn_decode's for that token after
 * the tokens before it, bit for bit. A position outside the cache gives a NaN row and no
 * cell. */
int mi355x_attn_prompt(const mi355x_attn_desc *a, int n_tokens, void *stream);
/* Attention kernel selector (A/B runs, parity of all): MI355X_ATTN_SPLIT (default: one
 * workgroup per query head; for caches past 256 cells each head split over 4 or 8 workgroups
 * by output dimension, where the slice's LDS fits), MI355X_ATTN_HEAD (one workgroup per query
 * head at every cache size) or MI355X_ATTN_GROUP (one workgroup per KV group where its cells
 * fit in LDS: cells [0, n_kv) read once and shared by the group's n_head/n_head_kv query
 * heads, 1/gsz of the cache reads). Returns the previous value, or MI355X_E_INVAL. */
#define MI355X_ATTN_GROUP 0
#define MI355X_ATTN_HEAD 1
#define MI355X_ATTN_SPLIT 2
int mi355x_attn_impl(int impl);
/* Prompt attention selector (A/B runs, parity of both): MI355X_ATTN_GROUP (default: one
 * workgroup per kv group and token, the group's query heads sharing every K/V load, where
 * n_head/n_head_kv <= 8 and its LDS fits) or MI355X_ATTN_HEAD (one per query head and
 * token). Returns the previous value, or MI355X_E_INVAL. */
int mi355x_attn_prompt_impl(int impl);

/* --------------------------------------------- ggml-backend mirror (C++) */
/* A minimal mirror of ggml-backend's device/buffer/graph interface
 * (ggml-backend-impl.h [U]; CPU sibling ggml-cpu.cpp:186, README.md:162),
 * enough for a ggml adapter to forward MUL_MAT nodes. */
/* Node ops: MUL_MAT and the other nodes of a llama decode token (llm_build_llama).
 * Operands (src[i]) and op_params per op:
 *   MUL_MAT      src0 K-quant weights [K, N], src1 f32 [K, M]            -> f32 [N, M]
 *   GET_ROWS     src0 table (F32/Q4_K/Q6_K) [K, rows], src1 I32 ids [n]  -> f32 [K, n]
 *   RMS_NORM     src0 f32 [n, rows]; op_params[0] = eps (float bits)     -> f32
 *   MUL, ADD     src0, src1 f32, same shape (contiguous)                 -> f32
 *   SWIGLU       src0 gate, src1 up (GGML_OP_GLU, GLU_OP_SWIGLU, split)  -> f32
 *   ROPE         src0 f32 [head_dim, n_heads], src1 I32 pos [1], src2 f32 rope table
 *                [n_dims, n_pos] (mi355x_rope_table); op_params[0] = n_dims (mode NORMAL)
 *   ATTN_DECODE  src0 q, src1 k, src2 v (f32, before rope), src3 I32 pos [1],
 *                src4 F16 k_cache [kvw, n_ctx], src5 F16 v_cache [n_ctx, kvw] (transposed),
 *                src6 rope table [head_dim, >= n_ctx], or [head_dim, 1]: the row of this
 *                token's position, staged with pos; op_params = {n_head, n_head_kv, head_dim, scale bits}
 *                -> f32 [head_dim*n_head]: the non-flash attention block
 *                (set_rows, mul_mat f16, soft_max_ext, mul_mat f16, permute, cont).
 *   ALL_GATHER   src0 f32 [n] (this rank's contiguous row slice of a row-split MUL_MAT
 *                chain stage) -> f32 [n * world]: the slices of every rank in rank order,
 *                one RCCL ncclAllGather over xGMI on the backend stream (captured in the
 *                hipGraph). Needs mi355x_backend_set_comm; the exchange step of the
 *                row split (weight rows of one matrix across the GPUs,
 *                the reference's per-thread row split README.md:125-131 across devices).
 *   ALL_REDUCE   src0 f32 [n] (this rank's PARTIAL output of a K-split MUL_MAT: the
 *                reference's fp32 chain over the rank's superblock range of K) -> f32 [n]
 *                the sum over ranks, one RCCL ncclAllReduce(sum) on the backend stream
 *                (captured in the hipGraph). The exchange step of the K-split ("Megatron")
 *                pairing of SURVEY.md §8e: o-proj and ffn_down split along K at 256-element
 *                superblock boundaries, 2 collectives per layer. The sum re-associates the
 *                row's fp32 chain: within SURVEY.md §8c's fp32 bound, not bit-exact. */
enum mi355x_op {
    MI355X_OP_NONE = 0, MI355X_OP_MUL_MAT = 1, MI355X_OP_GET_ROWS = 2, MI355X_OP_RMS_NORM = 3,
    MI355X_OP_MUL = 4, MI355X_OP_ADD = 5, MI355X_OP_SWIGLU = 6, MI355X_OP_ROPE = 7,
    MI355X_OP_ATTN_DECODE = 8, MI355X_OP_ALL_GATHER = 9, MI355X_OP_ALL_REDUCE = 10,
};
#define MI355X_MAX_SRC 8
#define MI355X_TENSOR_FLAG_OUTPUT 1  /* read by the caller after graph_compute: never elided by fusion */

typedef struct mi355x_tensor {
    int type;                      /* enum mi355x_type (+ F16 = 1, I32 = 26)    */
    int op;                        /* enum mi355x_op                            */
    int64_t ne[4];                 /* elements per dim (ggml order)            */
    size_t nb[4];                  /* bytes per dim                            */
    struct mi355x_tensor *src[MI355X_MAX_SRC];
    void *data;                    /* device pointer                            */
    int32_t op_params[8];
    int32_t flags;                 /* MI355X_TENSOR_FLAG_*                      */
} mi355x_tensor;

typedef struct mi355x_backend *mi355x_backend_t;

/* Devices this library runs on (gfx950 with its code object), for the ggml-backend
 * registration's get_device_count (ggml_backend_reg_i [U], ggml-backend-impl.h; the
 * CPU sibling registers one device, ggml-cpu.cpp). 0 without a GPU. */
int mi355x_device_count(void);
/* The HIP ordinal of the i-th device counted by mi355x_device_count (a host may list a
 * non-gfx950 GPU at a lower ordinal): the `device` argument the calls below take; -1 if
 * there is no such device. */
int mi355x_device_ordinal(int i);
/* Free / total device memory (ggml_backend_device_i.get_memory [U]): 0 or an error. */
int mi355x_device_memory(int device, size_t *free_bytes, size_t *total_bytes);
mi355x_backend_t mi355x_backend_init(int device);        /* NULL on failure */
void mi355x_backend_free(mi355x_backend_t backend);
const char *mi355x_backend_name(mi355x_backend_t backend);
void *mi355x_backend_stream(mi355x_backend_t backend);   /* hipStream_t */
void *mi355x_backend_alloc(mi355x_backend_t backend, size_t size); /* device buffer */
void mi355x_backend_free_buffer(mi355x_backend_t backend, void *ptr);
int mi355x_backend_set_tensor(mi355x_backend_t backend, void *dst, const void *host_src,
                              size_t size);              /* async H2D, bytes unchanged */
int mi355x_backend_get_tensor(mi355x_backend_t backend, void *host_dst, const void *src,
                              size_t size);              /* async D2H */
/* async device memset of `size` bytes to (uint8_t)value (ggml_backend_buffer_i.memset_tensor
 * / clear [U]) */
int mi355x_backend_memset(mi355x_backend_t backend, void *dst, int value, size_t size);
/* Waits for the backend stream. With the persistent layer on (set_layer_engine) it also
 * returns MI355X_E_LAYER when a layer launch since the last check gave up waiting for
 * another workgroup (outputs invalid; the counters are re-armed, as layer_error does). */
int mi355x_backend_synchronize(mi355x_backend_t backend);
int mi355x_backend_supports_op(const mi355x_tensor *op); /* 1 / 0 */
/* Node fusion in graph_compute (default on): RMS_NORM -> MUL(norm weight) ->
 * MUL_MAT(s) and SWIGLU -> MUL_MAT run as ONE GEMV launch whose prologue computes
 * the norm / swiglu before the Q8_K quantization, and MUL_MAT -> ADD(residual)
 * writes mul_mat + residual from the GEMV's epilogue; RMS_NORM -> MUL alone is one
 * kernel. Fused intermediates (not flagged OUTPUT, read by no other node) are not
 * written. Results are bit-identical with fusion off. Returns the previous value. */
int mi355x_backend_set_fusion(mi355x_backend_t backend, int enable);
/* Decode attention fused with the o-proj GEMV (default OFF: bit-identical, but measured 6-10 %
 * slower per token than the two launches; needs fusion on): an ATTN_DECODE
 * of one token whose output only the next node reads, a K-quant MUL_MAT (+ its residual
 * ADD), runs as ONE launch -- workgroup (s, rb) computes the heads of the o-proj's K
 * superblock s, quantizes them to that Q8_K superblock and writes the exact integer records
 * of rows block rb; the last workgroup of each row block replays every row's fp32 chain in
 * superblock order (csrc/kq_attn_oproj.hip). Bit-identical to the two launches. Applies with
 * the per-head attention kernel (mi355x_attn_impl ATTN_HEAD), head_dim 64 / 128, the heads
 * of one K superblock in one KV group, K <= 4096 and a KV cache of <= 256 cells. Returns
 * the previous value. */
int mi355x_backend_set_attn_oproj(mi355x_backend_t backend, int enable);
/* Persistent decode layer (default off; needs fusion on): the 15 nodes of one
 * llm_build_llama decode layer -- RMS_NORM, MUL, MUL_MAT q / k / v, ATTN_DECODE, MUL_MAT o,
 * ADD, RMS_NORM, MUL, MUL_MAT gate / up, SWIGLU, MUL_MAT down, ADD -- run as ONE launch of one
 * workgroup per CU (csrc/kq_layer.hip): each workgroup owns rows of every matrix, streams
 * the next stage's weights into LDS while the current stage's output is handed over
 * between workgroups, and replays each row's fp32 chain in superblock order, so every
 * output is bit-identical to the per-node path (ggml_compute_forward_mul_mat row by row,
 * README.md:125-137). Applies to K-quant weights with contiguous rows, n_embd <= 4096,
 * head_dim 64 / 128, the position's rope row staged with the inputs, and a KV cache whose
 * attention LDS fits beside the weight ring. Returns the previous value. */
int mi355x_backend_set_layer_engine(mi355x_backend_t backend, int enable);
/* Non-zero when a persistent-layer launch since the last call gave up waiting for another
 * workgroup (the device did not keep every workgroup resident): that graph's outputs are
 * invalid. Clears the flag and re-arms the launches' counters. 0 without such launches. */
int mi355x_backend_layer_error(mi355x_backend_t backend);
/* Runs nodes in order on the backend stream. Consecutive MUL_MAT nodes with
 * ne11 == 1 that share src[1] are fused into one launch. When `use_graph` is
 * non-zero the launch sequence is captured once into a hipGraph and replayed
 * on later calls with the same node list (same pointers and shapes).
 * Returns 0 (GGML_STATUS_SUCCESS) or an error code. */
int mi355x_backend_graph_compute(mi355x_backend_t backend, mi355x_tensor *const *nodes,
                                 int n_nodes, int use_graph);

/* ------------------------------------------- ggml graph lowering (host only) */
/* The adapter side of the drop-in: a ggml_tensor-shaped mirror
 * that a ggml backend's graph_compute fills from the ggml_cgraph it is handed
 * (ggml_backend_sched_compute_splits -> iface.graph_compute, README.md:162-163),
 * one mirror per ggml node/leaf with the same fields (type, ne, nb, op, op_params,
 * src, view_src/view_offs, data), and the lowering of llm_build_llama's decode
 * node sequence onto this backend's node list:
 *   GET_ROWS, RMS_NORM, MUL, ADD, MUL_MAT (K-quant x f32), GLU(SWIGLU, split) map 1:1;
 *   RESHAPE / VIEW / PERMUTE / TRANSPOSE are aliases (no node);
 *   the non-flash attention block — ROPE(Q), ROPE(K), SET_ROWS(K cache), SET_ROWS
 *   (V cache), MUL_MAT(K cache, Q), SOFT_MAX(kq, mask, scale), MUL_MAT(V cache, kq),
 *   PERMUTE, CONT — becomes ONE ATTN_DECODE node (rope table from the caller);
 *   [up, gate] MUL_MAT pairs read by SWIGLU(gate, up) are emitted as [gate, up]
 *   (independent nodes; the order the fused gate/up launch takes).
 * The op numbering is this library's (the adapter maps GGML_OP_* by name). */
enum mi355x_gop {
    MI355X_GOP_NONE = 0, MI355X_GOP_GET_ROWS, MI355X_GOP_RMS_NORM, MI355X_GOP_MUL, MI355X_GOP_ADD,
    MI355X_GOP_MUL_MAT, MI355X_GOP_ROPE, MI355X_GOP_SET_ROWS, MI355X_GOP_SOFT_MAX, MI355X_GOP_GLU,
    MI355X_GOP_RESHAPE, MI355X_GOP_VIEW, MI355X_GOP_PERMUTE, MI355X_GOP_TRANSPOSE, MI355X_GOP_CONT,
    MI355X_GOP_CPY,
};
#define MI355X_GLU_SWIGLU 2  /* op_params[0] of a GLU node (ggml_glu_op GGML_GLU_OP_SWIGLU) */
typedef struct mi355x_gtensor {
    int type;                       /* ggml_type numbering (F32 0, F16 1, Q4_K 12, ..., I32 26, I64 27) */
    int op;                         /* enum mi355x_gop                           */
    int64_t ne[4];
    size_t nb[4];
    int32_t op_params[16];          /* as ggml stores them (floats as bits)      */
    int32_t flags;                  /* MI355X_TENSOR_FLAG_OUTPUT for graph outputs */
    struct mi355x_gtensor *src[10];
    struct mi355x_gtensor *view_src;
    size_t view_offs;
    void *data;                     /* device pointer (leaves, and nodes' outputs) */
    char name[64];
} mi355x_gtensor;
typedef struct {
    void *rope_table;               /* f32 [head_dim, n_pos] from mi355x_rope_table  */
    int rope_n_pos;                 /* its rows (>= the KV cache size)           */
    float rope_freq_base, rope_freq_scale; /* the table's parameters (checked against ROPE) */
    int cells_eq_pos;               /* the adapter's promise, checked on the host before the
                                     * call: ONE sequence, every token's K/V cell index
                                     * (SET_ROWS k_idxs / v_idxs) equals its position
                                     * (inp_pos), the mask is the causal mask over cells
                                     * [0, pos] and the KQ / KQV views start at cell 0.
                                     * ATTN_DECODE writes cell == pos and attends over
                                     * [0, pos]; with 0 here attention blocks are not
                                     * lowered (MI355X_E_UNSUPPORTED). */
} mi355x_lower_opts;
/* Lowers `n` ggml nodes (graph order) into backend nodes. Tensors are written into
 * `arena` (cap entries: nodes and the leaf mirrors they reference); `nodes_out`
 * (cap nodes_cap) receives the node list for mi355x_backend_graph_compute and
 * *n_nodes its length. Returns 0, MI355X_E_UNSUPPORTED (a node or pattern this
 * backend does not take: the caller leaves the graph to another backend) or
 * MI355X_E_INVAL / MI355X_E_WORKSPACE (arena or output too small). */
int mi355x_lower_ggml_graph(mi355x_gtensor *const *gnodes, int n, const mi355x_lower_opts *opts,
                            mi355x_tensor *arena, int arena_cap, mi355x_tensor **nodes_out, int nodes_cap,
                            int *n_nodes);

/* Row split over one process per GPU. RCCL is resolved at run time
 * from the librccl.so.1 already loaded in the process, or /opt/rocm's (dlopen): the
 * library has no link-time RCCL dependency. Rank 0 creates the id, the caller ships
 * its bytes to the other ranks (any control channel: torch.distributed gloo, MPI,
 * a file), then every rank joins. mi355x_comm_id_size() == 128 (ncclUniqueId). */
size_t mi355x_comm_id_size(void);
int mi355x_comm_get_unique_id(void *id_out);                      /* rank 0 */
int mi355x_backend_set_comm(mi355x_backend_t backend, int rank, int world,
                            const void *unique_id);               /* collective: every rank */
int mi355x_backend_comm_world(mi355x_backend_t backend);         /* 0 if no communicator */
/* Test emulation of ONE rank of a world on a single GPU, without a communicator:
 * ALL_GATHER then copies this rank's slice to offset rank*n of its output and leaves
 * the other ranks' parts as the caller put them; ALL_REDUCE leaves its output as the
 * caller put it (the reduced vector the other ranks would deliver; the rank's partial
 * stays readable in its source node). world = 0 turns it off. */
int mi355x_backend_set_comm_loopback(mi355x_backend_t backend, int rank, int world);

/* ------------------------------------------------ GGUF model files (host) */
/* Reader for GGUF v2/v3 files, the loader side of the path: llama-bench reads the
 * model through ggml's gguf_reader (artifacts/perf/out.folded:2-3, 17-22) and
 * llama_model_loader (out.folded:39-46); format restated in kq_gguf.cpp [U].
 * The file is mapped read-only; tensor bytes (GGUF block layout, no repack) go to
 * the device with mi355x_gguf_upload. Host-only except the upload: works without
 * a GPU. */
typedef struct mi355x_gguf *mi355x_gguf_t;

typedef struct {
    const char *name;  /* valid while the file is open */
    int type;          /* ggml type number (enum mi355x_type for the K-quants / F32) */
    int n_dims;
    int64_t ne[4];     /* ne[0] = row length (K), ne[1] = rows (N), unused dims 1 */
    uint64_t offset;   /* absolute byte offset of the data in the file */
    uint64_t size;     /* bytes; 0 when the type's block size is unknown to the reader */
} mi355x_gguf_tensor;

/* GGUF metadata value types (gguf_type [U]) */
enum mi355x_gguf_type {
    MI355X_GGUF_U8 = 0, MI355X_GGUF_I8 = 1, MI355X_GGUF_U16 = 2, MI355X_GGUF_I16 = 3,
    MI355X_GGUF_U32 = 4, MI355X_GGUF_I32 = 5, MI355X_GGUF_F32 = 6, MI355X_GGUF_BOOL = 7,
    MI355X_GGUF_STRING = 8, MI355X_GGUF_ARRAY = 9, MI355X_GGUF_U64 = 10, MI355X_GGUF_I64 = 11,
    MI355X_GGUF_F64 = 12,
};

mi355x_gguf_t mi355x_gguf_open(const char *path);  /* NULL on error (reason on stderr) */
void mi355x_gguf_close(mi355x_gguf_t g);
uint32_t mi355x_gguf_version(mi355x_gguf_t g);
uint64_t mi355x_gguf_alignment(mi355x_gguf_t g);    /* general.alignment, default 32 */
uint64_t mi355x_gguf_data_offset(mi355x_gguf_t g);  /* start of the tensor data section */
int64_t mi355x_gguf_n_tensors(mi355x_gguf_t g);
int64_t mi355x_gguf_find_tensor(mi355x_gguf_t g, const char *name); /* index or -1 */
int mi355x_gguf_get_tensor(mi355x_gguf_t g, int64_t i, mi355x_gguf_tensor *out);
const void *mi355x_gguf_tensor_data(mi355x_gguf_t g, int64_t i);    /* host pointer (mapped) */
/* Async H2D copy of tensor i's bytes to device memory on `stream` (hipStream_t). */
int mi355x_gguf_upload(mi355x_gguf_t g, int64_t i, void *dst_device, size_t dst_size, void *stream);
int64_t mi355x_gguf_n_kv(mi355x_gguf_t g);
int64_t mi355x_gguf_find_key(mi355x_gguf_t g, const char *key);     /* index or -1 */
const char *mi355x_gguf_key(mi355x_gguf_t g, int64_t i);
int mi355x_gguf_kv_type(mi355x_gguf_t g, int64_t i);                /* enum mi355x_gguf_type */
int mi355x_gguf_get_int(mi355x_gguf_t g, int64_t i, int64_t *out);   /* integer / bool values */
int mi355x_gguf_get_float(mi355x_gguf_t g, int64_t i, double *out);  /* any numeric value */
const char *mi355x_gguf_get_str(mi355x_gguf_t g, int64_t i);        /* NULL unless a string */
int64_t mi355x_gguf_arr_n(mi355x_gguf_t g, int64_t i);              /* array length, or -1 */

#ifdef __cplusplus
}
#endif

#endif /* GGML_MI355X_H */
