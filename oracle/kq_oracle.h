/*
 * kq_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * Scalar C restatement of the reference's K-quant dot-product path, used ONLY by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
 * (never as the thing measured or shipped). The product path
 * (ggml-neon-opt_amd/) never links or calls this code.
 *
 * Parity status: the reference (/root/reference) ships no tests, fixtures or
 * golden vectors for this path and its llama.cpp submodule is not vendored, so
 * the oracle is "parity unpinned" against reference-produced outputs. It is
 * pinned instead to (1) the reference's own quoted NEON source
 * (README.md:686-779, optimized form :1455-1480), (2) its disassembly, which
 * fixes struct offsets and the FP contraction (fmsub README.md:551, fmadd :614),
 * and (3) an independent numpy restatement (oracle/kq_oracle_np.py) checked
 * bit-for-bit against this C code by tests/test_oracle.py; golden vectors made
 * from it are committed under tests/golden/ with their generator script.
 */
#ifndef KQ_ORACLE_H
#define KQ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KQO_QK_K 256

typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; } kqo_block_q4_K;
typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; } kqo_block_q5_K;
typedef struct { uint8_t ql[128]; uint8_t qh[64]; int8_t scales[16]; uint16_t d; } kqo_block_q6_K;
typedef struct { float d; int8_t qs[256]; int16_t bsums[16]; } kqo_block_q8_K;

float kqo_fp16_to_fp32(uint16_t h);
uint16_t kqo_fp32_to_fp16(float f); /* round-to-nearest-even, for generators */

/* quantize_row_q8_K_ref. fused=1: iscale*x + 12582912.f contracted into one
 * fma, as gcc -O2 -std=gnu11 (fp-contract=fast) builds it for aarch64, the
 * reference's build (README.md:673). fused=0: ISO-C two roundings. */
void kqo_quantize_row_q8_K(const float *x, kqo_block_q8_K *y, int64_t k, int fused);

void kqo_dequantize_row_q4_K(const kqo_block_q4_K *x, float *y, int64_t k);
void kqo_dequantize_row_q5_K(const kqo_block_q5_K *x, float *y, int64_t k);
void kqo_dequantize_row_q6_K(const kqo_block_q6_K *x, float *y, int64_t k);

/* ggml_vec_dot_t-shaped: (n, s, bs, vx, bx, vy, by, nrc); nrc must be 1. */
void kqo_vec_dot_q4_K_q8_K_neon(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc);
void kqo_vec_dot_q4_K_q8_K_generic(int n, float *s, size_t bs, const void *vx, size_t bx,
                                   const void *vy, size_t by, int nrc);
void kqo_set_contraction_variant(int which, int v); /* tests only: DESIGN.md §2 [U] choices */
void kqo_vec_dot_q5_K_q8_K_neon(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc);
void kqo_vec_dot_q6_K_q8_K_neon(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc);
void kqo_vec_dot_q6_K_q8_K_generic(int n, float *s, size_t bs, const void *vx, size_t bx,
                                   const void *vy, size_t by, int nrc);

/* AVX2 forms (kq_cpu_simd.c): same integers, same fp32 chain -> bit-identical. */
void kqo_vec_dot_q4_K_q8_K_simd(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc);
void kqo_vec_dot_q5_K_q8_K_simd(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc);
void kqo_vec_dot_q6_K_q8_K_simd(int n, float *s, size_t bs, const void *vx, size_t bx,
                                const void *vy, size_t by, int nrc);

/* Per-superblock integer partials (sumi, summins) of row . col, out[2*b+{0,1}].
 * Q6_K: (isum with unsigned 0..63 quants, isum_mins = sum bsums_g*sc_g). */
void kqo_block_partials(int type, int n, const void *vx, const void *vy, int32_t *out);

/* Restated ggml_compute_forward_mul_mat (ggml-cpu.c:1389) for src0 K-quant,
 * src1 f32: quantize src1 (per-thread slices), barrier, 64/16-row chunks handed
 * out by an atomic counter, one_chunk 16x16 blocking calling vec_dot per
 * (row, col). pthreads, n_threads >= 1. dst[j*N + i] (dst column j contiguous).
 * variant: 0 = NEON-order dot, 1 = generic dot, 2 = NEON order with AVX2 integer
 * parts (bit-identical to 0). Worker threads persist between calls. Returns 0 on success. */
int kqo_mul_mat(int type, const void *src0, int64_t K, int64_t N, size_t nb01,
                const float *src1, int64_t M, size_t nb11, float *dst,
                int n_threads, int variant);

/* Same, with src1 already in Q8_K (M rows of K/256 blocks, contiguous). */
int kqo_mul_mat_q8(int type, const void *src0, int64_t K, int64_t N, size_t nb01,
                   const void *src1_q8, int64_t M, float *dst, int n_threads, int variant);


/* Run fn(ctx, task) for task in [0, n_tasks) on the persistent worker pool. */
void kqo_pool_run(int n_threads, int n_tasks, void (*fn)(void *ctx, int task), void *ctx);

/* ---- non-matmul decode ops (kq_ops_oracle.c) ---- */
uint16_t kqo_f16_fma(uint16_t a, uint16_t b, uint16_t c);
uint16_t kqo_f16_add(uint16_t a, uint16_t b);
void kqo_fp32_to_fp16_row(const float *x, uint16_t *y, int64_t n);
float kqo_vec_dot_f16(int n, const uint16_t *x, const uint16_t *y);
float kqo_v_expf(float x);
void kqo_vec_swiglu_f32(int n, float *y, const float *x, const float *g);
void kqo_soft_max_row(int n, float *dp, const float *sp, const float *mask, float scale);
void kqo_rms_norm_f32(const float *x, float *y, int64_t n, float eps);
void kqo_mul_f32(const float *a, const float *b, float *y, int64_t n);
void kqo_add_f32(const float *a, const float *b, float *y, int64_t n);
float kqo_rope_theta_scale(float freq_base, int n_dims);
void kqo_rope_table(float *table, int n_pos, int n_dims, float freq_base, float freq_scale);
void kqo_rope_norm(const float *x, float *y, int head_dim, int n_dims, int n_heads, int pos, const float *table);
void kqo_get_rows(int type, const void *table, int64_t k, size_t row_stride, const int32_t *ids, int64_t n_ids,
                  float *out);
int kqo_attn_n_kv(int pos, int n_ctx);
void kqo_attn_decode(const float *q, const float *k, const float *v, uint16_t *k_cache, uint16_t *v_cache, int pos,
                     int n_ctx, int n_head, int n_head_kv, int head_dim, float scale, float *out);

/* ---- CPU-baseline forms (kq_cpu_simd.c), bit-identical to the restatements above ---- */
uint16_t kqo_f16_fma_fast(uint16_t a, uint16_t b, uint16_t c);  /* double TwoSum + midpoint fix */
uint16_t kqo_f16_add_fast(uint16_t a, uint16_t b);
long kqo_f16_fast_check(long n, uint64_t seed);  /* mismatches vs kqo_f16_fma / _add on random triples */
void kqo_attn_decode_fast(const float *q, const float *k, const float *v, uint16_t *k_cache, uint16_t *v_cache,
                          int pos, int n_ctx, int n_head, int n_head_kv, int head_dim, float scale, float *out,
                          int n_threads);

#ifdef __cplusplus
}
#endif
#endif
