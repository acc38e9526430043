// kq_common.h — shared device/host definitions for the gfx950 K-quant kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ggml_mi355x.h"

namespace kq {

constexpr int QK = 256;
constexpr int WAVE = 64;
constexpr int WG_THREADS = 256;     // 4 waves per workgroup
constexpr int WAVES_PER_WG = WG_THREADS / WAVE;
constexpr int LANES_PER_BLOCK = 8;  // 8 lanes cooperate on one superblock
constexpr int BLOCKS_PER_STEP = WAVE / LANES_PER_BLOCK;  // 8 superblocks per wave-step
constexpr int ACT_QS_STRIDE = 272;  // LDS bytes per activation superblock (256 + 16 pad)
constexpr int MAX_NCOL = 8;

constexpr int Q4_K = MI355X_TYPE_Q4_K;
constexpr int Q5_K = MI355X_TYPE_Q5_K;
constexpr int Q6_K = MI355X_TYPE_Q6_K;

__host__ __device__ constexpr int block_bytes(int type) {
    return type == Q4_K ? 144 : type == Q5_K ? 176 : type == Q6_K ? 210 : 0;
}

// Argument block of the GEMV / small-M kernel (passed by value).
struct GemvArgs {
    int n_desc;
    int nb;           // K / 256
    int R;            // rows per task (8: one per lane octet)
    int m_total;      // activation columns in total (grid.y covers ceil(m_total/NCOL))
    int tasks_total;
    int out_per_wg;   // LDS floats for staged outputs (tasks_per_wg * 8 * NCOL)
    int diag;         // diagnostics: bit0 prologue only, bit1 empty
    int ring;         // LDS ring depth D (weight steps in flight per wave)
    int ring_override; // host-side experiment knob (MI355X_GEMV_RING), 0 = auto
    int task_prefix[MI355X_MAX_FUSED + 1];
    int type[MI355X_MAX_FUSED];
    int n_rows[MI355X_MAX_FUSED];
    const uint8_t *w[MI355X_MAX_FUSED];
    int64_t row_stride[MI355X_MAX_FUSED];  // bytes
    float *y[MI355X_MAX_FUSED];
    int64_t y_col_stride[MI355X_MAX_FUSED];  // floats between dst columns
    const float *x;       // f32 input (FUSEDQ): column j at x + j*x_col_stride
    int64_t x_col_stride; // floats
    const uint8_t *xq;    // Q8_K input (!FUSEDQ): column j at xq + j*xq_col_stride
    int64_t xq_col_stride; // bytes
    int32_t *dbg;         // debug partials (DEBUG builds of the kernel only)
    uint64_t *stamps;     // diagnostics: per-wave s_memrealtime stamps (or null)
    int64_t stamps_cap;   // entries available in stamps
};

// LDS layout of one workgroup (dynamic shared memory).
//   ring: per wave D slots of `slot` bytes (8 rows x one superblock)
//   act:  per wave, its K-range of activations (f32 staging / raw Q8_K per column)
//   recs: 2 task slots x 3 waves x ncol x 8 rows x spw exact chain records
//   outs: staged results of wave 0 (tasks_per_wg x ncol x 8 floats)
struct LdsLayout {
    int ring, act, act_per_wave, act_col, recs, outs, spw, total;
};

__host__ __device__ inline LdsLayout lds_layout(int ncol, int nb, int out_per_wg, bool fusedq, int slot, int D) {
    LdsLayout L;
    L.spw = (nb + WAVES_PER_WG - 1) / WAVES_PER_WG;  // max superblocks per wave per task
    L.ring = 0;
    L.act = WAVES_PER_WG * D * slot;
    L.act_col = (L.spw * 292 + 16 + 15) & ~15;
    L.act_per_wave = fusedq ? L.spw * 1024 : ncol * L.act_col;
    L.recs = L.act + WAVES_PER_WG * L.act_per_wave;
    L.outs = L.recs + 2 * (WAVES_PER_WG - 1) * ncol * 8 * L.spw * 16;
    L.total = L.outs + out_per_wg * 4;
    return L;
}

// ---------------------------------------------------------------- row-stream decode GEMV
// kq_rows (M = 1): one workgroup of ROWS_WAVES waves per CU. Global wave index
// gw = wave * gridDim.x + blockIdx.x (active waves spread over every CU). Matrix d
// owns global waves [wave_prefix[d], wave_prefix[d+1]); its j-th wave owns rows
// [j*rbase[d] + min(j, rrem[d]), ...) — rbase[d] rows, one more for j < rrem[d].
#ifndef KQ_ROWS_WAVES
#define KQ_ROWS_WAVES 12
#endif
constexpr int ROWS_WAVES = KQ_ROWS_WAVES;  // the most waves per workgroup (LDS layout, launch bounds)
// Small launches run ROWS_WAVES_SMALL waves per workgroup (the wave count is a launch
// parameter: blockDim.x / 64): fewer waves to dispatch for a stream that is short anyway.
#ifndef KQ_ROWS_WAVES_SMALL
#define KQ_ROWS_WAVES_SMALL 6
#endif
constexpr int ROWS_WAVES_SMALL = KQ_ROWS_WAVES_SMALL;
constexpr int ROWS_QPASS = 3;  // fused-quantization passes of 4*ROWS_WAVES superblocks
// L2 prefetch issued with the first weight step (waves whose stream outlasts the
// ring): while the activation is fetched and quantized, each wave touches the next
// ROWS_PF x 4 KB of its stream past the ring (one dword per 64-B sector), so the HBM
// keeps streaming and those steps later DMA from L2 / the Infinity Cache.
#ifndef KQ_ROWS_PF
#define KQ_ROWS_PF 2
#endif
constexpr int ROWS_PF = KQ_ROWS_PF;  // touches per wave when a.pf != 0

struct RowsArgs {
    int n_desc;
    int nb;           // K / 256
    int rpw;          // max rows per wave (LDS sizing)
    int waves_total;
    int pre0;         // weight steps issued before the activation is quantized
    int pf;           // L2 prefetch on/off (ROWS_PF 4-KB touches of the stream past the ring)
    int bR;           // rows per chain batch (bR*nb % 16 == 0 unless bR >= rpw)
    int xmode;        // fused-quantization prologue: ROWS_X_* bits
    int diag;         // diagnostics (timing only): bit3 stream weights only, 16/32 prologue, 64 no quantization, 128 no SWIGLU epilogue, 256 empty launch
    int wave_prefix[MI355X_MAX_FUSED + 1];
    int rbase[MI355X_MAX_FUSED];
    int rrem[MI355X_MAX_FUSED];
    int type[MI355X_MAX_FUSED];
    const uint8_t *w[MI355X_MAX_FUSED];
    float *y[MI355X_MAX_FUSED];
    const float *x;       // f32 activation (FUSEDQ)
    const uint8_t *xq;    // Q8L activation row (!FUSEDQ), written by kq_quantize_q8L
    uint64_t *stamps;
    int64_t stamps_cap;
    // fused neighbours of the MUL_MAT in the decode graph (FUSEDQ only):
    int pro;              // ROWS_PRO_*: transform of x before its Q8_K quantization
    float eps;            // ROWS_PRO_NORM: rms_norm epsilon
    const float *x2;      // ROWS_PRO_NORM: norm weight (the MUL after RMS_NORM); ROWS_PRO_SWIGLU: up (x = gate)
    const float *res[MI355X_MAX_FUSED];  // y[m] = mul_mat + res[m] (the ADD after the MUL_MAT), or null
    int n_rows[MI355X_MAX_FUSED];
    // SWIGLU epilogue (epi != 0): y[0] = gate, y[1] = up with equal rows and wave counts,
    // up wave `wave` pairs with gate wave `wave - epi_wave_off` of the same workgroup
    // (identical row ranges); epi_y[r] = swiglu(gate[r], up[r]) for r < epi_n
    int epi, epi_n, epi_wave_off;
    float *epi_y;
    int64_t prio_bytes;  // the most weight bytes any wave streams (KQ_ROWS_PRIO: remaining-work priority)
    // kq_rows_dyn (claimed rows): workgroup b owns rows [b*N/G, (b+1)*N/G) of every matrix
    // (rpw = the most such rows over the matrices, summed); its waves claim units of dyn_u
    // rows from an LDS counter, the first dyn_p units of each wave assigned statically
    int dyn_u, dyn_p, dyn_ush;  // (dyn_u = 1 << dyn_ush; rbase[0] / rrem[0]: the rows N / G split)
};
constexpr int ROWS_PRO_NONE = 0, ROWS_PRO_NORM = 1, ROWS_PRO_SWIGLU = 2;
// Prologue of the fused quantization (a.xmode bits):
//  ROWS_X_ROT   workgroup b visits the activation's superblocks from b mod nb on, so the
//               256 workgroups do not all read the same L2 lines at the same moment;
//  ROWS_X_BAR   a workgroup barrier between every wave's activation loads and the first
//               weight DMA (the activation requests are queued ahead of the stream's);
//  ROWS_X_PIPE  pass i is transformed and quantized as soon as ITS loads landed, while
//               the later passes (and the weight steps) are still in flight.
constexpr int ROWS_X_ROT = 1, ROWS_X_BAR = 2, ROWS_X_PIPE = 4;

// One step = 16 consecutive superblocks of a wave's row stream (2304 / 2816 / 3360
// B), fetched as 16-B granules from the 16-B boundary below them (+1 granule of
// slack for a misaligned Q6_K stream): 145 / 177 / 211 granules = 3 / 3 / 4
// LDS-DMA instructions. Ring depth per type keeps 6.8-8.5 KB in flight per wave,
// ~80-100 KB per CU (measured ceiling: 2-3 KB steps, ~96 KB per CU, nt -> 7.1 TB/s).
constexpr int ROWS_SB = 16;     // superblocks per step (4 lanes each)
#ifndef KQ_MMQ_PF
#define KQ_MMQ_PF 0  // kq_mmq tiles: L2 warm-up distance of the weight tile in superblocks (0 off; 2, 3 measured neutral to -5 %)
#endif
constexpr int MMQ_PF_LDS = KQ_MMQ_PF ? 1024 : 0;  // its scratch: 256 B per wave
constexpr int Q8L_STRIDE = 304; // LDS/workspace Q8_K block: d @0, qs @16, bsums @272 (16-B aligned)
#ifndef KQ_MMQ_NBUF
#define KQ_MMQ_NBUF 2  // kq_mmq superblock buffers in LDS (experiment: 3 on the one-workgroup-per-CU tiles)
#endif
// Superblock buffers of a kq_mmq tile (RT weight rows x 64*CW columns): KQ_MMQ_NBUF where the
// tile already runs one workgroup per CU (128 x 64 at two waves per SIMD, 64 x 128) and the
// buffers fit the CU's LDS; else 2.
// Column groups of waves: 2 (a wave takes 32 x CW of the tile's 64 x CW columns), or 1 for
// CW = 4 (the 4-wave 128 x 128 tile: every wave all 128 columns of its 32 rows, one wave per
// SIMD with every register: each weight operand feeds four MFMA column tiles).
__host__ __device__ constexpr int mmq_cgroups(int cw) { return cw == 4 ? 1 : 2; }
__host__ __device__ constexpr int mmq_cols(int cw) { return 32 * cw * mmq_cgroups(cw); }
__host__ __device__ constexpr int mmq_waves(int rt, int cw) { return rt / 32 * mmq_cgroups(cw); }
// Q6_K rows staged at KQ_MMQ_Q6_STRIDE bytes: the 14 granules of a 210-B block (fetched from
// the 16-B boundary below it, 224 B) plus one padding granule at 240, so consecutive rows start
// 60 dwords apart (16 bank offsets) instead of 56 (8): the tile's realigned row reads
// conflicted for 71 % of the LDS's active cycles at 224 (profiles/r06_prefill_stall.md).
#ifndef KQ_MMQ_Q6_STRIDE
#define KQ_MMQ_Q6_STRIDE 240
#endif
static_assert(KQ_MMQ_Q6_STRIDE % 16 == 0 && KQ_MMQ_Q6_STRIDE >= 224, "whole granules");
__host__ __device__ constexpr int mmq_buf_bytes(int type, int rt, int cw) {
    return mmq_cols(cw) * Q8L_STRIDE + rt * (type == Q6_K ? KQ_MMQ_Q6_STRIDE : block_bytes(type));
}
__host__ __device__ constexpr int mmq_nbuf(int type, int rt, int cw) {
    return KQ_MMQ_NBUF == 1 ? 1 : KQ_MMQ_NBUF >= 3 && ((rt == 128 && cw == 1) || (rt == 64 && cw == 2)) &&
                   3 * mmq_buf_bytes(type, rt, cw) + 16 + MMQ_PF_LDS <= 160 * 1024
               ? 3
               : 2;
}
constexpr int ROWS_RECS = 64;   // chain records per wave per batch (soft cap)
__host__ __device__ constexpr int rows_gran(int type) { return block_bytes(type) + 1; }
__host__ __device__ constexpr int rows_slot(int type) { return 16 * rows_gran(type); }
__host__ __device__ constexpr int rows_ni(int type) { return (rows_gran(type) + 63) / 64; }
#ifndef KQ_ROWS_DQ4
#define KQ_ROWS_DQ4 3
#endif
#ifndef KQ_ROWS_DQ6
#define KQ_ROWS_DQ6 2
#endif
__host__ __device__ constexpr int rows_depth(int type) {
    return type == Q4_K ? KQ_ROWS_DQ4 : type == Q5_K ? 3 : KQ_ROWS_DQ6;
}
__host__ __device__ constexpr int rows_ring_bytes(int type) { return rows_depth(type) * rows_slot(type); }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }
__host__ __device__ constexpr int rows_ring(int tmask) {
    return 16 + cmax((tmask & 1) ? rows_ring_bytes(Q4_K) : 0,
                     cmax((tmask & 2) ? rows_ring_bytes(Q5_K) : 0, (tmask & 4) ? rows_ring_bytes(Q6_K) : 0));
}

//   act:  Q8_K activation row in the aligned Q8L layout (nb * 304 B)
//   ring: per wave, the ring of its type (+16 B tail slack for Q6_K realign reads)
//   recs: per wave bR*nb chain records (16 B), block-major [blk][row]
//   outs: per wave rpw staged results
struct RowsLayout {
    int act, ring, ring_stride, recs, recs_stride, outs, outs_stride, sums, total;
};
// nwv = the launch's waves per workgroup (blockDim.x / 64)
__host__ __device__ inline RowsLayout rows_layout(int nb, int tmask, int bR, int rpw, int nwv) {
    RowsLayout L;
    L.act = 0;
    L.ring = nb * Q8L_STRIDE;
    L.ring_stride = rows_ring(tmask);
    L.recs = L.ring + nwv * L.ring_stride;
    L.recs_stride = bR * nb * 16;
    L.outs = L.recs + nwv * L.recs_stride;
    L.outs_stride = (rpw * 4 + 15) & ~15;
    L.sums = L.outs + nwv * L.outs_stride;  // ROWS_PRO_NORM: per-superblock sums of squares (double)
    L.total = L.sums + nb * 8;
    return L;
}

// kq_rows_dyn: act | ring (per wave) | recs (per wave: a batch of bR rows, bR x nb records) |
// outs (the workgroup's rows of every matrix, flat) | sums | claim counter
struct RowsDynLayout {
    int act, ring, ring_stride, recs, recs_stride, outs, sums, cnt, total;
};
__host__ __device__ inline RowsDynLayout rows_dyn_layout(int nb, int tmask, int bR, int flat_rows, int nwv) {
    RowsDynLayout L;
    L.act = 0;
    L.ring = nb * Q8L_STRIDE;
    L.ring_stride = rows_ring(tmask);
    L.recs = L.ring + nwv * L.ring_stride;
    L.recs_stride = bR * nb * 16;
    L.outs = L.recs + nwv * L.recs_stride;
    L.sums = L.outs + ((flat_rows * 4 + 15) & ~15);
    L.cnt = L.sums + nb * 8;
    L.total = L.cnt + 16;
    return L;
}

// Decode attention block (kq_ops.hip): one workgroup per query head.
struct AttnArgs {
    const float *q, *k, *v;       // projections of this token (before rope)
    const int32_t *pos;           // device: the token's position (cache cell)
    const float *rope_table;      // [n_ctx][head_dim/2][cos, sin]
    uint16_t *k_cache;            // f16 [n_ctx][n_head_kv*head_dim]
    uint16_t *v_cache;            // f16 [n_head_kv*head_dim][n_ctx] (transposed, non-FA layout)
    float *out;                   // [n_head*head_dim]
    int n_ctx, n_head, n_head_kv, head_dim;
    float scale;
    int diag;  // diagnostics only (MI355X_ATTN_DIAG): 1/2/3 stop after loads/KQ/soft_max, 4 empty
    int rope_row;  // rope_table holds only the row of *pos (no position-dependent load)
    int no_store;     // prompt batch: the KV cells are already stored (the k/v GEMM's epilogue)
    uint8_t *q8_out;  // prompt batch (kq_attn_prompt_group): also the output rows as Q8L blocks
                      // for the next GEMM (row i's superblock b at (i*nb + b)*304), or null
    int v_lds;        // kq_attn_decode only, set by launch_attn: the head's V rows are staged in
                      // LDS by LDS-DMA as soon as the position is known (attn_lds_v bytes)
    int n_tok;        // prompt batch (kq_attn_prompt_group), set by launch_attn_prompt: its tokens
};

// Decode attention fused with the o-proj GEMV (kq_attn_oproj.hip): workgroup (s, rb) runs the
// attention of the heads of superblock s of the o-proj's K, quantizes them (one Q8_K
// superblock) and writes the exact per-superblock records of rows [rb*R, rb*R + R); the
// last of the nsb workgroups of row block rb replays each row's chain in superblock order.
struct AttnOprojArgs {
    AttnArgs at;              // the attention (this node's heads; at.out unused)
    const uint8_t *w;         // o-proj weights: n_rows rows of nsb superblocks, row_stride bytes
    int64_t row_stride;
    int n_rows, nsb, R, n_rb;
    int head_lds;             // LDS bytes per head (attn_lds, 16-B multiple)
    const float *res;         // residual (ggml_add after the mul_mat), or null
    float *y;                 // n_rows outputs
    uint8_t *recs;            // [n_rb][R][nsb] 16-B records (written sc1, read sc1)
    uint32_t *cnt;            // [n_rb] arrival counters (monotonic: last = old % nsb == nsb - 1)
};

// ---------------------------------------------------------------- persistent decode layer
// kq_layer (kq_layer.hip): one llm_build_llama decode layer as ONE launch of one workgroup
// per CU. Stages: 0 q/k/v (attn_norm prologue), attention, 1 o-proj (+ x -> x1),
// 2 gate/up (ffn_norm prologue, SWIGLU -> h), 3 down (+ x1 -> x2). Matrices m: 0 q, 1 k,
// 2 v, 3 o, 4 gate, 5 up, 6 down. Edges e (counter sets in `sync`): 0 q/k/v -> attention,
// 1 attention -> o-proj, 2 x1 -> gate/up, 3 h -> down.
constexpr int LAYER_WAVES = 8;       // 7 weight-stream waves + 1 control wave
constexpr int LAYER_SYNC_U32 = 32 * 33;  // epoch + 4 edges x 8 shards, each on its own 128-B line
struct LayerArgs {
    int G;                           // workgroups (one per CU, all co-resident)
    int E, F, nb_e, nb_f, nq, nkv;   // embd, ffn, K / 256 of each; rows of attn_q, attn_k (= attn_v)
    int type[7];
    const uint8_t *w[7];             // contiguous rows of K / 256 blocks
    float *y[3];                     // q / k / v (written sc1: the attention's inputs)
    const float *x;                  // layer input (written by the previous launch)
    const float *attn_norm, *ffn_norm;
    float eps;
    float *att, *x1, *h, *x2;        // attention output, ffn_inp = o + x, swiglu(gate, up), layer output
    AttnArgs at;                     // q / k / v = y[0..2], rope_row staged with the position
    int n_attn, hpw, attn_stride, head_lds;  // attention workgroups, heads per workgroup, placement
    uint32_t *sync;                  // this launch's counter block (LAYER_SYNC_U32 words, zeroed once)
    int *err;                        // set when a wait timed out (co-residency lost): results invalid
    uint32_t expect[4][8];           // producers per edge and shard
    int D, slot;                     // ring slots per stream wave, bytes per slot
    int o_aux, act_bytes, o_sums, o_res, lds;  // LDS layout (ring at 0)
    const uint8_t *tab;              // every workgroup's step table (layer_table_fill), tab_stride bytes apart
    int64_t tab_stride;
    uint64_t *stamps;                // KQ_LAYER_STAMPS builds: 32 s_memrealtime stamps per workgroup
    int64_t stamps_cap;
};

// ---------------------------------------------------------------- batched (prefill) MFMA GEMM
// kq_mmq (M > 1): 64 x 64 output tiles, Q8L activations in a workspace.
struct MmqArgs {
    const uint8_t *w;        // weight rows (16-B aligned, row_stride % 16 == 0)
    int64_t row_stride;      // bytes
    int n_rows;
    const uint8_t *xq;       // Q8L activation columns
    int64_t xq_col_stride;   // bytes (nb * 304)
    int m_cols;
    float *y;                // dst column j at y + j * y_col_stride
    int64_t y_col_stride;    // floats
    int nb;
    const float *res;        // ADD epilogue (null: none): y = mul_mat + res, res column j at
    int64_t res_col_stride;  //   res + j * res_col_stride (the one f32 add of ggml_add)
    // kq_mmq (64 x 64 tiles) over up to 4 matrices of one type sharing the activation
    // (q/k/v of a prompt batch): row tiles [tile0[d], tile0[d+1]) are matrix d's; n_mat 1:
    // the fields above only
    int n_mat;
    int tile0[5];
    int mtype[4];  // kq_mmq_mixed: each matrix's type (Q4_K / Q6_K)
    // KV-cache store epilogue of a prompt's k / v projections (kv_kind[d]: 1 k -> rope ->
    // f16 cache rows, 2 v -> f16 transposed cache; 0 none); kv_cur: this tile's matrix
    int kv_kind[4], kv_cur;
    const int32_t *kv_pos;   // cell of each column (token)
    const float *kv_rope;    // [n_ctx][head_dim/2][cos, sin]
    uint16_t *kv_k_cache, *kv_v_cache;
    int kv_n_ctx, kv_hd;
    const uint8_t *mw[4];
    int64_t mrow_stride[4];
    int mn_rows[4];
    float *my[4];
    int64_t my_col_stride[4];
};

// ------------------------------------------- batched (prefill) f16 MFMA GEMM, stated tolerance
// kq_mmf (MI355X_PREFILL_F16): 128 weight rows x 128 activation columns per 4-wave
// workgroup, K in half-superblock steps. The activation goes through kq_quantize_f16img
// (the reference's Q8_K quantization, then f16(d*q) in the kernel's k order, 512 B per
// superblock, plus f16(d*bsum16) x 16 = 32 B), the weights are dequantized in registers.
constexpr int MMF_RT = 128;                      // weight rows per workgroup (4 waves x 32)
constexpr int MMF_COLS = 128;                    // activation columns per workgroup (4 MFMA tiles)
constexpr int MMF_IMG = 512;                     // f16 image bytes per superblock and column
constexpr int MMF_BSB = 32;                      // f16 d*bsum16 bytes per superblock and column
constexpr int MMF_BUF = MMF_COLS * (MMF_IMG / 2 + MMF_BSB);  // one half-superblock LDS buffer (36 KB)
struct MmfArgs {
    const uint8_t *w;          // weight rows
    int64_t row_stride;        // bytes
    int n_rows;
    const uint8_t *img;        // activation image, column j at img + j * nb * 512
    const uint8_t *bs;         // d*bsum16, column j at bs + j * nb * 32
    int m_cols;
    float *y;                  // dst column j at y + j * y_col_stride (n_split == 1)
    int64_t y_col_stride;      // floats
    float *slab;               // n_split > 1: partial sums [n_split][m_cols][n_rows]
    int nb;                    // superblocks of K
    int nbs;                   // superblocks per K split
    int n_split;
    int n_ct;                  // column tiles
    int n_rt;                  // row tiles
    int order;                 // tile order (speed only): 0 row tiles, 1 column tiles consecutive per XCD
    const float *res;          // ADD epilogue (null: none): y = mul_mat + res, column j at
    int64_t res_col_stride;    //   res + j * res_col_stride
    // up to 4 matrices of one type on one activation image in one launch (a prompt batch's
    // q/k/v or gate/up): row tiles [tile0[d], tile0[d+1]) are matrix d's, its rows are slab
    // columns [roff[d], roff[d] + mn_rows[d]) of n_rows (the sum); n_mat 1: the fields above
    int n_mat;
    int tile0[5];
    int roff[4];
    const uint8_t *mw[4];
    int64_t mrow_stride[4];
    int mn_rows[4];
    float *my[4];
    int64_t my_col_stride[4];
};

}  // namespace kq
