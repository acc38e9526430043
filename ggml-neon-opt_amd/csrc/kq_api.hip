// kq_api.hip — C-ABI of libggml_mi355x.so: argument checking, launch planning and
// the ggml-surface mirrors (vec_dot / from_float / mul_mat). Declared in
// include/ggml_mi355x.h.
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_ext.h>

#include "kq_common.h"
#include "kq_internal.h"

namespace kq {

template <int NCOL, bool FUSEDQ, bool DEBUG, int TMASK>
__global__ void kq_gemv(const GemvArgs a);
__global__ void kq_quantize_q8K(const float *x, int64_t x_stride, uint8_t *y, int nb, int64_t nblocks);
template <int TMASK, bool FUSEDQ, int PRO>
__global__ void kq_rows(const RowsArgs a);
template <int TMASK, bool FUSEDQ, int PRO>
__global__ void kq_rows_dyn(const RowsArgs a);
template <bool AM>
__global__ void kq_quantize_q8L(const float *x, int64_t x_stride, uint8_t *y, int nb, int64_t nblocks);
template <int TYPE, int RT, int CW>
__global__ void kq_mmq(const MmqArgs a);
template <int RT, int CW>
__global__ void kq_mmq_mixed(const MmqArgs a);
__global__ void kq_stream_ceiling(const uint8_t *buf, int64_t per_wave, int waves_total, uint32_t *sink);
__global__ void kq_quantize_f16img(const float *x, int64_t x_stride, uint8_t *img, uint8_t *bs, int nb, int64_t nblocks);
template <int TYPE, int NW>
__global__ void kq_mmf(const MmfArgs a);
__global__ void kq_mmf_reduce(const float *slab, int n_split, int m_cols, int n_rows, int slab_rows, float *y,
                              int64_t y_col_stride, const float *res, int64_t res_col_stride);

namespace {

// Per-device probe (the caller's current device): 0 unknown, 1 gfx950, -1 not usable.
// A process may drive several devices (one backend each), so nothing here is cached
// for "the" device.
constexpr int kMaxDevices = 64;
std::mutex g_dev_mu;
std::atomic<int> g_dev_state[kMaxDevices];
int g_dev_cus[kMaxDevices] = {0};

int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return -1;
    return dev;
}

void probe_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || dev >= n) {
        g_dev_state[dev].store(-1);
        return;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
        g_dev_state[dev].store(-1);
        return;
    }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fprintf(stderr, "ggml_mi355x: device %d is %s, this library is built for gfx950 only\n", dev,
                prop.gcnArchName);
        g_dev_state[dev].store(-1);
        return;
    }
    g_dev_cus[dev] = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    g_dev_state[dev].store(1, std::memory_order_release);
}

template <int NCOL, bool FUSEDQ, bool DEBUG>
gemv_fn pick_tm(int tmask) {
    switch (tmask) {
        case 1: return kq_gemv<NCOL, FUSEDQ, DEBUG, 1>;
        case 4: return kq_gemv<NCOL, FUSEDQ, DEBUG, 4>;
        default: return kq_gemv<NCOL, FUSEDQ, DEBUG, 7>;
    }
}

gemv_fn pick_gemv(int ncol, bool fusedq, bool debug, int tmask) {
    if (debug) return pick_tm<1, false, true>(tmask);
    if (fusedq) return pick_tm<1, true, false>(tmask);
    switch (ncol) {
        case 1: return pick_tm<1, false, false>(tmask);
        case 2: return pick_tm<2, false, false>(tmask);
        case 4: return pick_tm<4, false, false>(tmask);
        default: return pick_tm<8, false, false>(tmask);
    }
}

int type_bit(int type) { return type == Q4_K ? 1 : type == Q5_K ? 2 : type == Q6_K ? 4 : 0; }

constexpr size_t kMaxLds = 160 * 1024;   // LDS per CU (one workgroup may use it all)
constexpr size_t kTargetLds = 80 * 1024; // aim for >= 2 resident workgroups per CU
constexpr int64_t kFusedQMaxNb = 32;      // kq_gemv: in-kernel quantization up to K = 8192
constexpr int64_t kRowsFusedMaxNb = ROWS_QPASS * 4 * ROWS_WAVES;  // kq_rows: up to K = 36864
// launches below this many weight bytes: ROWS_WAVES_SMALL waves. 10 MB -> 5 MB in round 5
// (TinyLlama's 6.5 / 9.5 MB ffn_down and the 8B's 9.4 MB o-proj on 12 waves): both tokens
// +0.3 %, six of six interleaved comparisons; 0 (never) -0.8 % (profiles/r05_gemv_small_mb_ab.txt)
constexpr double kRowsSmallBytes = 5e6;
std::atomic<int> g_rows_waves{0};         // mi355x_gemv_waves: 0 = by size, else fixed

// ------------------------------------------------------------------ debug knobs
// Product defaults; mi355x_debug_knob() (tools / A/B runs) overrides them per process.
struct KnobDef {
    const char *name;
    double def;
};
const KnobDef kKnobs[KNOB_COUNT] = {
    {"GEMV_DIAG", 0},  {"GEMV_RING", 0},     {"GEMV_PRE0", 1},       {"GEMV_PF", 0},
    {"GEMV_XMODE", 0}, {"GEMV_SMALL_MB", kRowsSmallBytes / 1e6},      {"GEMV_WPC", 0},
    {"GEMV_SMALL_WG", 0}, {"GEMV_FQMAX", (double)kRowsFusedMaxNb},   {"MMF_WAVES", 0},
    {"MMF_ORDER", 0},  {"ATTN_DIAG", 0},     {"LOOPBACK_NOCOPY", 0}, {"ATTN_OPROJ", 1},
    {"AO_NRB", 0},     {"GEMV_DYN", 8},    {"GEMV_DYN_P", 0},      {"GEMV_DYN_STEPS", 16},
};
std::atomic<double> g_knob[KNOB_COUNT];
std::atomic<bool> g_knob_set[KNOB_COUNT];
std::atomic<uint32_t> g_knob_gen{0};


uint64_t *g_stamps = nullptr;  // diagnostics (mi355x_diag_stamps)
int64_t g_stamps_cap = 0;

// Workgroups of one kernel resident per CU (registers / LDS), cached per
// (device, fn, lds): function attributes are set per device.
struct OccKey {
    int dev;
    const void *fn;
    size_t lds;
};
int resident_wgs(const void *fn, size_t lds) {
    static std::mutex mu;
    static std::vector<std::pair<OccKey, int>> cache;
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(mu);
    for (auto &e : cache)
        if (e.first.dev == dev && e.first.fn == fn && e.first.lds == lds) return e.second;
    int n = 0;
    if (lds > 64 * 1024) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, WG_THREADS, lds) != hipSuccess || n <= 0) n = 1;
    if (n > 8) n = 8;
    cache.push_back({{dev, fn, lds}, n});
    return n;
}

}  // namespace

double knob(Knob k) { return g_knob_set[k].load(std::memory_order_relaxed) ? g_knob[k].load() : kKnobs[k].def; }
uint32_t knob_generation() { return g_knob_gen.load(); }

// ------------------------------------------------------------ launch timing
struct TimedLaunch {
    std::string kernel;
    double bytes;
    hipEvent_t start, stop;
};
std::mutex g_tmu;
bool g_timing = false;
std::vector<TimedLaunch> g_tlog;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_tpool;
size_t g_tpool_used = 0;

bool capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) return false;
    return st != hipStreamCaptureStatusNone;
}

// Returns true (and the events) when this launch should be timed.
bool timing_slot(hipStream_t s, hipEvent_t &a, hipEvent_t &b) {
    std::lock_guard<std::mutex> lk(g_tmu);
    if (!g_timing || capturing(s)) return false;
    if (g_tpool_used == g_tpool.size()) {
        hipEvent_t e0, e1;
        if (hipEventCreate(&e0) != hipSuccess) return false;
        if (hipEventCreate(&e1) != hipSuccess) {
            hipEventDestroy(e0);
            return false;
        }
        g_tpool.push_back({e0, e1});
    }
    a = g_tpool[g_tpool_used].first;
    b = g_tpool[g_tpool_used].second;
    ++g_tpool_used;
    return true;
}

void timing_log(const std::string &kernel, double bytes, hipEvent_t a, hipEvent_t b) {
    std::lock_guard<std::mutex> lk(g_tmu);
    g_tlog.push_back({kernel, bytes, a, b});
}

namespace {

// Same spelling as rocprofv3's kernel names (kernel-trace "Kernel_Name").
std::string gemv_name(const GemvPlan &pl) {
    return std::string("kq::kq_gemv<") + std::to_string(pl.ncol) + ", " + (pl.fusedq ? "true" : "false") + ", " +
           (pl.debug ? "true" : "false") + ", " + std::to_string(pl.tmask) + ">";
}

// Algorithmic bytes of one launch: weights + activations read + f32 outputs.
double gemv_bytes(const GemvArgs &a, bool fusedq) {
    double w = 0, y = 0;
    for (int i = 0; i < a.n_desc; ++i) {
        w += (double)a.n_rows[i] * a.nb * block_bytes(a.type[i]);
        y += (double)a.n_rows[i] * 4.0 * a.m_total;
    }
    const double x = fusedq ? (double)a.nb * QK * 4.0 * a.m_total : (double)a.nb * 292.0 * a.m_total;
    return w + x + y;
}

}  // namespace

int device_ok() {
    const int dev = current_device();
    if (dev < 0) return 0;
    const int st = g_dev_state[dev].load(std::memory_order_acquire);
    if (st) return st > 0;
    std::lock_guard<std::mutex> lk(g_dev_mu);
    if (g_dev_state[dev].load() == 0) probe_device(dev);
    return g_dev_state[dev].load() > 0;
}

int num_cus() {
    if (!device_ok()) return 256;
    return g_dev_cus[current_device()];
}

int choose_ncol(int64_t M, int nb) {
    if (M <= 1) return 1;
    const int cands[4] = {8, 4, 2, 1};
    for (int i = 0; i < 4; ++i) {
        const int nc = cands[i];
        if (nc > M && nc > 1) continue;
        if ((size_t)lds_layout(nc, nb, 8 * nc, false, 8 * 16 * 14, 4).total <= kTargetLds) return nc;
    }
    return 1;
}

// Validates descriptors and fills the launch plan. Returns MI355X_OK or an error.
int plan_gemv(const mi355x_gemv_desc *d, int n_desc, int64_t K, int64_t M, int ncol, bool fusedq, bool debug,
              GemvPlan &pl) {
    GemvArgs &a = pl.a;
    if (n_desc < 1 || n_desc > MI355X_MAX_FUSED) return MI355X_E_INVAL;
    if (K <= 0 || K % QK != 0 || M < 0) return MI355X_E_INVAL;
    const int64_t nb = K / QK;
    if (nb > 0x7fffffff / 8) return MI355X_E_INVAL;
    memset(&a, 0, sizeof(a));
    int tmask = 0;
    for (int i = 0; i < n_desc; ++i) {
        const int bb = block_bytes(d[i].type);
        if (!bb) return MI355X_E_UNSUPPORTED;
        if (d[i].n_rows < 0 || d[i].n_rows > 0x7fffffff) return MI355X_E_INVAL;
        if (d[i].n_rows > 0) {
            if (!d[i].w || !d[i].y) return MI355X_E_INVAL;
            if (((uintptr_t)d[i].w & 3u) != 0) return MI355X_E_INVAL;
            if (d[i].row_stride < (size_t)(nb * bb) || (d[i].row_stride & 1u)) return MI355X_E_INVAL;
            if (d[i].type != Q6_K && (d[i].row_stride & 3u)) return MI355X_E_INVAL;
        }
        tmask |= type_bit(d[i].type);
    }
    if (tmask != 1 && tmask != 4) tmask = 7;
    a.n_desc = n_desc;
    a.nb = (int)nb;
    a.R = BLOCKS_PER_STEP;
    a.m_total = (int)M;
    int64_t tasks = 0;
    for (int i = 0; i < n_desc; ++i) {
        a.type[i] = d[i].type;
        a.n_rows[i] = (int)d[i].n_rows;
        a.w[i] = (const uint8_t *)d[i].w;
        a.row_stride[i] = (int64_t)d[i].row_stride;
        a.y[i] = d[i].y;
        a.task_prefix[i] = (int)tasks;
        tasks += (d[i].n_rows + a.R - 1) / a.R;
    }
    if (tasks > 0x7fffffff) return MI355X_E_INVAL;
    for (int i = n_desc; i <= MI355X_MAX_FUSED; ++i) a.task_prefix[i] = (int)tasks;
    a.tasks_total = (int)tasks;
    pl.ncol = ncol;
    pl.fusedq = fusedq;
    pl.debug = debug;
    pl.tmask = tmask;
    pl.fn = pick_gemv(ncol, fusedq, debug, tmask);
    a.diag = (int)knob(KNOB_GEMV_DIAG);
    a.ring_override = (int)knob(KNOB_GEMV_RING);
    a.stamps = g_stamps;
    a.stamps_cap = g_stamps_cap;
    // One workgroup per 8-row task, at most one round of resident workgroups; each
    // workgroup strides over tasks. Ring depth: as deep as LDS allows 2+ resident
    // workgroups per CU. Staged outputs bound the tasks per workgroup.
    const int slot = tmask == 1 ? 8 * 16 * 9 : 8 * 16 * 14;
    const int dcands[3] = {tmask == 1 ? 8 : 6, tmask == 1 ? 6 : 5, 4};
    int D = 4;
    for (int i = 0; i < 3; ++i) {
        D = dcands[i];
        if ((size_t)lds_layout(ncol, (int)nb, 8 * ncol, fusedq, slot, D).total <= kTargetLds) break;
    }
    if (a.ring_override > 0) D = a.ring_override < 13 ? a.ring_override : 13;
    a.ring = D;
    const int64_t base_lds = lds_layout(ncol, (int)nb, 0, fusedq, slot, D).total;
    if ((size_t)base_lds > kMaxLds) return MI355X_E_UNSUPPORTED;
    int64_t wgs = (int64_t)num_cus() * resident_wgs((const void *)pl.fn, (size_t)base_lds + 1024);
    if (wgs > tasks) wgs = tasks > 0 ? tasks : 1;
    int64_t tpw = (tasks + wgs - 1) / wgs;
    while (tpw * 8 * ncol * 4 > 4096 && tpw > 1) {
        wgs *= 2;
        tpw = (tasks + wgs - 1) / wgs;
    }
    a.out_per_wg = (int)(tpw * 8 * ncol);
    const LdsLayout L = lds_layout(ncol, (int)nb, a.out_per_wg, fusedq, slot, D);
    if ((size_t)L.total > kMaxLds) return MI355X_E_UNSUPPORTED;
    pl.lds = (size_t)L.total;
    pl.grid = dim3((unsigned)wgs, (unsigned)((M + ncol - 1) / ncol), 1);
    return MI355X_OK;
}

// Dynamic LDS above 64 KB must be opted into per kernel.
void allow_lds(const void *fn, size_t lds) {
    if (lds <= 64 * 1024) return;
    static std::mutex mu;
    static std::vector<std::pair<int, const void *>> done;  // (device, fn): set per device
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(mu);
    for (auto &e : done)
        if (e.first == dev && e.second == fn) return;
    hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds);
    done.push_back({dev, fn});
}

int launch_gemv(const GemvPlan &pl, hipStream_t stream) {
    const GemvArgs &a = pl.a;
    if (a.tasks_total == 0 || a.m_total == 0) return MI355X_OK;
    allow_lds((const void *)pl.fn, pl.lds);
    hipEvent_t e0, e1;
    if (timing_slot(stream, e0, e1)) {
        hipExtLaunchKernelGGL(pl.fn, pl.grid, dim3(WG_THREADS), (uint32_t)pl.lds, stream, e0, e1, 0, a);
        timing_log(gemv_name(pl), gemv_bytes(a, pl.fusedq), e0, e1);
    } else {
        hipLaunchKernelGGL(pl.fn, pl.grid, dim3(WG_THREADS), pl.lds, stream, a);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

// ------------------------------------------------------------ row-stream decode GEMV
std::atomic<int> g_impl{MI355X_GEMV_AUTO};
bool rows_enabled() {
    return g_impl.load() != MI355X_GEMV_TASKS;  // mi355x_gemv_impl()
}


template <int TM, bool FQ, int PR>
rows_fn rows_inst(bool dyn) {
    if constexpr (TM == 7) {
        return kq_rows<TM, FQ, PR>;
    } else {
        return dyn ? kq_rows_dyn<TM, FQ, PR> : kq_rows<TM, FQ, PR>;
    }
}

template <int TM>
rows_fn rows_pick_pro(bool fusedq, int pro, bool dyn) {
    if (!fusedq) return rows_inst<TM, false, 0>(dyn);
    return pro == ROWS_PRO_NORM ? rows_inst<TM, true, 1>(dyn) : pro == ROWS_PRO_SWIGLU ? rows_inst<TM, true, 2>(dyn)
                                                                                       : rows_inst<TM, true, 0>(dyn);
}

rows_fn pick_rows(int tmask, bool fusedq, int pro, bool dyn = false) {
    switch (tmask) {
        case 1: return rows_pick_pro<1>(fusedq, pro, dyn);
        case 2: return rows_pick_pro<2>(fusedq, pro, dyn);
        case 4: return rows_pick_pro<4>(fusedq, pro, dyn);
        default: return rows_pick_pro<7>(fusedq, pro, false);
    }
}

int plan_rows(const mi355x_gemv_desc *d, int n_desc, int64_t K, bool fusedq, RowsPlan &pl, int waves_per_cu) {
    RowsArgs &a = pl.a;
    if (n_desc < 1 || n_desc > MI355X_MAX_FUSED) return MI355X_E_INVAL;
    if (K <= 0 || K % QK != 0) return MI355X_E_INVAL;
    const int64_t nb = K / QK;
    if (nb > 4096) return MI355X_E_UNSUPPORTED;
    if (fusedq && nb > kRowsFusedMaxNb) return MI355X_E_UNSUPPORTED;
    memset(&a, 0, sizeof(a));
    int tmask = 0;
    double bytes_total = 0;
    for (int i = 0; i < n_desc; ++i) {
        const int bb = block_bytes(d[i].type);
        if (!bb) return MI355X_E_UNSUPPORTED;
        if (d[i].n_rows < 0 || d[i].n_rows > 0x7fffffff) return MI355X_E_INVAL;
        if (d[i].n_rows > 0) {
            if (!d[i].w || !d[i].y) return MI355X_E_INVAL;
            if (((uintptr_t)d[i].w & 3u) != 0) return MI355X_E_INVAL;
            // one contiguous stream per wave; Q4_K/Q5_K superblocks 16-B aligned in LDS
            if (d[i].row_stride != (size_t)(nb * bb)) return MI355X_E_UNSUPPORTED;
            if (d[i].type != Q6_K && ((uintptr_t)d[i].w & 15u)) return MI355X_E_UNSUPPORTED;
        }
        bytes_total += (double)d[i].n_rows * bb;
        tmask |= type_bit(d[i].type);
    }
    if (tmask != 1 && tmask != 2 && tmask != 4) tmask = 7;
    pl.tmask = tmask;
    pl.fusedq = fusedq;
    pl.fn = pick_rows(tmask, fusedq, ROWS_PRO_NONE);
    a.n_desc = n_desc;
    a.nb = (int)nb;
    for (int i = 0; i < n_desc; ++i) {
        a.type[i] = d[i].type;
        a.w[i] = (const uint8_t *)d[i].w;
        a.y[i] = d[i].y;
        a.n_rows[i] = (int)d[i].n_rows;
    }
    {
        a.pf = (int)knob(KNOB_GEMV_PF);
        a.xmode = (int)knob(KNOB_GEMV_XMODE) & 7;
        a.diag = (int)knob(KNOB_GEMV_DIAG);
        // weight steps issued before the activation is quantized. One: a deeper early burst
        // delays the activation loads queued behind it. Alone, K = 2048 GEMVs ran 5-9 %
        // faster with the whole ring (tools/gemv_sweep.py pre0=3), but with the fused norm
        // prologue (two vectors to fetch) the decode token was 1.6 % slower.
        const int pre = (int)knob(KNOB_GEMV_PRE0);
        a.pre0 = pre < 0 ? 0 : pre > 3 ? 3 : pre;
    }
    a.stamps = g_stamps;
    a.stamps_cap = g_stamps_cap;
    // Waves: one workgroup per CU of ROWS_WAVES waves, or of ROWS_WAVES_SMALL for a launch
    // under kRowsSmallBytes of weights (measured on the graph-replayed token: fewer waves
    // to dispatch, the short stream does not need them; profiles/r02_rows_waves.md). Each
    // matrix gets waves in proportion to its bytes (never more waves than rows), rows
    // split evenly.
    const double small_bytes = knob(KNOB_GEMV_SMALL_MB) * 1e6;  // (0: never)
    if (waves_per_cu <= 0) {
        const int fixed = g_rows_waves.load();
        const int want = fixed > 0 ? fixed : bytes_total * nb < small_bytes ? ROWS_WAVES_SMALL : ROWS_WAVES;
        // the fused quantization covers ROWS_QPASS passes of 4 superblocks per wave
        waves_per_cu = !fusedq || nb <= ROWS_QPASS * 4 * want ? want : ROWS_WAVES;
    }
    if (waves_per_cu > ROWS_WAVES) return MI355X_E_INVAL;
    pl.nwv = waves_per_cu;
    const int wpc_env = (int)knob(KNOB_GEMV_WPC);  // experiment knob: cap on active waves per CU
    if (wpc_env > 0 && wpc_env < waves_per_cu) waves_per_cu = wpc_env;
    // workgroups: one per CU; an A/B knob caps it for small launches (GEMV_SMALL_WG)
    const int small_wg_env = (int)knob(KNOB_GEMV_SMALL_WG);
    int64_t n_wg = num_cus();
    if (small_wg_env > 0 && bytes_total * nb < small_bytes && small_wg_env < n_wg) n_wg = small_wg_env;
    const int64_t cap = n_wg * waves_per_cu;
    int64_t wv[MI355X_MAX_FUSED] = {0, 0, 0, 0};
    int64_t waves = 0;
    for (int i = 0; i < n_desc; ++i) {
        if (d[i].n_rows == 0) continue;
        const double share = (double)d[i].n_rows * block_bytes(d[i].type) / bytes_total;
        int64_t w = (int64_t)(share * (double)cap);
        // at least one full 16-superblock step per wave (short rows: several rows per wave)
        const int64_t min_rows = (ROWS_SB + nb - 1) / nb;
        const int64_t wmax = (d[i].n_rows + min_rows - 1) / min_rows;
        if (w > wmax) w = wmax;
        if (w < 1) w = 1;
        wv[i] = w;
        waves += w;
    }
    while (waves > cap) {  // the max(1, .) floors may overshoot by < n_desc: trim the largest
        int big = 0;
        for (int i = 1; i < n_desc; ++i)
            if (wv[i] > wv[big]) big = i;
        --wv[big];
        --waves;
    }
    int64_t rpw = 0;
    waves = 0;
    for (int i = 0; i < n_desc; ++i) {
        a.wave_prefix[i] = (int)waves;
        if (wv[i] > 0) {
            a.rbase[i] = (int)(d[i].n_rows / wv[i]);
            a.rrem[i] = (int)(d[i].n_rows % wv[i]);
            const int64_t r = a.rbase[i] + (a.rrem[i] ? 1 : 0);
            rpw = r > rpw ? r : rpw;
        }
        waves += wv[i];
    }
    for (int i = n_desc; i <= MI355X_MAX_FUSED; ++i) a.wave_prefix[i] = (int)waves;
    a.waves_total = (int)waves;
    a.prio_bytes = 0;
    for (int i = 0; i < n_desc; ++i)
        if (wv[i] > 0) {
            const int64_t b = (int64_t)(a.rbase[i] + (a.rrem[i] ? 1 : 0)) * nb * block_bytes(d[i].type);
            a.prio_bytes = b > a.prio_bytes ? b : a.prio_bytes;
        }
    if (rpw > 0x7fffffff / 64) return MI355X_E_UNSUPPORTED;
    a.rpw = (int)(rpw > 0 ? rpw : 1);
    // rows per chain batch: ~ROWS_RECS records, batch ends on a step boundary (bR*nb % 16 == 0)
    int g16 = ROWS_SB;
    while (nb % g16) g16 >>= 1;
    const int u = ROWS_SB / g16;
    int bR_full = (int)(ROWS_RECS / nb) / u * u;
    if (bR_full < u) bR_full = u;
    a.bR = a.rpw <= bR_full ? a.rpw : bR_full;
    const RowsLayout L = rows_layout((int)nb, tmask, a.bR, a.rpw, pl.nwv);
    if ((size_t)L.total > kMaxLds) return MI355X_E_UNSUPPORTED;
    pl.lds = (size_t)L.total;
    const int64_t grid = waves < n_wg ? waves : n_wg;
    pl.grid = dim3((unsigned)(grid > 0 ? grid : 1), 1, 1);
    // Claimed rows (kq_rows_dyn) for one-type launches whose waves get enough units to balance
    // (GEMV_DYN units per wave on average; MI355X_GEMV_DYN: every one-type launch). A unit is
    // U whole rows of at least one 16-superblock step; each wave's first P units (a ring's
    // worth) are static.
    pl.dyn = false;
    const double dyn_min = knob(KNOB_GEMV_DYN);
    const bool force = g_impl.load() == MI355X_GEMV_DYN;
    bool same_rows = true;  // kq_rows_dyn: one workgroup row range for every matrix
    for (int i = 1; i < n_desc; ++i) same_rows = same_rows && d[i].n_rows == d[0].n_rows;
    if (tmask != 7 && same_rows && (force || dyn_min > 0)) {
        // U: whole rows, a power of two, at least one 16-superblock step; two steps where every
        // wave streams many (a claim and a unit's bookkeeping per two steps)
        int ush = 0;
        while ((int64_t)(1 << ush) * nb < ROWS_SB) ++ush;
        const double steps_per_wave = (double)n_desc * d[0].n_rows * nb / ROWS_SB / n_wg / pl.nwv;
        if ((int64_t)(1 << ush) * nb == ROWS_SB && steps_per_wave >= 16) ++ush;
        const int U = 1 << ush;
        const int Tu = (int)((U * nb + ROWS_SB - 1) / ROWS_SB);
        const int D = rows_depth(tmask == 1 ? Q4_K : tmask == 2 ? Q5_K : Q6_K);
        // flat output slots per workgroup: its row units (strided placement) or rows, per matrix
        const int64_t flat = (int64_t)n_desc * ((d[0].n_rows + n_wg - 1) / n_wg);
        const int64_t rows = (int64_t)n_desc * d[0].n_rows;
        // replay batch: ~ROWS_RECS records, whole units
        int bRd = (int)(ROWS_RECS / nb) / U * U;
        if (bRd < U) bRd = U;
        // AUTO (profiles/r06_dyn_ab.txt): claimed rows paid where every wave streams many steps
        // in many units (the Q6_K heads, 70B gate + up: -1 to -3 %); with few units per wave
        // (8B ffn_up, 70B ffn_down: +5 to +10 %) the units' bookkeeping costs more than the
        // balance gains
        const double per_wave = (double)rows / (double)n_wg / U / pl.nwv;
        const bool auto_ok = per_wave >= dyn_min && steps_per_wave >= knob(KNOB_GEMV_DYN_STEPS);
        const RowsDynLayout DL = rows_dyn_layout((int)nb, tmask, bRd, (int)flat, pl.nwv);
        if ((force || auto_ok) && rows > 0 && (size_t)DL.total <= kMaxLds && flat < 0x7fffffff / 64) {
            pl.dyn = true;
            a.dyn_u = U;
            a.dyn_ush = ush;
            a.rbase[0] = (int)(d[0].n_rows / n_wg);
            a.rrem[0] = (int)(d[0].n_rows % n_wg);
            a.dyn_p = (D + Tu - 1) / Tu;
            const int p_knob = (int)knob(KNOB_GEMV_DYN_P);
            if (p_knob > 0) a.dyn_p = p_knob;
            a.bR = bRd;
            a.rpw = (int)flat;
            pl.lds = (size_t)DL.total;
            pl.grid = dim3((unsigned)n_wg, 1, 1);
            pl.fn = pick_rows(tmask, fusedq, ROWS_PRO_NONE, true);
        }
    }
    return MI355X_OK;
}

std::string rows_name(const RowsPlan &pl) {
    return std::string(pl.dyn ? "kq::kq_rows_dyn<" : "kq::kq_rows<") + std::to_string(pl.tmask) + ", " + (pl.fusedq ? "true" : "false") + ", " +
           std::to_string(pl.a.pro) + ">";
}

double rows_bytes(const RowsArgs &a, bool fusedq) {
    double w = 0, y = 0;
    for (int i = 0; i < a.n_desc; ++i) {
        const double rows = (double)a.n_rows[i];
        w += rows * a.nb * block_bytes(a.type[i]);
        y += rows * 4.0;
    }
    return w + y + (fusedq ? (double)a.nb * QK * 4.0 : (double)a.nb * Q8L_STRIDE);
}

int launch_rows(const RowsPlan &pl, hipStream_t stream) {
    const RowsArgs &a = pl.a;
    if (a.waves_total == 0) return MI355X_OK;
    allow_lds((const void *)pl.fn, pl.lds);
    hipEvent_t e0, e1;
    if (timing_slot(stream, e0, e1)) {
        hipExtLaunchKernelGGL(pl.fn, pl.grid, dim3(pl.nwv * 64), (uint32_t)pl.lds, stream, e0, e1, 0, a);
        timing_log(rows_name(pl), rows_bytes(a, pl.fusedq), e0, e1);
    } else {
        hipLaunchKernelGGL(pl.fn, pl.grid, dim3(pl.nwv * 64), pl.lds, stream, a);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

int launch_quantize_q8L(const float *x, int64_t x_stride_floats, void *y, int64_t k, int64_t nrows,
                        hipStream_t stream, bool mmq) {
    const auto kern = mmq ? kq_quantize_q8L<true> : kq_quantize_q8L<false>;
    const int64_t nb = k / QK;
    const int64_t nblocks = nb * nrows;
    if (nblocks == 0) return MI355X_OK;
    const int64_t wgs = (nblocks + 15) / 16;
    hipEvent_t e0, e1;
    if (timing_slot(stream, e0, e1)) {
        hipExtLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(WG_THREADS), 0, stream, e0, e1, 0, x,
                              x_stride_floats, (uint8_t *)y, (int)nb, nblocks);
        timing_log("kq::kq_quantize_q8L", (double)nblocks * (QK * 4.0 + Q8L_STRIDE), e0, e1);
    } else {
        hipLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(WG_THREADS), 0, stream, x, x_stride_floats,
                           (uint8_t *)y, (int)nb, nblocks);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

// ------------------------------------------------------------ batched MFMA path
constexpr int64_t kMmqMinCols = 16;  // below this the NCOL GEMV streams the weights fewer times

// Prefill kernel selector (mi355x_mmq_impl): -1 until first read from MI355X_MMQ_IMPL.
// Round 3 removed the streamed Q4_K kernel (kq_mmq_k4): equal to the 64 x 64 tiles
// within the box spread at pp512, 17-40 % slower on every shape forced onto it
// (profiles/r02_mmq_impl_ab.txt); AUTO and TILE64 now both select the 64 x 64 tiles.
std::atomic<int> g_mmq_impl{MI355X_MMQ_AUTO};  // mi355x_mmq_impl()
int mmq_impl() { return g_mmq_impl.load(); }

// Prefill tile shape (kq_mmq's RT x CW): weight rows per workgroup RT = 64 (4 waves) or 128
// (8 waves: the activation tile fetched once per 128 rows), activation columns 64 * CW (CW = 2:
// each wave's weight operands feed two MFMA column tiles, half the operand-building vector
// work per MFMA). AUTO, by the grid each shape would launch (profiles/r03_mmq_tiles.txt):
//  * a grid of >= 160 workgroups at 128 x 128: 128 x 128 (TinyLlama Q6_K head 256 -> 167 us,
//    gate/up 28.3 -> 26.0, 8B ffn_up 98 -> 95, 8B Q5_K ffn_up 147 -> 125); on 128-workgroup
//    grids it loses 30-40 % (half the CUs idle);
//  * else Q6_K whose 64 x 128 grid has >= 192 workgroups: 64 x 128 (one 4-wave workgroup
//    per CU, every register: 8B Q6_K ffn_down 219-226 -> 192-194 us; Q4_K / Q5_K are slower
//    on it);
//  * else Q4_K / Q5_K whose 128 x 64 grid has >= 256 workgroups: 128 x 64 (8B q/o 33 -> 31,
//    ffn_down 108-116 -> 101-106; Q5_K q/o 42.4 -> 40.5, ffn_down 132 -> 128 with the
//    three-MFMA Q5_K split, profiles/r03_mmq_q5_tiles.txt);
//  * else 64 x 64 (small grids).
struct MmqShape {
    int rt, cw;
};
MmqShape mmq_shape(int type, int64_t rows, int64_t M) {
    const int impl = mmq_impl();
    if (impl == MI355X_MMQ_TILE128) return {128, 1};
    if (impl == MI355X_MMQ_TILE128W) return {128, 2};
    if (impl == MI355X_MMQ_TILE64W) return {64, 2};
    if (impl == MI355X_MMQ_TILE64) return {64, 1};
    if (impl == MI355X_MMQ_TILE128X) return {128, type == Q6_K ? 2 : 4};
    if (impl == MI355X_MMQ_TILE192) return type == Q6_K ? MmqShape{128, 1} : MmqShape{192, 1};
    const int64_t rt128 = (rows + 127) / 128;
    const int64_t g128x128 = rt128 * ((M + 127) / 128), g128x64 = rt128 * ((M + 63) / 64);
    // a 128 x 128 grid that fills under ~3/4 of two workgroups per CU, where the 128 x 64 one
    // has two per CU: 128 x 64 (TinyLlama's 11264-row gate+up at M = 512: 352 against 704
    // workgroups, 49.8 -> 41.6 us; Llama-3-8B ffn_up's 448 keep 128 x 128, 95 against 97 us;
    // profiles/r05_mmq_tl_tiles.txt)
    if (type != Q6_K && g128x128 >= 160 && g128x128 < 384 && g128x64 >= 512) return {128, 1};
    if (g128x128 >= 160) return {128, 2};
    if (type == Q6_K && ((rows + 63) / 64) * ((M + 127) / 128) >= 192) return {64, 2};
    if (type != Q6_K && rt128 * ((M + 63) / 64) >= 256) return {128, 1};
    return {64, 1};
}
const void *mmq_fn(int type, bool mixed, MmqShape sh) {
#define KQ_MMQ_PICK(RT, CW)                                                      \
    return mixed          ? (const void *)kq_mmq_mixed<RT, CW>                 \
         : type == Q5_K ? (const void *)kq_mmq<Q5_K, RT, CW>                   \
         : type == Q6_K ? (const void *)kq_mmq<Q6_K, RT, CW>                   \
                        : (const void *)kq_mmq<Q4_K, RT, CW>;
    if (sh.rt == 192 && !mixed && type != Q6_K)
        return type == Q5_K ? (const void *)kq_mmq<Q5_K, 192, 1> : (const void *)kq_mmq<Q4_K, 192, 1>;
    if (sh.rt == 128 && sh.cw == 4 && !mixed && type != Q6_K)
        return type == Q5_K ? (const void *)kq_mmq<Q5_K, 128, 4> : (const void *)kq_mmq<Q4_K, 128, 4>;
    if (sh.rt == 128 && sh.cw == 2) KQ_MMQ_PICK(128, 2)
    if (sh.rt == 64 && sh.cw == 2) KQ_MMQ_PICK(64, 2)
    if (sh.rt == 128) KQ_MMQ_PICK(128, 1)
    KQ_MMQ_PICK(64, 1)
#undef KQ_MMQ_PICK
}
// two superblock buffers: mmq_cols(cw) Q8L columns + rt weight rows (Q6_K: KQ_MMQ_Q6_STRIDE, the 224-B granule span + padding),
// +16 B for the Q6_K realign reads past the last row
size_t mmq_lds(int type, MmqShape sh) {
    return (size_t)mmq_nbuf(type, sh.rt, sh.cw) * (size_t)mmq_buf_bytes(type, sh.rt, sh.cw) + 16 + MMQ_PF_LDS;
}

int launch_mmq(int type, const void *w, int64_t K, int64_t N, size_t row_stride, const uint8_t *xq, int64_t M,
               float *y, int64_t y_col_stride, hipStream_t stream, const float *res, int64_t res_col_stride) {
    MmqArgs a;
    memset(&a, 0, sizeof(a));
    a.n_mat = 1;
    a.res = res;
    a.res_col_stride = res_col_stride;
    a.w = (const uint8_t *)w;
    a.row_stride = (int64_t)row_stride;
    a.n_rows = (int)N;
    a.xq = xq;
    a.nb = (int)(K / QK);
    a.xq_col_stride = (int64_t)a.nb * Q8L_STRIDE;
    a.m_cols = (int)M;
    a.y = y;
    a.y_col_stride = y_col_stride;
    const MmqShape sh = mmq_shape(type, N, M);
    const void *fn = mmq_fn(type, false, sh);
    const size_t lds = mmq_lds(type, sh);
    const int cols = mmq_cols(sh.cw);
    dim3 grid((unsigned)((M + cols - 1) / cols), (unsigned)((N + sh.rt - 1) / sh.rt), 1);
    dim3 block((unsigned)(64 * mmq_waves(sh.rt, sh.cw)));
    std::string name = std::string("kq::kq_mmq<") + std::to_string(type) + ">";
    allow_lds(fn, lds);
    hipEvent_t e0, e1;
    const bool timed = timing_slot(stream, e0, e1);
    void *args[] = {&a};
    hipError_t e;
    if (timed) {
        e = hipExtLaunchKernel(fn, grid, block, args, lds, stream, e0, e1, 0);
        timing_log(name, (double)N * a.nb * block_bytes(type) + (double)M * a.nb * Q8L_STRIDE + (double)M * N * 4.0,
                   e0, e1);
    } else {
        e = hipLaunchKernel(fn, grid, block, args, lds, stream);
    }
    if (e != hipSuccess) return (int)e;
    e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

// ------------------------------------------- prefill on the f16 matrix core (stated tolerance)
// mi355x_prefill_precision: MI355X_PREFILL_EXACT (kq_mmq, bit-exact, the default) or
// MI355X_PREFILL_F16 (kq_mmf: the reference's Q8_K activation and integer unpacking, the
// accumulated dot on v_mfma_f32_32x32x16_f16 within the tolerance of kq_mmf.hip's header).
// Set only through mi355x_prefill_precision(): the numerics never change from the environment.
std::atomic<int> g_prefill{MI355X_PREFILL_EXACT};
int prefill_precision() { return g_prefill.load(); }

// Waves per kq_mmf workgroup (MI355X_MMF_WAVES, A/B only): 4 (128-row workgroups, two per
// CU) or 8 (256-row workgroups, one per CU); 0 by shape: 8 from K >= 8192, where the
// activation tile's refill is the longer wait (8B ffn_down Q4_K 99-106 -> 88-96 us, Q6_K
// 134 -> 117-122, Q5_K 104 -> 93), 4 below it (8B ffn_up 82.5 vs 99.7 us on 8 waves:
// its 224-workgroup grid leaves CUs idle) -- profiles/r03_mmf_waves_ab.txt.
int mmf_nw(int64_t K) {
    const int v = (int)knob(KNOB_MMF_WAVES);
    return v == 4 || v == 8 ? v : K >= 8192 ? 8 : 4;
}
// K split of kq_mmf: double it while the grid has fewer workgroups than CUs and every
// split keeps >= 4 superblocks (8 half-superblock steps); splits combine in order (NW = 4:
// filling both resident slots per CU with a 4-way split measured slower on 8B q/o, 34 ->
// 37 us).
struct MmfPlan {
    int nw, n_ct, n_rt, n_split, nbs;
};
MmfPlan mmf_plan_nw(int64_t N, int64_t M, int64_t nb, int nw) {
    MmfPlan p;
    p.nw = nw;
    p.n_ct = (int)((M + MMF_COLS - 1) / MMF_COLS);
    p.n_rt = (int)((N + 32 * nw - 1) / (32 * nw));
    int s = 1;
    while ((int64_t)p.n_ct * p.n_rt * s < 256 && nb >= 8 * s) s *= 2;
    p.nbs = (int)((nb + s - 1) / s);
    p.n_split = (int)((nb + p.nbs - 1) / p.nbs);
    return p;
}
size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }
// workspace: activation image + d*bsum16 (+ the split-K slabs of either tile shape)
size_t mmf_workspace(int64_t N, int64_t M, int64_t nb) {
    size_t w = al256((size_t)M * nb * MMF_IMG) + al256((size_t)M * nb * MMF_BSB), slab = 0;
    for (int nw = 4; nw <= 8; nw += 4) {
        const MmfPlan p = mmf_plan_nw(N, M, nb, nw);
        const size_t sb = p.n_split > 1 ? al256((size_t)p.n_split * M * N * 4) : 0;
        slab = sb > slab ? sb : slab;
    }
    return w + slab;
}
// Where the f16 path is the faster one (M = 512, profiles/r03_mmf_*): Q5_K and Q6_K
// everywhere; Q4_K from N*K >= 32 M elements (8B ffn_up / ffn_down), while the int8 tiles
// stay ahead on the smaller Q4_K GEMMs (8B q/o 36 vs 38 us, TinyLlama gate 31 vs 36 us).
// The precision switch promises the stated tolerance, which the bit-exact kernel meets
// trivially; MI355X_PREFILL_F16_ALL forces the f16 kernel on every shape (A/B, tests).
bool mmf_prefers(int type, int64_t N, int64_t K) {
    return prefill_precision() == MI355X_PREFILL_F16_ALL || type != Q4_K || N * K >= ((int64_t)32 << 20);
}
bool mmf_applies(int type, const void *w, int64_t N, size_t row_stride, int64_t M, int64_t K) {
    if (prefill_precision() < MI355X_PREFILL_F16) return false;
    if (!rows_enabled() || M < kMmqMinCols || N <= 0) return false;
    if (type != Q4_K && type != Q5_K && type != Q6_K) return false;
    if (N >= (1ll << 31) || M >= (1ll << 31)) return false;
    if (!mmf_prefers(type, N, K)) return false;
    if (type == Q6_K) return true;  // 210-B blocks: unaligned vector loads
    return ((uintptr_t)w & 15u) == 0 && (row_stride & 15u) == 0;
}

bool mmf_on() { return prefill_precision() >= MI355X_PREFILL_F16; }

int launch_f16img(const float *x, int64_t x_stride, uint8_t *ws, int64_t K, int64_t M, hipStream_t stream) {
    const int64_t nb = K / QK;
    uint8_t *img = ws, *bs = ws + al256((size_t)M * nb * MMF_IMG);
    const int64_t nblocks = nb * M;
    if (nblocks == 0) return MI355X_OK;
    const int64_t qwgs = (nblocks + WAVES_PER_WG - 1) / WAVES_PER_WG;
    hipEvent_t e0, e1;
    if (timing_slot(stream, e0, e1)) {
        hipExtLaunchKernelGGL(kq_quantize_f16img, dim3((unsigned)qwgs), dim3(WG_THREADS), 0, stream, e0, e1, 0, x,
                              x_stride, img, bs, (int)nb, nblocks);
        timing_log("kq::kq_quantize_f16img", (double)nblocks * (QK * 4.0 + MMF_IMG + MMF_BSB), e0, e1);
    } else {
        hipLaunchKernelGGL(kq_quantize_f16img, dim3((unsigned)qwgs), dim3(WG_THREADS), 0, stream, x, x_stride, img, bs,
                           (int)nb, nblocks);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

int launch_mmf_multi(int type, int n_mat, const void *const *w, const int64_t *N, const size_t *row_stride,
                     float *const *y, const int64_t *y_col_stride, int64_t K, uint8_t *ws, size_t ws_size, int64_t M,
                     hipStream_t stream, const float *res, int64_t res_col_stride) {
    if (n_mat < 1 || n_mat > 4 || (res && n_mat > 1)) return MI355X_E_INVAL;
    const int64_t nb = K / QK;
    const int nw = mmf_nw(K);
    int64_t n_total = 0, tiles = 0;
    for (int d = 0; d < n_mat; ++d) {
        n_total += N[d];
        tiles += (N[d] + 32 * nw - 1) / (32 * nw);
    }
    MmfPlan p = mmf_plan_nw(tiles * 32 * nw, M, nb, nw);  // the split by the grid's row tiles
    uint8_t *img = ws, *bs = ws + al256((size_t)M * nb * MMF_IMG);
    uint8_t *slab_at = bs + al256((size_t)M * nb * MMF_BSB);
    if (p.n_split > 1 && (size_t)(slab_at - ws) + (size_t)p.n_split * M * n_total * 4 > ws_size) {
        p.n_split = 1;  // the slabs do not fit this workspace: no K split
        p.nbs = (int)nb;
    }
    MmfArgs a;
    memset(&a, 0, sizeof(a));
    a.w = (const uint8_t *)w[0];
    a.row_stride = (int64_t)row_stride[0];
    a.n_rows = (int)n_total;
    a.img = img;
    a.bs = bs;
    a.m_cols = (int)M;
    a.y = y[0];
    a.y_col_stride = y_col_stride[0];
    a.slab = (float *)slab_at;
    a.nb = (int)nb;
    a.nbs = p.nbs;
    a.n_split = p.n_split;
    a.n_ct = p.n_ct;
    a.n_rt = (int)tiles;
    a.res = res;
    a.res_col_stride = res_col_stride;
    a.n_mat = n_mat;
    int64_t t0 = 0, r0 = 0;
    for (int d = 0; d < n_mat; ++d) {
        a.tile0[d] = (int)t0;
        a.roff[d] = (int)r0;
        a.mw[d] = (const uint8_t *)w[d];
        a.mrow_stride[d] = (int64_t)row_stride[d];
        a.mn_rows[d] = (int)N[d];
        a.my[d] = y[d];
        a.my_col_stride[d] = y_col_stride[d];
        t0 += (N[d] + 32 * nw - 1) / (32 * nw);
        r0 += N[d];
    }
    a.tile0[n_mat] = (int)t0;
    if (n_mat == 1) a.n_rows = (int)N[0];
    a.order = (int)knob(KNOB_MMF_ORDER);  // A/B only
    const void *fn = nw == 8 ? (type == Q5_K ? (const void *)kq_mmf<Q5_K, 8> : type == Q6_K ? (const void *)kq_mmf<Q6_K, 8>
                                                                                        : (const void *)kq_mmf<Q4_K, 8>)
                             : (type == Q5_K ? (const void *)kq_mmf<Q5_K, 4> : type == Q6_K ? (const void *)kq_mmf<Q6_K, 4>
                                                                                        : (const void *)kq_mmf<Q4_K, 4>);
    const size_t lds = 2 * (size_t)MMF_BUF;
    allow_lds(fn, lds);
    const dim3 grid((unsigned)((int64_t)p.n_ct * tiles * p.n_split)), block(64 * nw);
    void *args[] = {&a};
    hipEvent_t e0, e1;
    hipError_t e;
    if (timing_slot(stream, e0, e1)) {
        e = hipExtLaunchKernel(fn, grid, block, args, lds, stream, e0, e1, 0);
        timing_log(std::string("kq::kq_mmf<") + std::to_string(type) + ", " + std::to_string(nw) + ">",
                   (double)n_total * nb * block_bytes(type) + (double)M * nb * (MMF_IMG + MMF_BSB) +
                       (double)M * n_total * 4.0,
                   e0, e1);
    } else {
        e = hipLaunchKernel(fn, grid, block, args, lds, stream);
    }
    if (e != hipSuccess) return (int)e;
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    if (p.n_split > 1) {
        for (int d = 0; d < n_mat; ++d) {
            const int64_t total = M * N[d];
            const dim3 rg((unsigned)((total + 255) / 256));
            const float *sl = (const float *)slab_at + a.roff[d];
            const float *rs = n_mat == 1 ? res : nullptr;
            if (timing_slot(stream, e0, e1)) {
                hipExtLaunchKernelGGL(kq_mmf_reduce, rg, dim3(256), 0, stream, e0, e1, 0, sl, p.n_split, (int)M, (int)N[d],
                                      (int)n_total, y[d], y_col_stride[d], rs, res_col_stride);
                timing_log("kq::kq_mmf_reduce", (double)total * 4.0 * (p.n_split + 1), e0, e1);
            } else {
                hipLaunchKernelGGL(kq_mmf_reduce, rg, dim3(256), 0, stream, sl, p.n_split, (int)M, (int)N[d], (int)n_total,
                                   y[d], y_col_stride[d], rs, res_col_stride);
            }
            e = hipGetLastError();
            if (e != hipSuccess) return (int)e;
        }
    }
    return MI355X_OK;
}

int launch_mmf_gemm(int type, const void *w, int64_t K, int64_t N, size_t row_stride, uint8_t *ws, int64_t M,
                    float *y, int64_t y_col_stride, hipStream_t stream, const float *res, int64_t res_col_stride) {
    return launch_mmf_multi(type, 1, &w, &N, &row_stride, &y, &y_col_stride, K, ws, mmf_workspace(N, M, K / QK), M,
                            stream, res, res_col_stride);
}

// Whether launch_mmq would run this GEMM on the 64 x 64 tile kernel: every GEMM since the
// streamed kernel was removed (kept as the backend's batching test).
bool mmq_tile64(int type, int64_t N, int64_t M) {
    (void)type, (void)N, (void)M;
    return true;
}

// Up to 4 matrices of one type on one Q8L activation in ONE 64 x 64-tile launch (a prompt
// batch's q/k/v: the small k/v GEMMs no longer run as half-empty launches of their own).
// Mixed Q4_K / Q6_K matrices run on kq_mmq_mixed (each row tile its matrix's body).
int launch_mmq_multi(const int *types, int n_mat, const void *const *w, const int64_t *N, const size_t *row_stride,
                     float *const *y, const int64_t *y_col_stride, int64_t K, const uint8_t *xq, int64_t M,
                     hipStream_t stream, const MmqKv *kv) {
    if (n_mat < 1 || n_mat > 4) return MI355X_E_INVAL;
    const int type = types[0];
    bool mixed = false;
    for (int d = 1; d < n_mat; ++d) mixed |= types[d] != type;
    if (mixed)
        for (int d = 0; d < n_mat; ++d)
            if (types[d] != Q4_K && types[d] != Q5_K && types[d] != Q6_K) return MI355X_E_INVAL;
    int64_t all_rows = 0;
    for (int d = 0; d < n_mat; ++d) all_rows += N[d];
    MmqShape sh = mmq_shape(types[0], all_rows, M);  // (several types: on the first one's choice)
    bool has_q5 = false;
    for (int d = 0; d < n_mat; ++d) has_q5 |= types[d] == Q5_K;
    if (mixed && has_q5 && sh.rt == 128 && sh.cw == 2) sh = {128, 1};  // kq_mmq_mixed<128, 2> has no Q5_K body
    if (sh.cw == 4 && (mixed || type == Q6_K)) sh = {128, 2};  // the 4-wave 128 x 128 tile: Q4_K / Q5_K only
    if (sh.rt == 192 && (mixed || type == Q6_K)) sh = {128, 1};  // the 12-wave 192-row tile: Q4_K / Q5_K only
    const int rt = sh.rt;
    MmqArgs a;
    memset(&a, 0, sizeof(a));
    a.n_mat = n_mat;
    a.xq = xq;
    a.nb = (int)(K / QK);
    a.xq_col_stride = (int64_t)a.nb * Q8L_STRIDE;
    a.m_cols = (int)M;
    int tiles = 0;
    double wbytes = 0, ybytes = 0;
    for (int d = 0; d < n_mat; ++d) {
        a.tile0[d] = tiles;
        a.mw[d] = (const uint8_t *)w[d];
        a.mrow_stride[d] = (int64_t)row_stride[d];
        a.mn_rows[d] = (int)N[d];
        a.my[d] = y[d];
        a.my_col_stride[d] = y_col_stride[d];
        a.mtype[d] = types[d];
        tiles += (int)((N[d] + rt - 1) / rt);
        wbytes += (double)N[d] * a.nb * block_bytes(types[d]);
        ybytes += (double)M * N[d] * 4.0;
    }
    a.tile0[n_mat] = tiles;
    if (kv) {
        for (int d = 0; d < n_mat; ++d) a.kv_kind[d] = kv->kind[d];
        a.kv_pos = kv->pos;
        a.kv_rope = kv->rope;
        a.kv_k_cache = kv->k_cache;
        a.kv_v_cache = kv->v_cache;
        a.kv_n_ctx = kv->n_ctx;
        a.kv_hd = kv->hd;
    }
    a.w = a.mw[0];
    a.row_stride = a.mrow_stride[0];
    a.n_rows = a.mn_rows[0];
    a.y = a.my[0];
    a.y_col_stride = a.my_col_stride[0];
    const void *fn = mmq_fn(type, mixed, sh);
    size_t lds = mmq_lds(mixed ? Q6_K : type, sh);  // mixed: the largest tile of its bodies
    if (mixed) lds = std::max(lds, std::max(mmq_lds(Q4_K, sh), mmq_lds(Q5_K, sh)));
    const dim3 grid((unsigned)((M + mmq_cols(sh.cw) - 1) / mmq_cols(sh.cw)), (unsigned)tiles, 1);
    allow_lds(fn, lds);
    hipEvent_t e0, e1;
    void *args[] = {&a};
    hipError_t e;
    if (timing_slot(stream, e0, e1)) {
        e = hipExtLaunchKernel(fn, grid, dim3((unsigned)(64 * mmq_waves(rt, sh.cw))), args, lds, stream, e0, e1, 0);
        timing_log(mixed ? std::string("kq::kq_mmq_mixed") : std::string("kq::kq_mmq<") + std::to_string(type) + ">", wbytes + (double)M * a.nb * Q8L_STRIDE + ybytes,
                   e0, e1);
    } else {
        e = hipLaunchKernel(fn, grid, dim3((unsigned)(64 * mmq_waves(rt, sh.cw))), args, lds, stream);
    }
    if (e != hipSuccess) return (int)e;
    e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

bool mmq_applies(int type, const void *w, int64_t N, size_t row_stride, int64_t M) {
    if (!rows_enabled() || M < kMmqMinCols || N <= 0) return false;
    if (type != Q4_K && type != Q5_K && type != Q6_K) return false;
    if (N >= (1ll << 31) || M >= (1ll << 31)) return false;
    if (type == Q6_K) return true;  // any alignment: fetched from the 16-B boundary below each block
    return ((uintptr_t)w & 15u) == 0 && (row_stride & 15u) == 0;
}

int launch_quantize(const float *x, int64_t x_stride_floats, void *y, int64_t k, int64_t nrows,
                    hipStream_t stream) {
    const int64_t nb = k / QK;
    const int64_t nblocks = nb * nrows;
    if (nblocks == 0) return MI355X_OK;
    const int64_t wgs = (nblocks + WAVES_PER_WG - 1) / WAVES_PER_WG;
    hipEvent_t e0, e1;
    if (timing_slot(stream, e0, e1)) {
        hipExtLaunchKernelGGL(kq_quantize_q8K, dim3((unsigned)wgs), dim3(WG_THREADS), 0, stream, e0, e1, 0, x,
                              x_stride_floats, (uint8_t *)y, (int)nb, nblocks);
        timing_log("kq::kq_quantize_q8K", (double)nblocks * (QK * 4.0 + 292.0), e0, e1);
    } else {
        hipLaunchKernelGGL(kq_quantize_q8K, dim3((unsigned)wgs), dim3(WG_THREADS), 0, stream, x, x_stride_floats,
                           (uint8_t *)y, (int)nb, nblocks);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

// One activation column (decode): kq_rows when the rows are contiguous (always for
// GGUF tensors), kq_gemv otherwise. x is quantized inside the GEMV for K <= 8192
// (x 16-B aligned), else into `ws` first.
// With `ext` (fused prologue / residual epilogue): kq_rows applies them in-kernel
// when it takes the shape with the fused quantizer; otherwise the prologue runs as its
// own kernel into the front of the workspace and the residual adds follow the GEMV
// (the same kernels as the separate nodes, so the bits do not depend on the path).
size_t ext_x_bytes(int64_t k) { return ((size_t)k * 4 + 255) & ~(size_t)255; }

int gemv_m1(const mi355x_gemv_desc *d, int n, const float *x, int64_t k, void *ws, size_t ws_size,
            hipStream_t stream, const mi355x_gemv_ext *ext) {
    const bool has_ext = ext && (ext->prologue != MI355X_PRO_NONE || ext->epilogue != MI355X_EPI_NONE || [&] {
        for (int i = 0; i < n && i < MI355X_MAX_FUSED; ++i)
            if (ext->residual[i]) return true;
        return false;
    }());
    if (has_ext) {
        if (ext->prologue != MI355X_PRO_NONE && !ext->x2) return MI355X_E_INVAL;
        const bool epi = ext->epilogue == MI355X_EPI_SWIGLU;
        if (ext->epilogue != MI355X_EPI_NONE && !epi) return MI355X_E_INVAL;
        if (epi && (n != 2 || !ext->epi_y || d[0].n_rows != d[1].n_rows || ext->residual[0] || ext->residual[1]))
            return MI355X_E_INVAL;
        const bool x2_ok = ext->prologue == MI355X_PRO_NONE || ((uintptr_t)ext->x2 & 15u) == 0;
        if (rows_enabled() && k / QK <= kRowsFusedMaxNb && ((uintptr_t)x & 15u) == 0 && x2_ok) {
            RowsPlan rp;
            const int rc = plan_rows(d, n, k, true, rp);
            if (rc == MI355X_OK) {
                rp.a.x = x;
                rp.a.pro = ext->prologue == MI355X_PRO_RMS_NORM ? ROWS_PRO_NORM
                           : ext->prologue == MI355X_PRO_SWIGLU ? ROWS_PRO_SWIGLU
                                                                : ROWS_PRO_NONE;
                rp.a.x2 = ext->x2;
                rp.a.eps = ext->eps;
                rp.fn = pick_rows(rp.tmask, true, rp.a.pro, rp.dyn);
                for (int i = 0; i < n; ++i) {
                    rp.a.res[i] = ext->residual[i];
                    rp.a.n_rows[i] = (int)d[i].n_rows;
                }
                // SWIGLU epilogue in-kernel when gate wave j and up wave j land in the same
                // workgroup with the same rows: equal wave counts, up's first wave on a
                // workgroup boundary (gw = wave * grid + block)
                const int g = (int)rp.grid.x;
                // (kq_rows_dyn: a workgroup owns the same rows of both by construction)
                const bool paired = epi && (rp.dyn || (rp.a.wave_prefix[2] == 2 * rp.a.wave_prefix[1] &&
                                                       rp.a.wave_prefix[1] % g == 0 && rp.a.rbase[0] == rp.a.rbase[1] &&
                                                       rp.a.rrem[0] == rp.a.rrem[1]));
                if (!epi || paired) {
                    if (paired) {
                        rp.a.epi = 1;
                        rp.a.epi_n = (int)d[0].n_rows;
                        rp.a.epi_wave_off = rp.a.wave_prefix[1] / g;
                        rp.a.epi_y = ext->epi_y;
                    }
                    if (!device_ok()) return MI355X_E_NODEVICE;
                    return launch_rows(rp, stream);
                }
            } else if (rc != MI355X_E_UNSUPPORTED) {
                return rc;
            }
        }
        // staged: prologue kernel -> GEMV -> residual adds
        const float *xs = x;
        uint8_t *w8 = (uint8_t *)ws;
        size_t wsz = ws_size;
        if (ext->prologue != MI355X_PRO_NONE) {
            if (!ws || ws_size < ext_x_bytes(k) || ((uintptr_t)ws & 15u)) return MI355X_E_WORKSPACE;
            if (!device_ok()) return MI355X_E_NODEVICE;
            float *xt = (float *)ws;
            const int rc = ext->prologue == MI355X_PRO_RMS_NORM ? launch_rms_norm(x, ext->x2, xt, k, 1, ext->eps, stream)
                                                                : launch_swiglu(x, ext->x2, xt, k, stream);
            if (rc) return rc;
            xs = xt;
            w8 += ext_x_bytes(k);
            wsz -= ext_x_bytes(k);
        }
        int rc = gemv_m1(d, n, xs, k, w8, wsz, stream, nullptr);
        if (rc) return rc;
        for (int i = 0; i < n; ++i)
            if (ext->residual[i] && d[i].n_rows > 0) {
                rc = launch_binary(0, d[i].y, ext->residual[i], d[i].y, d[i].n_rows, stream);
                if (rc) return rc;
            }
        if (epi && d[0].n_rows > 0) return launch_swiglu(d[0].y, d[1].y, ext->epi_y, d[0].n_rows, stream);
        return MI355X_OK;
    }
    const bool fusedq = k / QK <= kFusedQMaxNb && ((uintptr_t)x & 15u) == 0;
    const size_t need = (size_t)(k / QK) * 292;
    if (rows_enabled()) {
        RowsPlan rp;
        // GEMV_FQMAX (A/B only): the most superblocks quantized inside kq_rows; above it one
        // kq_quantize_q8L launch first and the GEMV DMAs the Q8L row
        const int64_t fq_max = (int64_t)knob(KNOB_GEMV_FQMAX);
        const bool rows_fq = k / QK <= fq_max && k / QK <= kRowsFusedMaxNb && ((uintptr_t)x & 15u) == 0;
        int rc = plan_rows(d, n, k, rows_fq, rp);
        if (rc == MI355X_OK) {
            if (rows_fq) {
                rp.a.x = x;
                if (!device_ok()) return MI355X_E_NODEVICE;
                return launch_rows(rp, stream);
            }
            const size_t need_l = (size_t)(k / QK) * Q8L_STRIDE;
            if (!ws || ws_size < need_l || ((uintptr_t)ws & 15u)) return MI355X_E_WORKSPACE;
            if (!device_ok()) return MI355X_E_NODEVICE;
            rc = launch_quantize_q8L(x, k, ws, k, 1, stream);
            if (rc) return rc;
            rp.a.xq = (const uint8_t *)ws;
            return launch_rows(rp, stream);
        }
        if (rc != MI355X_E_UNSUPPORTED) return rc;
    }
    GemvPlan pl;
    int rc = plan_gemv(d, n, k, 1, 1, fusedq, false, pl);
    if (rc) return rc;
    if (fusedq) {
        pl.a.x = x;
        pl.a.x_col_stride = k;
        if (!device_ok()) return MI355X_E_NODEVICE;
        return launch_gemv(pl, stream);
    }
    if (!ws || ws_size < need || ((uintptr_t)ws & 3u)) return MI355X_E_WORKSPACE;
    if (!device_ok()) return MI355X_E_NODEVICE;
    rc = launch_quantize(x, k, ws, k, 1, stream);
    if (rc) return rc;
    pl.a.xq = (const uint8_t *)ws;
    pl.a.xq_col_stride = (int64_t)need;
    return launch_gemv(pl, stream);
}

uint64_t api_selector_key() {
    return (uint64_t)(uint32_t)(g_impl.load() + 1) | ((uint64_t)(uint32_t)g_rows_waves.load() << 8) |
           ((uint64_t)(uint32_t)(mmq_impl() + 1) << 16) | ((uint64_t)(uint32_t)(prefill_precision() + 1) << 24) |
           ((uint64_t)knob_generation() << 32);
}

}  // namespace kq

using namespace kq;

extern "C" {

size_t mi355x_row_size(int type, int64_t k) {
    if (k < 0 || k % QK) return 0;
    const int64_t nb = k / QK;
    if (type == MI355X_TYPE_Q8_K) return (size_t)(nb * 292);
    if (type == MI355X_TYPE_F32) return (size_t)(k * 4);
    return (size_t)(nb * block_bytes(type));
}

const char *mi355x_version(void) { return "ggml-mi355x 0.1.0 (gfx950, wave64, K-quant GEMV)"; }

int mi355x_device_available(void) { return device_ok(); }

int mi355x_quantize_q8_K(const float *x, size_t x_stride, void *y, int64_t k, int64_t nrows, void *stream) {
    if (k <= 0 || k % QK || nrows < 0) return MI355X_E_INVAL;
    if (nrows == 0) return MI355X_OK;
    if (!x || !y || (x_stride & 3u) || ((uintptr_t)x & 3u) || ((uintptr_t)y & 3u)) return MI355X_E_INVAL;
    if (nrows > 1 && x_stride < (size_t)k * 4) return MI355X_E_INVAL;
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_quantize(x, (int64_t)(x_stride / 4), y, k, nrows, (hipStream_t)stream);
}

static void die(const char *fn, const char *msg) {
    fprintf(stderr, "%s: %s\n", fn, msg);
    abort();
}

// ---- the trait-table surface (ggml_vec_dot_t / ggml_from_float_t): called by
// ggml-cpu's mul_mat from nth threads at once with HOST pointers into its own buffers
// (src0 rows, params->wdata; README.md:121-137, :449), or with device pointers. Each
// calling thread owns a non-blocking stream on its current device plus device staging;
// host operands are copied in, results copied out, and only that stream is synchronized,
// so concurrent callers never serialize on the default stream or share a buffer.
namespace {
struct ThreadCtx {
    int dev = -1;
    hipStream_t st = nullptr;
    void *buf = nullptr;
    size_t cap = 0;
    ~ThreadCtx() {
        if (buf) hipFree(buf);
        if (st) hipStreamDestroy(st);
    }
};
thread_local ThreadCtx t_ctx;

ThreadCtx *thread_ctx(size_t need) {
    ThreadCtx &c = t_ctx;
    const int dev = current_device();
    if (c.dev != dev) {  // the thread moved to another device: new stream and staging there
        if (c.buf) hipFree(c.buf);
        if (c.st) hipStreamDestroy(c.st);
        c.buf = nullptr;
        c.st = nullptr;
        c.cap = 0;
        c.dev = -1;
        if (hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking) != hipSuccess) return nullptr;
        c.dev = dev;
    }
    if (need > c.cap) {
        if (c.buf) hipFree(c.buf);
        c.buf = nullptr;
        c.cap = 0;
        if (hipMalloc(&c.buf, need) != hipSuccess) return nullptr;
        c.cap = need;
    }
    return &c;
}

// True when p is device-accessible memory of the current device (hipMalloc / managed).
// A buffer of another GPU is foreign here: it is staged like host memory (a peer copy),
// never read in place by a kernel of this device.
bool on_device(const void *p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // plain pageable host memory: not an error to keep
        return false;
    }
    if (at.type == hipMemoryTypeManaged) return true;
    return at.type == hipMemoryTypeDevice && at.device == current_device();
}
}  // namespace

void mi355x_quantize_row_q8_K(const float *x, void *y, int64_t k) {
    if (k % QK) die(__func__, "k % QK_K != 0");
    if (k == 0) return;
    if (!device_ok()) die(__func__, "no gfx950 device");
    const size_t xb = (size_t)k * 4, yb = (size_t)(k / QK) * 292;
    const bool xd = on_device(x), yd = on_device(y);
    ThreadCtx *c = thread_ctx(((xd ? 0 : xb + 16) + (yd ? 0 : yb) + 255) & ~(size_t)255);
    if (!c) die(__func__, "stream / staging allocation failed");
    const float *dx = x;
    void *dy = y;
    uint8_t *stage = (uint8_t *)c->buf;
    if (!xd) {
        if (hipMemcpyAsync(stage, x, xb, hipMemcpyDefault, c->st) != hipSuccess) die(__func__, "copy in failed");
        dx = (const float *)stage;
        stage += (xb + 15) & ~(size_t)15;
    }
    if (!yd) dy = stage;
    if (mi355x_quantize_q8_K(dx, xb, dy, k, 1, c->st)) die(__func__, "launch failed");
    if (!yd && hipMemcpyAsync(y, dy, yb, hipMemcpyDefault, c->st) != hipSuccess) die(__func__, "copy out failed");
    if (hipStreamSynchronize(c->st) != hipSuccess) die(__func__, "hipStreamSynchronize failed");
}

size_t mi355x_mul_mat_workspace_size(int src0_type, int64_t ne00, int64_t ne01, int64_t ne11) {
    if (!block_bytes(src0_type) || ne00 <= 0 || ne00 % QK || ne11 < 0) return 0;
    if (ne11 == 0 || (ne11 == 1 && ne00 / QK <= kFusedQMaxNb)) return 0;
    size_t bytes = (size_t)ne11 * (size_t)(ne00 / QK) * Q8L_STRIDE;  // >= raw 292-B blocks
    // the f16 prefill path runs instead at ne11 >= 16 once mi355x_prefill_precision selects it
    // (its image and split-K slabs; callers re-query after switching)
    if (ne11 >= kMmqMinCols && ne01 > 0 && prefill_precision() >= MI355X_PREFILL_F16) {
        const size_t f = mmf_workspace(ne01, ne11, ne00 / QK);
        bytes = f > bytes ? f : bytes;
    }
    return (bytes + 255) & ~(size_t)255;
}

size_t mi355x_gemv_fused_workspace_size(int64_t k) {
    if (k <= 0 || k % QK || k / QK <= kFusedQMaxNb) return 0;
    return ((size_t)(k / QK) * Q8L_STRIDE + 255) & ~(size_t)255;
}

int mi355x_mul_mat_q8(int src0_type, const void *src0, int64_t ne00, int64_t ne01, size_t nb01,
                      const void *src1_q8, int64_t ne11, size_t nb11, float *dst, size_t nb1, void *stream) {
    if (ne11 < 0 || ne01 < 0) return MI355X_E_INVAL;
    if (ne11 == 0 || ne01 == 0) return MI355X_OK;
    if (!src1_q8 || ((uintptr_t)src1_q8 & 3u) || (nb11 & 3u) || ((uintptr_t)dst & 3u) || (nb1 & 3u))
        return MI355X_E_INVAL;
    if (ne00 <= 0 || ne00 % QK) return MI355X_E_INVAL;
    if (ne11 > 1 && (nb11 < (size_t)(ne00 / QK) * 292 || nb1 < (size_t)ne01 * 4)) return MI355X_E_INVAL;
    if (ne11 > 0x7fffffff) return MI355X_E_INVAL;
    mi355x_gemv_desc d = {src0_type, src0, ne01, nb01, dst};
    const int ncol = choose_ncol(ne11, (int)(ne00 / QK));
    GemvPlan pl;
    int rc = plan_gemv(&d, 1, ne00, ne11, ncol, false, false, pl);
    if (rc) return rc;
    pl.a.xq = (const uint8_t *)src1_q8;
    pl.a.xq_col_stride = (int64_t)nb11;
    pl.a.y_col_stride[0] = (int64_t)(nb1 / 4);
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_gemv(pl, (hipStream_t)stream);
}

int mi355x_mul_mat(int src0_type, const void *src0, int64_t ne00, int64_t ne01, size_t nb01, const float *src1,
                   int64_t ne11, size_t nb11, float *dst, size_t nb1, void *workspace, size_t workspace_size,
                   void *stream) {
    if (ne11 < 0 || ne01 < 0 || ne00 <= 0 || ne00 % QK) return MI355X_E_INVAL;
    if (!block_bytes(src0_type)) return MI355X_E_UNSUPPORTED;
    if (ne11 == 0 || ne01 == 0) return MI355X_OK;
    if (!src1 || ((uintptr_t)src1 & 3u) || (nb11 & 3u) || !dst || ((uintptr_t)dst & 3u) || (nb1 & 3u))
        return MI355X_E_INVAL;
    if (ne11 > 1 && (nb11 < (size_t)ne00 * 4 || nb1 < (size_t)ne01 * 4)) return MI355X_E_INVAL;
    if (ne11 == 1) {
        mi355x_gemv_desc d = {src0_type, src0, ne01, nb01, dst};
        return gemv_m1(&d, 1, src1, ne00, workspace, workspace_size, (hipStream_t)stream);
    }
    size_t need = mi355x_mul_mat_workspace_size(src0_type, ne00, ne01, ne11);
    if (!workspace || workspace_size < need) return MI355X_E_WORKSPACE;
    if (mmf_applies(src0_type, src0, ne01, nb01, ne11, ne00) && ((uintptr_t)workspace & 15u) == 0) {
        if (!device_ok()) return MI355X_E_NODEVICE;
        int rc = launch_f16img(src1, (int64_t)(nb11 / 4), (uint8_t *)workspace, ne00, ne11, (hipStream_t)stream);
        if (rc) return rc;
        return launch_mmf_gemm(src0_type, src0, ne00, ne01, nb01, (uint8_t *)workspace, ne11, dst, (int64_t)(nb1 / 4),
                               (hipStream_t)stream);
    }
    if (mmq_applies(src0_type, src0, ne01, nb01, ne11) && ((uintptr_t)workspace & 15u) == 0) {
        if (!device_ok()) return MI355X_E_NODEVICE;
        int rc = launch_quantize_q8L(src1, (int64_t)(nb11 / 4), workspace, ne00, ne11, (hipStream_t)stream, true);
        if (rc) return rc;
        return launch_mmq(src0_type, src0, ne00, ne01, nb01, (const uint8_t *)workspace, ne11, dst,
                          (int64_t)(nb1 / 4), (hipStream_t)stream);
    }
    if (!device_ok()) return MI355X_E_NODEVICE;
    int rc = launch_quantize(src1, (int64_t)(nb11 / 4), workspace, ne00, ne11, (hipStream_t)stream);
    if (rc) return rc;
    const size_t q8_row = (size_t)(ne00 / QK) * 292;
    return mi355x_mul_mat_q8(src0_type, src0, ne00, ne01, nb01, workspace, ne11, q8_row, dst, nb1, stream);
}

int mi355x_gemv_fused(const mi355x_gemv_desc *descs, int n_desc, const float *x, int64_t k, void *workspace,
                      size_t workspace_size, void *stream) {
    if (!descs || !x || ((uintptr_t)x & 3u)) return MI355X_E_INVAL;
    if (k <= 0 || k % QK) return MI355X_E_INVAL;
    for (int i = 0; i < n_desc && i < MI355X_MAX_FUSED; ++i)
        if (descs[i].y && ((uintptr_t)descs[i].y & 3u)) return MI355X_E_INVAL;
    return gemv_m1(descs, n_desc, x, k, workspace, workspace_size, (hipStream_t)stream);
}

size_t mi355x_gemv_ext_workspace_size(int64_t k) {
    if (k <= 0 || k % QK) return 0;
    return ext_x_bytes(k) + mi355x_gemv_fused_workspace_size(k);
}

int mi355x_gemv_fused_ext(const mi355x_gemv_desc *descs, int n_desc, const float *x, int64_t k,
                          const mi355x_gemv_ext *ext, void *workspace, size_t workspace_size, void *stream) {
    if (!descs || !x || ((uintptr_t)x & 3u)) return MI355X_E_INVAL;
    if (k <= 0 || k % QK || n_desc < 1 || n_desc > MI355X_MAX_FUSED) return MI355X_E_INVAL;
    if (ext && (ext->prologue < MI355X_PRO_NONE || ext->prologue > MI355X_PRO_SWIGLU)) return MI355X_E_INVAL;
    if (ext && ext->prologue == MI355X_PRO_RMS_NORM && !(ext->eps >= 0.0f)) return MI355X_E_INVAL;
    if (ext && ext->epilogue == MI355X_EPI_SWIGLU && ((uintptr_t)ext->epi_y & 3u)) return MI355X_E_INVAL;
    for (int i = 0; i < n_desc; ++i) {
        if (descs[i].y && ((uintptr_t)descs[i].y & 3u)) return MI355X_E_INVAL;
        if (ext && ext->residual[i] && ((uintptr_t)ext->residual[i] & 3u)) return MI355X_E_INVAL;
    }
    return gemv_m1(descs, n_desc, x, k, workspace, workspace_size, (hipStream_t)stream, ext);
}

int mi355x_debug_stream(const void *buf, size_t bytes, void *sink, void *stream) {
    if (!buf || !sink || ((uintptr_t)buf & 15u)) return MI355X_E_INVAL;
    int dev = current_device();
    if (dev < 0 || !device_ok()) return MI355X_E_NODEVICE;
    const int cus = g_dev_cus[dev] > 0 ? g_dev_cus[dev] : 256;
    const int waves = cus * 12;
    const int64_t per_wave = (int64_t)(bytes / waves) / 2048 * 2048;
    if (per_wave <= 0) return MI355X_E_INVAL;
    const size_t lds = 4 * 4 * 2048;
    allow_lds((const void *)kq_stream_ceiling, lds);
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0, e1;
    if (timing_slot(st, e0, e1)) {
        hipExtLaunchKernelGGL(kq_stream_ceiling, dim3((unsigned)(cus * 3)), dim3(256), (uint32_t)lds, st, e0, e1, 0,
                              (const uint8_t *)buf, per_wave, waves, (uint32_t *)sink);
        timing_log("kq::kq_stream_ceiling", (double)per_wave * waves, e0, e1);
    } else {
        hipLaunchKernelGGL(kq_stream_ceiling, dim3((unsigned)(cus * 3)), dim3(256), lds, st, (const uint8_t *)buf,
                           per_wave, waves, (uint32_t *)sink);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MI355X_OK : (int)e;
}

int mi355x_debug_block_partials(int src0_type, const void *src0, int64_t ne00, int64_t ne01, size_t nb01,
                                const void *src1_q8, int32_t *out, void *stream) {
    if (!out || !src1_q8 || ((uintptr_t)src1_q8 & 3u)) return MI355X_E_INVAL;
    if (ne01 == 0) return MI355X_OK;
    // the DEBUG kernel stores only the partials; dst is a placeholder
    const int64_t nb = ne00 / QK;
    float *dst = (float *)out;
    mi355x_gemv_desc d = {src0_type, src0, ne01, nb01, dst};
    GemvPlan pl;
    int rc = plan_gemv(&d, 1, ne00, 1, 1, false, true, pl);
    if (rc) return rc;
    pl.a.xq = (const uint8_t *)src1_q8;
    pl.a.xq_col_stride = (int64_t)(nb * 292);
    pl.a.dbg = out;
    if (!device_ok()) return MI355X_E_NODEVICE;
    return launch_gemv(pl, (hipStream_t)stream);
}

int mi355x_gemv_impl(int impl) {
    if (impl < MI355X_GEMV_AUTO || impl > MI355X_GEMV_DYN) return MI355X_E_INVAL;
    return g_impl.exchange(impl);
}

int mi355x_debug_knob(const char *name, double value, double *previous) {
    if (!name) return MI355X_E_INVAL;
    for (int k = 0; k < KNOB_COUNT; ++k) {
        if (strcmp(name, kKnobs[k].name) != 0) continue;
        if (previous) *previous = knob((Knob)k);
        if (value != value) {  // NaN: back to the product default
            g_knob_set[k].store(false);
        } else {
            g_knob[k].store(value);
            g_knob_set[k].store(true);
        }
        g_knob_gen.fetch_add(1);
        return MI355X_OK;
    }
    return MI355X_E_INVAL;
}

int mi355x_mmq_impl(int impl) {
    if (impl < MI355X_MMQ_AUTO || impl > MI355X_MMQ_TILE192) return MI355X_E_INVAL;
    const int prev = mmq_impl();
    g_mmq_impl.store(impl);
    return prev;
}

int mi355x_prefill_precision(int precision) {
    if (precision < 0) return prefill_precision();  // query
    if (precision > MI355X_PREFILL_F16_ALL) return MI355X_E_INVAL;
    const int prev = prefill_precision();
    g_prefill.store(precision);
    return prev;
}

int mi355x_gemv_waves(int waves) {
    if (waves < 0 || waves > ROWS_WAVES) return MI355X_E_INVAL;
    return g_rows_waves.exchange(waves);
}

}  // extern "C"
namespace kq {
uint64_t *diag_stamps(int64_t *cap) {
    if (cap) *cap = g_stamps_cap;
    return g_stamps;
}
}  // namespace kq
extern "C" {
int mi355x_diag_stamps(void *buf, size_t bytes) {
    g_stamps = (uint64_t *)buf;
    g_stamps_cap = buf ? (int64_t)(bytes / 8) : 0;
    return MI355X_OK;
}

int mi355x_timing_enable(int enable) {
    std::lock_guard<std::mutex> lk(g_tmu);
    g_timing = enable != 0;
    g_tlog.clear();
    g_tpool_used = 0;
    return MI355X_OK;
}

int mi355x_timing_read(mi355x_launch_timing *out, int max) {
    if (hipDeviceSynchronize() != hipSuccess) return MI355X_E_NODEVICE;
    std::lock_guard<std::mutex> lk(g_tmu);
    const int n = (int)g_tlog.size();
    for (int i = 0; i < n && i < max && out; ++i) {
        memset(out[i].kernel, 0, sizeof(out[i].kernel));
        strncpy(out[i].kernel, g_tlog[i].kernel.c_str(), sizeof(out[i].kernel) - 1);
        out[i].bytes = g_tlog[i].bytes;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, g_tlog[i].start, g_tlog[i].stop) != hipSuccess) ms = -1.f;
        out[i].ms = ms;
    }
    return n;
}

static void vec_dot_dev(int type, const char *fn, int n, float *s, const void *vx, const void *vy, int nrc) {
    if (nrc != 1) die(fn, "nrc != 1 unsupported (reference configuration: nrows == 1)");
    if (n <= 0 || n % QK) die(fn, "n % QK_K != 0");
    if (!device_ok()) die(fn, "no gfx950 device");
    const size_t wb = mi355x_row_size(type, n), qb = mi355x_row_size(MI355X_TYPE_Q8_K, n);
    const bool xd = on_device(vx), yd = on_device(vy), sd = on_device(s);
    const size_t need = (xd ? 0 : (wb + 15) & ~(size_t)15) + (yd ? 0 : (qb + 15) & ~(size_t)15) + 16;
    ThreadCtx *c = thread_ctx(need);
    if (!c) die(fn, "stream / staging allocation failed");
    uint8_t *stage = (uint8_t *)c->buf;
    const void *dx = vx, *dy = vy;
    if (!xd) {
        if (hipMemcpyAsync(stage, vx, wb, hipMemcpyDefault, c->st) != hipSuccess) die(fn, "copy in failed");
        dx = stage;
        stage += (wb + 15) & ~(size_t)15;
    }
    if (!yd) {
        if (hipMemcpyAsync(stage, vy, qb, hipMemcpyDefault, c->st) != hipSuccess) die(fn, "copy in failed");
        dy = stage;
        stage += (qb + 15) & ~(size_t)15;
    }
    float *ds = sd ? s : (float *)stage;
    const int rc = mi355x_mul_mat_q8(type, dx, n, 1, wb, dy, 1, qb, ds, 4, c->st);
    if (rc) die(fn, "launch failed");
    if (!sd && hipMemcpyAsync(s, ds, 4, hipMemcpyDefault, c->st) != hipSuccess) die(fn, "copy out failed");
    if (hipStreamSynchronize(c->st) != hipSuccess) die(fn, "hipStreamSynchronize failed");
}

void mi355x_vec_dot_q4_K_q8_K(int n, float *s, size_t bs, const void *vx, size_t bx, const void *vy, size_t by,
                              int nrc) {
    (void)bs; (void)bx; (void)by;
    vec_dot_dev(MI355X_TYPE_Q4_K, __func__, n, s, vx, vy, nrc);
}
void mi355x_vec_dot_q5_K_q8_K(int n, float *s, size_t bs, const void *vx, size_t bx, const void *vy, size_t by,
                              int nrc) {
    (void)bs; (void)bx; (void)by;
    vec_dot_dev(MI355X_TYPE_Q5_K, __func__, n, s, vx, vy, nrc);
}
void mi355x_vec_dot_q6_K_q8_K(int n, float *s, size_t bs, const void *vx, size_t bx, const void *vy, size_t by,
                              int nrc) {
    (void)bs; (void)bx; (void)by;
    vec_dot_dev(MI355X_TYPE_Q6_K, __func__, n, s, vx, vy, nrc);
}

}  // extern "C"
