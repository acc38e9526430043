// kq_device.h — device helpers shared by the gfx950 K-quant kernels (Q8_K
// quantization, per-type lane partials, the exact fp32 chain records, LDS-DMA).
#pragma once

#include "kq_common.h"


namespace kq {


typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef float f32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define LDS __attribute__((address_space(3)))

__device__ __forceinline__ u32x4 gload16(const uint8_t *p) { return *(const u32x4a *)p; }
__device__ __forceinline__ uint32_t gload4(const uint8_t *p) { return *(const uint32_t *)p; }

__device__ __forceinline__ float h2f(uint32_t h16) {
    _Float16 h;
    uint16_t b = (uint16_t)h16;
    __builtin_memcpy(&h, &b, 2);
    return (float)h;
}

__device__ __forceinline__ int sdot4(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// Sum over the 8 lanes of an aligned lane-octet (DPP only, no LDS).
__device__ __forceinline__ int octet_sum(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true);  // row_half_mirror
    return v;
}

__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Full-wave reductions with DPP only (no LDS crossbar): quad swaps, 8/16-lane
// mirrors, then row_bcast15/row_bcast31 fold the four rows into lane 63.
template <typename Op>
__device__ __forceinline__ int wave_reduce_dpp(int v, Op op) {
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false));  // row_mirror
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ float wave_max_f32(float v) {
    // |x| values are non-negative (or NaN): their int bit patterns order like the floats.
    // NaN must never win (serial `ax > amax` is false for NaN): map NaN to 0.
    int b = (v == v) ? __float_as_int(v) : 0;
    b = wave_reduce_dpp(b, [](int a, int c) { return a > c ? a : c; });
    return __int_as_float(b);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    return (uint32_t)wave_reduce_dpp((int)v, [](int a, int c) { return (uint32_t)a < (uint32_t)c ? a : c; });
}

// nearest_int(iscale * x) with the multiply-add contracted (aarch64 gcc build of
// quantize_row_q8_K_ref): 12582912.f = 1.5*2^23 rounds to integer, RNE.
__device__ __forceinline__ int nearest_int_fused(float iscale, float x) {
    const float v = __builtin_fmaf(iscale, x, 12582912.f);
    const int i = __float_as_int(v);
    return (i & 0x007fffff) - 0x00400000;
}

// One Q8_K superblock quantized by one wave (quantize_row_q8_K_ref semantics):
// lane l owns x[4l..4l+3]. Returns packed qs of the lane, the 16-element bsum
// (valid on every lane of each lane-quad), and d (uniform).
struct Q8Lane {
    uint32_t qs4;
    int bsum;
    float d;
};

__device__ __forceinline__ Q8Lane quant_values_wave(const f32x4a v, int lane) {
    const float a0 = fabsf(v.x), a1 = fabsf(v.y), a2 = fabsf(v.z), a3 = fabsf(v.w);
    // amax; NaN never wins (fmaxf drops NaN, as `ax > amax` is false for NaN)
    const float m = wave_max_f32(fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)));  // fmaxf drops NaN
    Q8Lane r;
    if (m == 0.f) {  // wave-uniform: the `if (!amax)` branch
        r.qs4 = 0;
        r.bsum = 0;
        r.d = 0.f;
        return r;
    }
    // first index j with |x_j| == amax (serial `if (ax > amax)` keeps the first);
    // key = 2*j + sign(x_j)
    uint32_t key = 0xffffffffu;
    const uint32_t base = 8u * (uint32_t)lane;
    if (a3 == m) key = base + 6u + (v.w < 0.f ? 1u : 0u);
    if (a2 == m) key = base + 4u + (v.z < 0.f ? 1u : 0u);
    if (a1 == m) key = base + 2u + (v.y < 0.f ? 1u : 0u);
    if (a0 == m) key = base + 0u + (v.x < 0.f ? 1u : 0u);
    key = wave_min_u32(key);
    const float maxv = (key & 1u) ? -m : m;
    const float iscale = -127.f / maxv;  // correctly rounded (-fhip-fp32-correctly-rounded-divide-sqrt)
    int q0 = nearest_int_fused(iscale, v.x);
    int q1 = nearest_int_fused(iscale, v.y);
    int q2 = nearest_int_fused(iscale, v.z);
    int q3 = nearest_int_fused(iscale, v.w);
    // y.qs[j] = MIN(127, v) stored as int8 (truncating, as the C assignment does when
    // an overflowed iscale drives v below -128); bsums sum the stored int8 values.
    q0 = (int)(int8_t)(q0 < 127 ? q0 : 127);
    q1 = (int)(int8_t)(q1 < 127 ? q1 : 127);
    q2 = (int)(int8_t)(q2 < 127 ? q2 : 127);
    q3 = (int)(int8_t)(q3 < 127 ? q3 : 127);
    r.qs4 = (uint32_t)(q0 & 0xff) | ((uint32_t)(q1 & 0xff) << 8) | ((uint32_t)(q2 & 0xff) << 16) |
            ((uint32_t)(q3 & 0xff) << 24);
    int s = q0 + q1 + q2 + q3;
    s += __builtin_amdgcn_mov_dpp(s, 0xB1, 0xF, 0xF, true);
    s += __builtin_amdgcn_mov_dpp(s, 0x4E, 0xF, 0xF, true);
    r.bsum = s;
    r.d = 1.f / iscale;
    return r;
}

__device__ __forceinline__ Q8Lane quant_block_wave(const float *xb, int lane) {
    return quant_values_wave(*(const f32x4a *)(xb + 4 * lane), lane);
}

// ------------------------------------------------------------------ per-type lane kernels
// Register image of one lane's share of one superblock.
struct Regs {
    u32x4 a, b, c;
    uint32_t e0, e1, e2, dh;
};

__device__ __forceinline__ u32x4 realign(u32x4 v, uint32_t ex, uint32_t s) {
    u32x4 o;
    o.x = __builtin_amdgcn_alignbyte(v.y, v.x, s);
    o.y = __builtin_amdgcn_alignbyte(v.z, v.y, s);
    o.z = __builtin_amdgcn_alignbyte(v.w, v.z, s);
    o.w = __builtin_amdgcn_alignbyte(ex, v.w, s);
    return o;
}

__device__ __forceinline__ int dot16(u32x4 q, u32x4 a) {
    int d = sdot4(q.x, a.x, 0);
    d = sdot4(q.y, a.y, d);
    d = sdot4(q.z, a.z, d);
    d = sdot4(q.w, a.w, d);
    return d;
}

// 6-bit scales/mins of a Q4_K/Q5_K header (get_scale_min_k4 / README.md:732-739).
struct ScMn {
    int sc_lo, sc_hi, mn;
};
__device__ __forceinline__ ScMn scales_k4(u32x4 hdr, int p) {
    const int j = p >> 1;
    const uint32_t s03 = hdr.y & 0x3f3f3f3fu;
    const uint32_t m03 = hdr.z & 0x3f3f3f3fu;
    const uint32_t s47 = (hdr.w & 0x0f0f0f0fu) | ((hdr.y >> 2) & 0x30303030u);
    const uint32_t m47 = ((hdr.w >> 4) & 0x0f0f0f0fu) | ((hdr.z >> 2) & 0x30303030u);
    const uint32_t sw = (j < 2) ? s03 : s47;
    const uint32_t sh = (uint32_t)((2 * j) & 3) * 8u;
    ScMn r;
    r.sc_lo = (int)((sw >> sh) & 0xffu);
    r.sc_hi = (int)((sw >> (sh + 8u)) & 0xffu);
    const uint32_t mw = (p < 4) ? m03 : m47;
    r.mn = (int)((mw >> ((uint32_t)(p & 3) * 8u)) & 0xffu);
    return r;
}

// Lane partials against one activation column held in LDS.
//   aq: LDS qs of the activation superblock (256 B, 4-byte aligned: raw Q8_K
//   layout), abs: its 16 bsums (4-byte aligned).
__device__ __forceinline__ void lane_q4K(const Regs &r, const uint8_t *aq, const int16_t *abs, int p,
                                         int &isum, int &imin) {
    const int j = p >> 1, h = p & 1;
    const ScMn s = scales_k4(r.a, p);
    const u32x4 alo = *(const u32x4a *)(aq + 64 * j + 16 * h);
    const u32x4 ahi = *(const u32x4a *)(aq + 64 * j + 32 + 16 * h);
    const u32x4 lo = r.b & 0x0f0f0f0fu;
    const u32x4 hi = (r.b >> 4) & 0x0f0f0f0fu;
    isum = __mul24(dot16(lo, alo), s.sc_lo) + __mul24(dot16(hi, ahi), s.sc_hi);  // |dot| < 2^17: i24
    const uint32_t bs2 = *(const uint32_t *)(abs + 2 * p);
    imin = ((int)(int16_t)(bs2 & 0xffffu) + (int)(int16_t)(bs2 >> 16)) * s.mn;
}

__device__ __forceinline__ void lane_q5K(const Regs &r, const uint8_t *aq, const int16_t *abs, int p,
                                         int &isum, int &imin) {
    const int j = p >> 1, h = p & 1;
    const ScMn s = scales_k4(r.a, p);
    const u32x4 alo = *(const u32x4a *)(aq + 64 * j + 16 * h);
    const u32x4 ahi = *(const u32x4a *)(aq + 64 * j + 32 + 16 * h);
    const uint32_t sl = (uint32_t)(2 * j), shh = (uint32_t)(2 * j + 1);
    const u32x4 lo = (r.c & 0x0f0f0f0fu) | (((r.b >> sl) & 0x01010101u) << 4);
    const u32x4 hi = ((r.c >> 4) & 0x0f0f0f0fu) | (((r.b >> shh) & 0x01010101u) << 4);
    isum = __mul24(dot16(lo, alo), s.sc_lo) + __mul24(dot16(hi, ahi), s.sc_hi);  // |dot| < 2^17: i24
    const uint32_t bs2 = *(const uint32_t *)(abs + 2 * p);
    imin = ((int)(int16_t)(bs2 & 0xffffu) + (int)(int16_t)(bs2 >> 16)) * s.mn;
}

__device__ __forceinline__ int sbyte(u32x4 w, int idx) {
    const uint32_t d = (idx < 4) ? w.x : (idx < 8) ? w.y : (idx < 12) ? w.z : w.w;
    return (int)(int8_t)((d >> ((uint32_t)(idx & 3) * 8u)) & 0xffu);
}

// Q6_K lane p: ql[16p..16p+16) of half n=p>>2; part=p&3 selects low/high 32 of the
// half: low nibbles -> elements 128n+32(part>>1)+16(part&1)+[0,16), high nibbles
// the same +64; qh bits (part>>1)*2 and +4.
__device__ __forceinline__ void lane_q6K(const Regs &r, const uint8_t *aq, const int16_t *abs, int p,
                                         int &isum, int &imin, uint32_t &dh) {
    const int n = p >> 2, part = p & 3;
    const u32x4 L = r.a, H = r.b, SC = r.c;
    const uint32_t shl = (uint32_t)(part >> 1) * 2u;
    const u32x4 qlo = (L & 0x0f0f0f0fu) | (((H >> shl) & 0x03030303u) << 4);
    const u32x4 qhi = ((L >> 4) & 0x0f0f0f0fu) | (((H >> (shl + 4u)) & 0x03030303u) << 4);
    const int elo = 128 * n + 32 * (part >> 1) + 16 * (part & 1);
    const u32x4 alo = *(const u32x4a *)(aq + elo);
    const u32x4 ahi = *(const u32x4a *)(aq + elo + 64);
    const int sb = elo >> 4;
    isum = __mul24(dot16(qlo, alo), sbyte(SC, sb)) + __mul24(dot16(qhi, ahi), sbyte(SC, sb + 4));  // i24
    const uint32_t bs2 = *(const uint32_t *)(abs + 2 * p);
    imin = (int)(int16_t)(bs2 & 0xffffu) * sbyte(SC, 2 * p) + (int)(int16_t)(bs2 >> 16) * sbyte(SC, 2 * p + 1);
    dh = r.dh;
}

// Per-block record consumed by the fp32 chain.
struct Rec {
    int a, b;
    float c, e;
};

// The reference's per-superblock fp32 update, by type.
__device__ __forceinline__ float chain_step(int type, const Rec &r, float s) {
    if (type == Q4_K) {
        s = fmaf(-(float)r.b, r.e, s);  // sumf -= dmin * summins   (fmsub, README.md:551)
        s = fmaf((float)r.a, r.c, s);   // sumf += d * sumi         (fmadd, README.md:614)
    } else if (type == Q5_K) {
        const float t = fmaf(r.c, (float)r.a, -(r.e * (float)r.b));  // d*sumi - dmin*sumi_mins
        s = s + t;
    } else {                             // Q6_K: sum += d_all*y.d*(isum - 32*isum_mins)
        s = fmaf(r.c, (float)r.a, s);
    }
    return s;
}

// ------------------------------------------------------------------ weight streaming
// Pieces (16 B) per superblock in the LDS ring: Q4_K 9 (144 B), Q5_K 11 (176 B),
// Q6_K 14 (210 B fetched from the 16-B boundary below the block: 224 B).
__host__ __device__ constexpr int pieces_of(int type) { return type == Q4_K ? 9 : type == Q5_K ? 11 : 14; }
__host__ __device__ constexpr int slot_bytes(int tmask) { return 8 * 16 * (tmask == 1 ? 9 : 14); }

// LDS-DMA of one 16-B granule per lane: lane i's granule lands at dst + 16*i.
// Issued as inline asm on purpose: for the builtin, the compiler's waitcnt pass
// treats every later LDS read as possibly aliasing the pending DMA and inserts
// s_waitcnt vmcnt(0) before it (seen in the ISA: it drained the whole ring each
// step). Completion is tracked by hand with counted vmcnt waits instead; the
// "memory" clobber keeps earlier LDS reads of a recycled slot ahead of the DMA.
// s_nop: SALU write of M0 -> LDS-DMA needs one wait state. M0 is reserved by the
// compiler (never allocated to values; set right before each instruction that
// reads it), so clobbering it here is safe; the warning saying so is silenced.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(const void *src, LDS void *dst) {
    const uint32_t m0 = (uint32_t)(uintptr_t)dst;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(src)
                 : "memory", "m0");
}
// One dword per lane (the 4-B form: 256 B per wave instruction).
__device__ __forceinline__ void dma4(const void *src, LDS void *dst) {
    const uint32_t m0 = (uint32_t)(uintptr_t)dst;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off" ::"s"(m0), "v"(src)
                 : "memory", "m0");
}
// Same, non-temporal (nt): for the once-read weight stream (measured on this part:
// 6.2 -> 7.1 TB/s chip-wide, profiles/r01_lds_dma_stream_ceiling.txt).
__device__ __forceinline__ void dma16_nt(const void *src, LDS void *dst) {
    const uint32_t m0 = (uint32_t)(uintptr_t)dst;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m0), "v"(src)
                 : "memory", "m0");
}
// dma16_nt for lanes [0, n) only, the lane mask applied inside the asm: the instruction
// is issued on every path (no compiler branch around a partial mask), so a counted wait
// that covers it holds on every path the ISA lint walks (tools/vmem_lint.py). A
// vector-memory instruction counts in vmcnt whatever its mask (kq_rows' prologue step,
// KQ_ROWS_MASKED).
__device__ __forceinline__ void dma16_nt_lanes(const void *src, LDS void *dst, int lane, int n) {
    const uint32_t m0 = (uint32_t)(uintptr_t)dst;
    uint64_t save;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "v_cmp_gt_i32_e32 vcc, %2, %3\n\t"
        "s_and_b64 exec, exec, vcc\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %4, off nt\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(save)
        : "s"(m0), "s"(n), "v"(lane), "v"(src)
        : "memory", "m0", "vcc");
}
#pragma clang diagnostic pop

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wait until at most `steps` ring steps (2 DMA instructions each) are in flight.
__device__ __forceinline__ void vm_wait_steps(int steps) {
    switch (steps) {
        case 0: vm_wait<0>(); break;
        case 1: vm_wait<2>(); break;
        case 2: vm_wait<4>(); break;
        case 3: vm_wait<6>(); break;
        case 4: vm_wait<8>(); break;
        case 5: vm_wait<10>(); break;
        case 6: vm_wait<12>(); break;
        case 7: vm_wait<14>(); break;
        case 8: vm_wait<16>(); break;
        case 9: vm_wait<18>(); break;
        case 10: vm_wait<20>(); break;
        case 11: vm_wait<22>(); break;
        default: vm_wait<24>(); break;
    }
}

// Register image of one lane's share of a superblock, read from its LDS ring slot.
//   region: LDS bytes of row g's superblock copy; sh: byte offset of the block
//   inside the region (Q6_K: block start mod 16; 0 otherwise).
template <int TMASK>
__device__ __forceinline__ void lds_block(Regs &r, const uint8_t *region, uint32_t sh, int type, int p) {
    if (TMASK == 1 || (TMASK != 4 && type == Q4_K)) {
        r.a = *(const u32x4 *)(region);
        r.b = *(const u32x4 *)(region + 16 + 16 * p);
    } else if (TMASK != 4 && type == Q5_K) {
        r.a = *(const u32x4 *)(region);
        r.b = *(const u32x4 *)(region + 16 + 16 * (p & 1));
        r.c = *(const u32x4 *)(region + 48 + 16 * p);
    } else {
        const int n = p >> 2, part = p & 3;
        const uint32_t s4 = sh & 3u;
        const uint8_t *b = region + (sh & ~3u);
        const int fql = 16 * p, fqh = 128 + 32 * n + 16 * (part & 1);
        r.a = realign(*(const u32x4a *)(b + fql), *(const uint32_t *)(b + fql + 16), s4);
        r.b = realign(*(const u32x4a *)(b + fqh), *(const uint32_t *)(b + fqh + 16), s4);
        r.c = realign(*(const u32x4a *)(b + 192), *(const uint32_t *)(b + 208), s4);
        r.dh = (*(const uint32_t *)(b + 208) >> (8u * s4)) & 0xffffu;
    }
}

template <int TMASK>
__device__ __forceinline__ void lane_partials(const Regs &rr, const uint8_t *aq, const int16_t *ab, int type, int p,
                                              int &isum, int &imin, uint32_t &dh) {
    if (TMASK == 1 || (TMASK != 4 && type == Q4_K)) lane_q4K(rr, aq, ab, p, isum, imin);
    else if (TMASK != 4 && type == Q5_K) lane_q5K(rr, aq, ab, p, isum, imin);
    else lane_q6K(rr, aq, ab, p, isum, imin, dh);
}

// Exact record of one superblock: the operands of the reference's fp32 update.
template <int TMASK>
__device__ __forceinline__ Rec make_rec(int type, int isum, int imin, const Regs &rr, uint32_t dh, float yd) {
    if (TMASK == 1) type = Q4_K;
    if (TMASK == 4) type = Q6_K;
    Rec r;
    if (type == Q6_K) {
        r.a = isum - 32 * imin;
        r.b = 0;
        r.c = h2f(dh) * yd;  // d_all * y.d
        r.e = 0.f;
    } else {
        r.a = isum;
        r.b = imin;
        r.c = yd * h2f(rr.a.x & 0xffffu);  // y.d * fp16(x.d)
        r.e = yd * h2f(rr.a.x >> 16);      // y.d * fp16(x.dmin)
    }
    return r;
}


}  // namespace kq
