// stream_size.hip — single-launch LDS-DMA streaming time by buffer size (the ceiling a
// decode GEMV launch of that many weight bytes can approach, start-up included), with
// the best stream_bench shape (2 KB steps, 4 in flight, nt, 12 waves per CU) and the
// kq_rows-like shape (one 12-wave workgroup per CU, 3 KB steps x 3). Buffers are
// rotated past the Infinity Cache; one event pair per launch, median of 20.
//   build: hipcc -O3 --offload-arch=gfx950 tools/stream_size.hip -o tools/_build/stream_size
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define LDS __attribute__((address_space(3)))

__device__ __forceinline__ void dma16nt(const void *src, LDS void *dst) {
    const unsigned m0 = (unsigned)(uintptr_t)dst;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m0), "v"(src)
                 : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void vmw() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int IPS, int D>
__global__ void stream(const unsigned char *buf, long per_wave, int waves_total, unsigned *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = wave * gridDim.x + blockIdx.x;  // kq_rows' map: adjacent streams on different CUs
    if (gw >= waves_total) return;
    unsigned char *ring = smem + wave * D * IPS * 1024;
    const unsigned char *src = buf + (long)gw * per_wave;
    const int T = (int)(per_wave / (IPS * 1024));
    int is = 0;
    auto issue = [&](int t) {
        unsigned char *slot = ring + (is % D) * IPS * 1024;
#pragma unroll
        for (int i = 0; i < IPS; ++i) dma16nt(src + (long)t * IPS * 1024 + i * 1024 + 16 * lane, (LDS void *)(slot + 1024 * i));
        ++is;
    };
    for (int t = 0; t < D && t < T; ++t) issue(t);
    unsigned acc = 0;
    for (int t = 0; t < T; ++t) {
        if (T - t >= D) vmw<IPS * (D - 1)>();
        else vmw<0>();
        acc += *(volatile unsigned *)(ring + (t % D) * IPS * 1024 + 4 * lane);
        if (t + D < T) issue(t + D);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// kq_rows' stream shape: steps of GR 16-B granules (Q4_K: 16 superblocks + 1 slack granule
// = 145: three instructions, the last with 17 lanes), D steps in flight, wave gw owns rows
// [gw*rbase + min(gw, rrem), ...) of RB bytes each (uneven shares as in kq_rows).
template <int GR, int D>
__global__ void rows_stream(const unsigned char *buf, long rb, int rbase, int rrem, int waves_total, unsigned *sink) {
    constexpr int NI = (GR + 63) / 64, SLOT = 16 * GR;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = wave * gridDim.x + blockIdx.x;
    if (gw >= waves_total) return;
    const int nrows = rbase + (gw < rrem ? 1 : 0);
    const long r0 = (long)gw * rbase + (gw < rrem ? gw : rrem);
    const unsigned char *src = buf + r0 * rb;
    const long bytes = nrows * rb;
    const int T = (int)((bytes + 16 * (GR - 1) - 1) / (16 * (GR - 1)));
    unsigned char *ring = smem + wave * D * SLOT;
    auto issue = [&](int t) {
        const unsigned char *base = src + (long)t * 16 * (GR - 1) + 16 * lane;
        unsigned char *slot = ring + (t % D) * SLOT;
#pragma unroll
        for (int i = 0; i < NI; ++i)
            if (i + 1 < NI || lane < GR - 64 * (NI - 1)) dma16nt(base + 1024 * i, (LDS void *)(slot + 1024 * i));
    };
    for (int t = 0; t < D && t < T; ++t) issue(t);
    unsigned acc = 0;
    for (int t = 0; t < T; ++t) {
        if (T - t >= D) vmw<NI * (D - 1)>();
        else vmw<0>();
        acc += *(volatile unsigned *)(ring + (t % D) * SLOT + 4 * lane);
        if (t + D < T) issue(t + D);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

void run_rows(unsigned char *pool, size_t pool_bytes, long rows, long rb, int waves_per_cu, int cus, unsigned *sink,
              bool even) {
    const int waves = cus * waves_per_cu;
    int rbase = (int)(rows / waves), rrem = (int)(rows % waves);
    long rbb = rb;
    if (even) {  // same bytes, every wave an equal share (rows resized)
        rbb = rows * rb / waves / 2304 * 2304;
        rbase = 1;
        rrem = 0;
    }
    constexpr int GR = 145, D = 3;
    const size_t lds = (size_t)waves_per_cu * D * 16 * GR;
    auto fn = rows_stream<GR, D>;
    hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const size_t bytes = (size_t)rows * rb;
    const int nbuf = (int)(pool_bytes / bytes) < 8 ? (int)(pool_bytes / bytes) : 8;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < 24; ++r) {
        const unsigned char *b = pool + (size_t)(r % nbuf) * bytes;
        hipExtLaunchKernelGGL(fn, dim3(cus), dim3(waves_per_cu * 64), lds, 0, e0, e1, 0, b, rbb, rbase, rrem, waves, sink);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 4) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2] * 1e3;
    printf("rows-shape %6.1f MB %s (ext events): %7.2f us  %.3f of 8 TB/s\n", bytes / 1e6, even ? "equal shares " : "kq_rows shares",
           us, bytes / (us * 1e-6) / 8e12);
}

template <int IPS, int D>
void run(unsigned char *pool, size_t pool_bytes, size_t bytes, int wpg, int wgs_per_cu, int cus, unsigned *sink) {
    const int waves = cus * wgs_per_cu * wpg;
    const long per_wave = (long)(bytes / waves) / (IPS * 1024) * (IPS * 1024);
    const size_t lds = (size_t)wpg * D * IPS * 1024;
    auto fn = stream<IPS, D>;
    hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int nbuf = (int)(pool_bytes / bytes) < 8 ? (int)(pool_bytes / bytes) : 8;
    std::vector<float> t;
    for (int r = 0; r < 24; ++r) {
        const unsigned char *b = pool + (size_t)(r % nbuf) * bytes;
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(fn, dim3(cus * wgs_per_cu), dim3(wpg * 64), lds, 0, b, per_wave, waves, sink);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 4) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2] * 1e3, moved = (double)per_wave * waves;
    printf("%7.1f MB  IPS=%d D=%d waves/WG=%2d WGs/CU=%d : %7.2f us  %7.1f GB/s  (%.3f of 8 TB/s)\n", moved / 1e6, IPS, D,
           wpg, wgs_per_cu, us, moved / (us * 1e-6) / 1e9, moved / (us * 1e-6) / 8e12);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const size_t pool = (size_t)3 << 30;
    unsigned char *buf;
    unsigned *sink;
    hipMalloc(&buf, pool);
    hipMalloc(&sink, 64);
    hipMemset(buf, 1, pool);
    hipDeviceSynchronize();
    // kq_rows' shape against an equal-share stream, 70B ffn_down (8192 rows x 16128 B) and
    // 8B ffn_up (14336 x 2304 B), launch events inside the kernel's dispatch (hipExt)
    for (int rep = 0; rep < 2; ++rep) {
        run_rows(buf, pool, 8192, 16128, 12, cus, sink, false);
        run_rows(buf, pool, 8192, 16128, 12, cus, sink, true);
        run_rows(buf, pool, 14336, 2304, 12, cus, sink, false);
        run_rows(buf, pool, 14336, 2304, 12, cus, sink, true);
    }
    const size_t sizes[] = {(size_t)13e6, (size_t)33e6, (size_t)66e6, (size_t)132e6, (size_t)265e6, (size_t)431e6};
    for (size_t s : sizes) {
        run<2, 4>(buf, pool, s, 4, 3, cus, sink);
        run<3, 3>(buf, pool, s, 12, 1, cus, sink);
        run<2, 6>(buf, pool, s, 12, 1, cus, sink);
    }
    hipFree(buf);
    hipFree(sink);
    return 0;
}
