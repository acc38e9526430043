// stream_bench.hip — LDS-DMA streaming ceiling on this MI355X: how fast can waves
// pull a once-read buffer into per-wave LDS rings (global_load_lds_dwordx4),
// as a function of waves per CU, instructions per step, ring depth and the nt
// (non-temporal) policy. No arithmetic: the number this prints is the roofline
// a decode GEMV can approach, not a kernel result.
//   build: hipcc -O3 --offload-arch=gfx950 tools/stream_bench.hip -o tools/_build/stream_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define LDS __attribute__((address_space(3)))

template <bool NT>
__device__ __forceinline__ void dma16(const void *src, LDS void *dst) {
    const unsigned m0 = (unsigned)(uintptr_t)dst;
    if (NT)
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m0), "v"(src)
                     : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(src)
                     : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void vmw() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Each wave streams `per_wave` contiguous bytes in steps of IPS KB (IPS
// instructions of 1 KB), D steps in flight. Grid: waves_total waves.
template <int IPS, int D, bool NT>
__global__ void stream(const unsigned char *buf, long per_wave, int waves_total, unsigned *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = blockIdx.x * (blockDim.x >> 6) + wave;
    if (gw >= waves_total) return;
    unsigned char *ring = smem + wave * D * IPS * 1024;
    const unsigned char *src = buf + (long)gw * per_wave;
    const int T = (int)(per_wave / (IPS * 1024));
    int is = 0;
    auto issue = [&](int t) {
        unsigned char *slot = ring + (is % D) * IPS * 1024;
#pragma unroll
        for (int i = 0; i < IPS; ++i) dma16<NT>(src + (long)t * IPS * 1024 + i * 1024 + 16 * lane, (LDS void *)(slot + 1024 * i));
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

template <int IPS, int D, bool NT>
void run(const unsigned char *buf, size_t bytes, int wpg, int wgs_per_cu, int cus, unsigned *sink) {
    const int waves = cus * wgs_per_cu * wpg;
    const long per_wave = (long)(bytes / waves) / (IPS * 1024) * (IPS * 1024);
    const size_t lds = (size_t)wpg * D * IPS * 1024;
    auto fn = stream<IPS, D, NT>;
    if (lds > 65536) hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, wpg * 64, lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(fn, dim3(cus * wgs_per_cu), dim3(wpg * 64), lds, 0, buf, per_wave, waves, sink);
    hipEventRecord(e0, 0);
    const int reps = 10;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(fn, dim3(cus * wgs_per_cu), dim3(wpg * 64), lds, 0, buf, per_wave, waves, sink);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double gbs = (double)per_wave * waves * reps / (ms * 1e-3) / 1e9;
    printf("IPS=%d KB/step D=%d nt=%d waves/WG=%d WGs/CU=%d (occ %d) inflight/CU=%5.1f KB : %7.1f GB/s\n", IPS, D,
           (int)NT, wpg, wgs_per_cu, occ, (double)wgs_per_cu * wpg * D * IPS, gbs);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const size_t bytes = (size_t)1 << 30;  // 1 GiB: far beyond the 256 MiB Infinity Cache
    unsigned char *buf;
    unsigned *sink;
    hipMalloc(&buf, bytes);
    hipMalloc(&sink, 64);
    hipMemset(buf, 1, bytes);
    printf("CUs=%d\n", cus);
    // vary in-flight bytes per CU and wave count
    run<1, 4, false>(buf, bytes, 4, 2, cus, sink);
    run<1, 8, false>(buf, bytes, 4, 2, cus, sink);
    run<1, 8, false>(buf, bytes, 4, 3, cus, sink);
    run<1, 8, true>(buf, bytes, 4, 3, cus, sink);
    run<2, 4, false>(buf, bytes, 4, 2, cus, sink);
    run<2, 4, false>(buf, bytes, 4, 3, cus, sink);
    run<2, 4, true>(buf, bytes, 4, 3, cus, sink);
    run<2, 6, true>(buf, bytes, 4, 3, cus, sink);
    run<4, 3, false>(buf, bytes, 4, 3, cus, sink);
    run<4, 3, true>(buf, bytes, 4, 3, cus, sink);
    run<4, 4, true>(buf, bytes, 4, 2, cus, sink);
    run<1, 16, true>(buf, bytes, 4, 2, cus, sink);
    run<2, 8, true>(buf, bytes, 4, 2, cus, sink);
    run<2, 8, true>(buf, bytes, 8, 1, cus, sink);
    run<2, 4, true>(buf, bytes, 8, 2, cus, sink);
    run<1, 8, true>(buf, bytes, 16, 1, cus, sink);
    run<3, 3, true>(buf, bytes, 4, 3, cus, sink);
    run<3, 4, true>(buf, bytes, 4, 3, cus, sink);
    hipFree(buf);
    hipFree(sink);
    return 0;
}
