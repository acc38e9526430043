// percu_stream.hip — how fast can a FEW workgroups pull a small weight slice each?
// (feasibility of a fused q/k/v + attention launch: one workgroup per query head streams
// its q rows and its group's k/v rows, ~221 KB for TinyLlama, on 32 of the 256 CUs.)
// Each workgroup streams `per_wg` contiguous bytes split over its waves into per-wave LDS
// rings (LDS-DMA nt, 2 KB steps, D in flight); one launch per timing, buffers rotated over
// > 512 MB so every launch reads cold HBM. Prints us per launch (hipEvent pair) and GB/s.
//   build: hipcc -O3 --offload-arch=gfx950 tools/percu_stream.hip -o tools/_build/percu_stream
#include <hip/hip_runtime.h>
#include <stdio.h>

#define LDS __attribute__((address_space(3)))

__device__ __forceinline__ void dma16nt(const void *src, LDS void *dst) {
    const unsigned m0 = (unsigned)(uintptr_t)dst;
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m0), "v"(src) : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void vmw() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int D>
__global__ void stream(const unsigned char *buf, long per_wg, unsigned *sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const long per_wave = per_wg / nw / 2048 * 2048;
    unsigned char *ring = smem + wave * D * 2048;
    const unsigned char *src = buf + (long)blockIdx.x * per_wg + (long)wave * per_wave;
    const int T = (int)(per_wave / 2048);
    int is = 0;
    auto issue = [&](int t) {
        unsigned char *slot = ring + (is % D) * 2048;
        dma16nt(src + (long)t * 2048 + 16 * lane, (LDS void *)slot);
        dma16nt(src + (long)t * 2048 + 1024 + 16 * lane, (LDS void *)(slot + 1024));
        ++is;
    };
    for (int t = 0; t < D && t < T; ++t) issue(t);
    unsigned acc = 0;
    for (int t = 0; t < T; ++t) {
        if (T - t >= D) vmw<2 * (D - 1)>();
        else vmw<0>();
        acc += *(volatile unsigned *)(ring + (t % D) * 2048 + 4 * lane);
        if (t + D < T) issue(t + D);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int D>
void run(const unsigned char *buf, size_t bytes, int wgs, int waves, long per_wg, unsigned *sink) {
    const size_t lds = (size_t)waves * D * 2048;
    auto fn = stream<D>;
    if (lds > 65536) hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const long span = (long)wgs * per_wg;
    const int nrot = (int)(bytes / span);
    float tot = 0;
    const int reps = 40;
    for (int r = 0; r < reps + 3; ++r) {
        const unsigned char *b = buf + (long)(r % nrot) * span;
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(fn, dim3(wgs), dim3(waves * 64), lds, 0, b, per_wg, sink);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 3) tot += ms;
    }
    const double us = tot * 1e3 / reps;
    printf("WGs=%4d waves=%2d D=%d per_wg=%7.1f KB total=%7.2f MB : %7.2f us/launch  %7.1f GB/s  (%5.1f GB/s per WG)\n",
           wgs, waves, D, per_wg / 1024.0, span / 1e6, us, span / (us * 1e-6) / 1e9, per_wg / (us * 1e-6) / 1e9);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    unsigned char *buf;
    unsigned *sink;
    hipMalloc(&buf, bytes);
    hipMalloc(&sink, 64);
    hipMemset(buf, 1, bytes);
    // the current q/k/v launch: 2.97 MB over 256 workgroups of 6 waves
    run<3>(buf, bytes, 256, 6, 12 * 1024, sink);
    run<3>(buf, bytes, 256, 6, 2970000 / 256 / 2048 * 2048, sink);
    // one workgroup per query head: 32 x 221 KB (q head rows + the group's k / v rows)
    for (int w : {4, 8, 12, 16}) {
        run<3>(buf, bytes, 32, w, 221184, sink);
        run<4>(buf, bytes, 32, w, 221184, sink);
    }
    run<6>(buf, bytes, 32, 12, 221184, sink);
    run<8>(buf, bytes, 32, 8, 221184, sink);
    // 64 workgroups (two per head, half the rows each) for comparison
    run<4>(buf, bytes, 64, 12, 110592, sink);
    hipFree(buf);
    hipFree(sink);
    return 0;
}
