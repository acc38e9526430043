// launch_floor.hip — per-launch floor of a decode stage on this MI355X: a chain of
// 89 back-to-back launches (TinyLlama's token) of kernels that do (almost) nothing,
// replayed from a hipGraph, for several launch shapes. The gap between this floor
// and kq_rows' ~5.3 us per stage is what any per-launch optimisation can win.
//   build: hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o tools/_build/launch_floor
#include <hip/hip_runtime.h>
#include <stdio.h>

// mode 0: return; mode 1: each wave reads 16 floats of x (the activation fetch) and
// lane 0 of wave 0 writes one float (a dependent chain through memory).
template <int MODE>
__global__ void stage(const float *x, float *y) {
    extern __shared__ float lds[];
    if (MODE == 0) return;
    float v = x[threadIdx.x & 255];
    lds[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) y[blockIdx.x] = lds[7] + 1.f;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    float *x, *y;
    hipMalloc(&x, 1 << 20);
    hipMalloc(&y, 1 << 20);
    hipMemset(x, 0, 1 << 20);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipFuncSetAttribute((const void *)stage<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void *)stage<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Cfg {
        int mode, wgs, threads, lds;
    } cfgs[] = {{0, cus, 768, 0},      {0, cus, 768, 100 << 10}, {0, cus, 256, 0},  {0, cus / 4, 256, 0},
                {1, cus, 768, 100 << 10}, {1, cus, 256, 0},      {1, cus / 4, 256, 0}, {1, 1, 64, 0},
                // the GEMV's 3072 waves as 12-wave / 4-wave workgroups, with their LDS
                {1, cus, 768, 0},         {1, 3 * cus, 256, 0},    {1, 3 * cus, 256, 32 << 10},
                {1, 2 * cus, 384, 50 << 10}, {1, 2 * cus, 256, 0}};
    for (const Cfg &c : cfgs) {
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < 89; ++i) {
            const float *xi = (i & 1) ? y : x;
            float *yi = (i & 1) ? x + 4096 : y;
            if (c.mode == 0) hipLaunchKernelGGL(stage<0>, dim3(c.wgs), dim3(c.threads), c.lds, s, xi, yi);
            else hipLaunchKernelGGL(stage<1>, dim3(c.wgs), dim3(c.threads), c.lds, s, xi, yi);
        }
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int w = 0; w < 5; ++w) hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        hipEventRecord(e0, s);
        const int reps = 50;
        for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, s);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("mode=%d wgs=%4d threads=%4d lds=%6d : %.2f us per launch (89-launch graph)\n", c.mode, c.wgs,
               c.threads, c.lds, ms * 1e3 / (reps * 89));
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
    }
    return 0;
}
