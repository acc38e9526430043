// xfresh.hip — what a consumer launch pays for reading an activation the previous launch
// just wrote, by the writer's store flavour. hipGraphs of 88 launches, alternating a writer
// (256 workgroups, each storing its 32-B slice of an 8 KB vector: the shape of a GEMV's
// output) and a consumer (256 workgroups of 256 threads, each reading the whole 8 KB: the
// shape of the next GEMV's activation fetch, then one float out). The consumer reads either
// the vector just written (fresh) or another one nobody writes (stable); fresh - stable is
// the hand-off's price for that store flavour.
//   build: hipcc -O3 --offload-arch=gfx950 tools/xfresh.hip -o tools/_build/xfresh
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int FLAVOUR>
__global__ void __launch_bounds__(64) writer(u32x4 *x, unsigned seed) {
    if (threadIdx.x >= 2) return;
    u32x4 *p = x + blockIdx.x * 2 + threadIdx.x;
    const u32x4 v = {seed, seed + 1u, seed + 2u, blockIdx.x};
    if (FLAVOUR == 0) *p = v;
    if (FLAVOUR == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    if (FLAVOUR == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    if (FLAVOUR == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

__global__ void __launch_bounds__(256) consumer(const u32x4 *__restrict__ x, unsigned *__restrict__ out) {
    const u32x4 a = x[threadIdx.x], b = x[256 + threadIdx.x];
    unsigned v = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
    __shared__ unsigned red[256];
    red[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned s = 0;
        for (int i = 0; i < 256; i += 32) s ^= red[i];
        out[blockIdx.x] = s;
    }
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    u32x4 *x, *y;
    unsigned *out;
    (void)hipMalloc(&x, 1 << 16);
    (void)hipMalloc(&y, 1 << 16);
    (void)hipMalloc(&out, 1 << 16);
    (void)hipMemset(x, 0, 1 << 16);
    (void)hipMemset(y, 0, 1 << 16);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *fl[] = {"plain", "nt", "sc1", "sc0 sc1"};
    const int L = 88;
    for (int f = 0; f < 4; ++f) {
        for (int fresh = 1; fresh >= 0; --fresh) {
            hipGraph_t g;
            hipGraphExec_t ge;
            (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
            for (int i = 0; i < L / 2; ++i) {
                if (f == 0) hipLaunchKernelGGL(writer<0>, dim3(256), dim3(64), 0, s, x, (unsigned)i);
                if (f == 1) hipLaunchKernelGGL(writer<1>, dim3(256), dim3(64), 0, s, x, (unsigned)i);
                if (f == 2) hipLaunchKernelGGL(writer<2>, dim3(256), dim3(64), 0, s, x, (unsigned)i);
                if (f == 3) hipLaunchKernelGGL(writer<3>, dim3(256), dim3(64), 0, s, x, (unsigned)i);
                hipLaunchKernelGGL(consumer, dim3(256), dim3(256), 0, s, fresh ? x : y, out);
            }
            (void)hipStreamEndCapture(s, &g);
            (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            for (int w = 0; w < 5; ++w) (void)hipGraphLaunch(ge, s);
            (void)hipStreamSynchronize(s);
            const int reps = 40;
            (void)hipEventRecord(e0, s);
            for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, s);
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("writer %-8s consumer reads %-6s : %.3f us per (writer, consumer) pair\n", fl[f], fresh ? "fresh" : "stable",
                   ms * 1e3 / (reps * (L / 2)));
            (void)hipGraphExecDestroy(ge);
            (void)hipGraphDestroy(g);
        }
    }
    return 0;
}
