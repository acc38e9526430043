// slot_cost.hip — what one more (empty or tiny) launch costs inside a decode-like chain:
// hipGraphs of 88 launches replayed back to back, where "S" streams a fresh 3 MB slice of a
// 1 GiB buffer (256 workgroups, non-temporal 16-B loads, one float out per workgroup: a GEMV's
// shape without its arithmetic) and "E" is a 32-workgroup kernel that returns at once, "R"
// one that reads 8 KB written by the previous launch and writes 8 KB (an attention's
// dependent shape without its body). Per chain: us per launch; the added cost of E / R
// after S = (T(S,X,S,X...) - T(S only) / 2) / (launches / 2).
//   build: hipcc -O3 --offload-arch=gfx950 tools/slot_cost.hip -o tools/_build/slot_cost
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512) stream_k(const f4 *__restrict__ src, size_t n4_per_wg, float *__restrict__ out) {
    const f4 *p = src + (size_t)blockIdx.x * n4_per_wg;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (size_t i = threadIdx.x; i < n4_per_wg; i += 512) acc += __builtin_nontemporal_load(p + i);
    float v = acc.x + acc.y + acc.z + acc.w;
    __shared__ float red[512];
    red[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int i = 0; i < 512; i += 64) s += red[i];
        out[blockIdx.x] = s;
    }
}

__global__ void __launch_bounds__(256) empty_k(float *) {}

__global__ void __launch_bounds__(256) dep_k(const float *__restrict__ in, float *__restrict__ out) {
    // 8 KB in (2048 floats), 8 KB out, spread over the workgroups
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < 2048) out[i] = in[i] * 0.5f + 1.f;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const size_t big = (size_t)1 << 30;
    const size_t slice = 3u << 20;  // bytes per S launch
    f4 *buf;
    float *o1, *o2;
    hipMalloc(&buf, big);
    hipMemset(buf, 0, big);
    hipMalloc(&o1, 1 << 20);
    hipMalloc(&o2, 1 << 20);
    hipMemset(o1, 0, 1 << 20);
    hipMemset(o2, 0, 1 << 20);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"S only", "S,E alternating", "S,R alternating", "E only", "R only"};
    const int L = 88;
    size_t off = 0;
    for (int mode = 0; mode < 5; ++mode) {
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < L; ++i) {
            const bool is_s = mode == 0 || ((mode == 1 || mode == 2) && (i & 1) == 0);
            if (is_s) {
                hipLaunchKernelGGL(stream_k, dim3(256), dim3(512), 0, s, (const f4 *)((char *)buf + off),
                                   slice / 16 / 256, o1);
                off = (off + slice) % (big - slice);
            } else if (mode == 1 || mode == 3) {
                hipLaunchKernelGGL(empty_k, dim3(32), dim3(256), 0, s, o2);
            } else {
                hipLaunchKernelGGL(dep_k, dim3(32), dim3(256), 0, s, (i & 1) ? o1 : o2, (i & 1) ? o2 : o1);
            }
        }
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int w = 0; w < 5; ++w) hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        const int reps = 40;
        hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, s);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-18s : %.3f us per launch, %.1f us per %d-launch graph\n", names[mode], ms * 1e3 / (reps * L),
               ms * 1e3 / reps, L);
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
    }
    return 0;
}
