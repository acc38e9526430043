// barrier_bench.hip — cost of a grid-wide stage hand-off on this MI355X, the
// quantity that decides whether a persistent multi-stage decode kernel can beat
// one launch per GEMV (~1.5 us kernel boundary + cold start).
// One 768-thread workgroup per CU; per stage every workgroup publishes a slice of
// the stage output (plain stores + release fence), arrives on a counter, waits for
// all, then reads the whole vector back (what the next GEMV's activation fetch does).
//   build: hipcc -O3 --offload-arch=gfx950 tools/barrier_bench.hip -o tools/_build/barrier_bench
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE>  // 0: one counter; 1: per-XCD counters + top counter
__global__ void __launch_bounds__(768) stages(unsigned *ctr, float *vec, int n_stages, int vec_floats, float *sink) {
    const int lane = threadIdx.x & 63;
    const int nwg = gridDim.x;
    float acc = 0.f;
    for (int s = 0; s < n_stages; ++s) {
        // publish: this workgroup's slice of the stage output
        const int per = vec_floats / nwg;
        if (threadIdx.x < per) vec[(s & 1) * vec_floats + blockIdx.x * per + threadIdx.x] = (float)s;
        __syncthreads();
        if (threadIdx.x == 0) {
            __atomic_thread_fence(__ATOMIC_RELEASE);  // agent-scope release (L2 writeback)
            if (MODE == 0) {
                __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned target = (unsigned)(s + 1) * nwg;
                while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
                    __builtin_amdgcn_s_sleep(1);
            } else {
                const int xcd = blockIdx.x & 7;  // round-robin placement
                const unsigned per_xcd = (unsigned)((nwg - xcd + 7) / 8);
                const unsigned old = __hip_atomic_fetch_add(ctr + 64 + 64 * xcd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (old + 1 == (unsigned)(s + 1) * per_xcd)  // last of its XCD
                    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned target = (unsigned)(s + 1) * 8u;
                while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
                    __builtin_amdgcn_s_sleep(1);
            }
            __atomic_thread_fence(__ATOMIC_ACQUIRE);  // agent-scope acquire (L2 invalidate)
        }
        __syncthreads();
        // consume: every workgroup reads the whole vector (the next stage's activation)
        const float *v = vec + (s & 1) * vec_floats;
        for (int i = threadIdx.x; i < vec_floats; i += blockDim.x) acc += v[i];
        (void)lane;
    }
    if (acc == -1.f) sink[0] = acc;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    unsigned *ctr;
    float *vec, *sink;
    hipMalloc(&ctr, 4096);
    hipMalloc(&vec, 2 * 65536 * 4);
    hipMalloc(&sink, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int mode = 0; mode < 2; ++mode) {
        for (int vf : {2048, 5632, 32768}) {
            for (int S : {1, 200}) {
                float best = 1e30f;
                for (int r = 0; r < 5; ++r) {
                    hipMemset(ctr, 0, 4096);
                    hipEventRecord(e0, 0);
                    if (mode == 0) hipLaunchKernelGGL(stages<0>, dim3(cus), dim3(768), 0, 0, ctr, vec, S, vf, sink);
                    else hipLaunchKernelGGL(stages<1>, dim3(cus), dim3(768), 0, 0, ctr, vec, S, vf, sink);
                    hipEventRecord(e1, 0);
                    hipEventSynchronize(e1);
                    float ms;
                    hipEventElapsedTime(&ms, e0, e1);
                    best = ms < best ? ms : best;
                }
                printf("mode=%s vec=%5d floats stages=%3d : %8.2f us total, %6.2f us/stage\n",
                       mode ? "xcd-tree" : "flat    ", vf, S, best * 1e3, best * 1e3 / S);
            }
        }
    }
    return 0;
}
