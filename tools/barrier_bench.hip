// barrier_bench.hip — cost of a grid-wide stage hand-off on this MI355X, the
// quantity that decides whether a persistent multi-stage decode kernel can beat
// one launch per GEMV (~1.5 us kernel boundary + cold start).
// One 768-thread workgroup per CU; per stage every workgroup publishes a slice of
// the stage output, arrives on a counter, waits for all, then reads the whole
// vector back (what the next GEMV's activation fetch does) and checks it.
//   modes 0/1: agent-scope release/acquire fences (L2 writeback + invalidate),
//              flat counter / per-XCD counters;
//   mode 4:    no counter — each published element carries its stage tag
//              (64-bit {value, tag} stored sc0 sc1); consumers re-read until
//              every tag matches: the activation read IS the barrier.
//   modes 2/3: no fences — the published slice is stored with sc0 sc1 (written
//              through to memory) and read back with sc0 sc1 loads (L2 miss), so
//              no L2 maintenance is needed; flat / per-XCD counters.
//   build: hipcc -O3 --offload-arch=gfx950 tools/barrier_bench.hip -o tools/_build/barrier_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ void store_sys(float *p, float v) {
    asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float4 load_sys4(const float4 *p) {
    float4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

__device__ __forceinline__ void store_sys2(float *p, float v, unsigned tag) {
    asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(make_uint2(__float_as_uint(v), tag)) : "memory");
}

// mode 4: tagged elements, vec holds 2 x vec_floats {value, tag} pairs per buffer
__global__ void __launch_bounds__(768) stages_tagged(float *vec, int n_stages, int vec_floats, unsigned *bad) {
    const int nwg = gridDim.x;
    unsigned nbad = 0;
    for (int s = 0; s < n_stages; ++s) {
        float *out = vec + (s & 1) * 2 * vec_floats;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < vec_floats; i += nwg * blockDim.x)
            store_sys2(out + 2 * i, (float)(s * 7 + (i & 1023)), (unsigned)s + 1);
        const float4 *v = (const float4 *)out;  // 2 elements per float4
        for (int i = threadIdx.x; i < vec_floats / 2; i += blockDim.x) {
            float4 a = load_sys4(v + i);
            int spins = 0;  // bail-out so a visibility bug cannot hang the GPU
            while ((__float_as_uint(a.y) != (unsigned)s + 1 || __float_as_uint(a.w) != (unsigned)s + 1) && ++spins < (1 << 12)) {
                __builtin_amdgcn_s_sleep(1);
                a = load_sys4(v + i);
            }
            const int e = 2 * i;
            nbad += a.x != (float)(s * 7 + ((e + 0) & 1023));
            nbad += a.z != (float)(s * 7 + ((e + 1) & 1023));
        }
        __syncthreads();  // the whole workgroup has consumed stage s before it publishes s+1
    }
    if (nbad) atomicAdd(bad, nbad);
}

// mode 5: {v0, v1, v2, tag} granules (one 16-byte store / load each): 5.3 B per element
__global__ void __launch_bounds__(768) stages_tagged3(float *vec, int n_stages, int vec_floats, unsigned *bad) {
    const int nwg = gridDim.x;
    const int ng = (vec_floats + 2) / 3;
    unsigned nbad = 0;
    for (int s = 0; s < n_stages; ++s) {
        float4 *out = (float4 *)(vec + (s & 1) * 2 * vec_floats);
        for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += nwg * blockDim.x) {
            const int e = 3 * g;
            float4 v = make_float4((float)(s * 7 + (e & 1023)), (float)(s * 7 + ((e + 1) & 1023)),
                                   (float)(s * 7 + ((e + 2) & 1023)), __uint_as_float((unsigned)s + 1));
            typedef float f4 __attribute__((ext_vector_type(4)));
            const f4 w = {v.x, v.y, v.z, v.w};
            asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(out + g), "v"(w) : "memory");
        }
        for (int g = threadIdx.x; g < ng; g += blockDim.x) {
            float4 a = load_sys4(out + g);
            int spins = 0;
            while (__float_as_uint(a.w) != (unsigned)s + 1 && ++spins < (1 << 12)) {
                __builtin_amdgcn_s_sleep(1);
                a = load_sys4(out + g);
            }
            const int e = 3 * g;
            nbad += a.x != (float)(s * 7 + (e & 1023));
            nbad += a.y != (float)(s * 7 + ((e + 1) & 1023));
            nbad += a.z != (float)(s * 7 + ((e + 2) & 1023));
        }
        __syncthreads();
    }
    if (nbad) atomicAdd(bad, nbad);
}

template <int MODE>
__global__ void __launch_bounds__(768) stages(unsigned *ctr, float *vec, int n_stages, int vec_floats, unsigned *bad) {
    const int nwg = gridDim.x;
    const bool nofence = MODE >= 2;
    const bool tree = MODE & 1;
    unsigned nbad = 0;
    for (int s = 0; s < n_stages; ++s) {
        float *out = vec + (s & 1) * vec_floats;
        // publish: this workgroup's slice of the stage output
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < vec_floats; i += nwg * blockDim.x) {
            const float v = (float)(s * 7 + (i & 1023));
            if (nofence) store_sys(out + i, v);
            else out[i] = v;
        }
        if (nofence) __builtin_amdgcn_s_waitcnt(0);  // stores acknowledged before arriving
        __syncthreads();
        if (threadIdx.x == 0) {
            if (!nofence) __atomic_thread_fence(__ATOMIC_RELEASE);
            if (!tree) {
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
            if (!nofence) __atomic_thread_fence(__ATOMIC_ACQUIRE);
        }
        __syncthreads();
        // consume: every workgroup reads the whole vector (the next stage's activation)
        const float4 *v = (const float4 *)out;
        for (int i = threadIdx.x; i < vec_floats / 4; i += blockDim.x) {
            const float4 a = nofence ? load_sys4(v + i) : v[i];
            const int e = 4 * i;
            nbad += a.x != (float)(s * 7 + ((e + 0) & 1023));
            nbad += a.y != (float)(s * 7 + ((e + 1) & 1023));
            nbad += a.z != (float)(s * 7 + ((e + 2) & 1023));
            nbad += a.w != (float)(s * 7 + ((e + 3) & 1023));
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    unsigned *ctr, *bad;
    float *vec;
    hipMalloc(&ctr, 4096);
    hipMalloc(&vec, 4 * 65536 * 4);
    hipMalloc(&bad, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[6] = {"fence-flat", "fence-xcd ", "sc-flat   ", "sc-xcd    ", "tagged    ", "tagged3   "};
    hipMemset(vec, 0, 4 * 65536 * 4);
    for (int mode = 0; mode < 6; ++mode) {
        if (only >= 0 && mode != only) continue;
        for (int vf : {2048, 5632, 32768}) {
            for (int S : {1, 200}) {
                float best = 1e30f;
                unsigned nbad = 0;
                for (int r = 0; r < 5; ++r) {
                    hipMemset(ctr, 0, 4096);
                    hipMemset(bad, 0, 64);
                    hipEventRecord(e0, 0);
                    switch (mode) {
                    case 0: hipLaunchKernelGGL(stages<0>, dim3(cus), dim3(768), 0, 0, ctr, vec, S, vf, bad); break;
                    case 1: hipLaunchKernelGGL(stages<1>, dim3(cus), dim3(768), 0, 0, ctr, vec, S, vf, bad); break;
                    case 2: hipLaunchKernelGGL(stages<2>, dim3(cus), dim3(768), 0, 0, ctr, vec, S, vf, bad); break;
                    case 3: hipLaunchKernelGGL(stages<3>, dim3(cus), dim3(768), 0, 0, ctr, vec, S, vf, bad); break;
                    case 4: hipMemset(vec, 0, 4 * 65536 * 4); hipEventRecord(e0, 0);
                        hipLaunchKernelGGL(stages_tagged, dim3(cus), dim3(768), 0, 0, vec, S, vf, bad); break;
                    default: hipMemset(vec, 0, 4 * 65536 * 4); hipEventRecord(e0, 0);
                        hipLaunchKernelGGL(stages_tagged3, dim3(cus), dim3(768), 0, 0, vec, S, vf, bad); break;
                    }
                    hipEventRecord(e1, 0);
                    hipEventSynchronize(e1);
                    float ms;
                    hipEventElapsedTime(&ms, e0, e1);
                    best = ms < best ? ms : best;
                    unsigned b = 0;
                    hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost);
                    nbad += b;
                }
                printf("mode=%s vec=%5d floats stages=%3d : %8.2f us total, %6.2f us/stage  mismatches=%u\n",
                       names[mode], vf, S, best * 1e3, best * 1e3 / S, nbad);
            }
        }
    }
    return 0;
}
