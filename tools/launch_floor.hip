// launch_floor.hip — the dispatch floor of back-to-back launches (round 5).
// The decode token is ~90 launches; its model prices each GEMV's fixed part at
// ~3.4 us and an empty attention-shaped launch at ~4.2 us in event timing. This probe
// replays, from a hipGraph and eagerly, 60 launches of an empty kernel that records
// s_memrealtime at the entry of every workgroup, for several block sizes, grid sizes and
// kernarg sizes, and prints the median interval between consecutive launches' first
// entries (the dispatch cadence) and the median entry spread within a launch.
//   build: hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o tools/_build/launch_floor
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

struct Big {  // kernarg payload of kq_rows' order of size
    unsigned long long *rec;
    int pad[250];
};

__global__ void entry_small(unsigned long long *rec) {
    if (threadIdx.x == 0) rec[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

__global__ void entry_big(const Big a) {
    if (threadIdx.x == 0)
        a.rec[blockIdx.x] = __builtin_amdgcn_s_memrealtime() + (unsigned long long)a.pad[blockIdx.x & 127] * 0;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int launches = 60, maxwg = 2048;
    unsigned long long *rec;
    hipMalloc(&rec, (size_t)launches * maxwg * 8);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::vector<unsigned long long> h((size_t)launches * maxwg);
    struct Cfg {
        int wgs, threads, big;
    } cfgs[] = {{256, 768, 0}, {256, 768, 1}, {256, 384, 0}, {256, 256, 0}, {256, 64, 0},
                {512, 384, 0}, {1024, 256, 0}, {2048, 256, 0}, {64, 768, 0}, {8, 64, 0}};
    for (int graph = 0; graph < 2; ++graph) {
        for (const Cfg &c : cfgs) {
            hipMemset(rec, 0, (size_t)launches * maxwg * 8);
            auto issue = [&]() {
                for (int l = 0; l < launches; ++l) {
                    if (c.big) {
                        Big b{};
                        b.rec = rec + (size_t)l * maxwg;
                        hipLaunchKernelGGL(entry_big, dim3(c.wgs), dim3(c.threads), 0, s, b);
                    } else {
                        hipLaunchKernelGGL(entry_small, dim3(c.wgs), dim3(c.threads), 0, s, rec + (size_t)l * maxwg);
                    }
                }
            };
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            float ms = 0;
            if (graph) {
                hipGraph_t g;
                hipGraphExec_t ge;
                hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
                issue();
                hipStreamEndCapture(s, &g);
                hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
                for (int r = 0; r < 3; ++r) hipGraphLaunch(ge, s);
                hipEventRecord(e0, s);
                hipGraphLaunch(ge, s);
                hipEventRecord(e1, s);
                hipStreamSynchronize(s);
                hipGraphExecDestroy(ge);
                hipGraphDestroy(g);
            } else {
                for (int r = 0; r < 3; ++r) issue();
                hipEventRecord(e0, s);
                issue();
                hipEventRecord(e1, s);
                hipStreamSynchronize(s);
            }
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost);
            std::vector<double> cad, spr;
            unsigned long long prev = 0;
            for (int l = 0; l < launches; ++l) {
                const unsigned long long *r = h.data() + (size_t)l * maxwg;
                unsigned long long mn = ~0ull, mx = 0;
                for (int b = 0; b < c.wgs; ++b) mn = std::min(mn, r[b]), mx = std::max(mx, r[b]);
                spr.push_back((mx - mn) / 100.0);
                if (l) cad.push_back(((long long)mn - (long long)prev) / 100.0);
                prev = mn;
            }
            std::sort(cad.begin(), cad.end());
            std::sort(spr.begin(), spr.end());
            printf("%s wgs %4d x %3d threads kernarg %4zu B: cadence med %.2f us (p10 %.2f p90 %.2f) | entry spread med %.2f us | "
                   "events %.2f us/launch\n",
                   graph ? "graph" : "eager", c.wgs, c.threads, c.big ? sizeof(Big) : sizeof(void *), cad[cad.size() / 2],
                   cad[cad.size() / 10], cad[cad.size() * 9 / 10], spr[spr.size() / 2], ms * 1000 / launches);
        }
    }
    return 0;
}
