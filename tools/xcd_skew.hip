// xcd_skew.hip — when does each XCD start its workgroups of a launch? (round 5)
// kq_rows' per-wave stamps showed the TinyLlama-shaped GEMVs starting their workgroups
// XCD by XCD over ~1.5 us (logical XCD = block % 8), and their ends following (corr 0.99),
// while the Llama-3-8B shapes started within 0.3 us. This probe launches a kernel of
// 256 workgroups x 12 waves that records, per workgroup, s_memrealtime at entry and the
// physical XCC id, then spins for SPIN us; back-to-back launches (eager, then replayed from
// a hipGraph), several spin lengths and LDS sizes. Output: per launch shape, the median
// entry of each XCC relative to the launch's first workgroup.
//   build: hipcc -O3 --offload-arch=gfx950 tools/xcd_skew.hip -o tools/_build/xcd_skew
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <chrono>
#include <vector>

__global__ void __launch_bounds__(768) probe(unsigned long long *rec, int spin_ticks, int slow_xcc, int extra_ticks) {
    extern __shared__ float lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) {
        rec[2 * blockIdx.x] = t0;
        rec[2 * blockIdx.x + 1] = xcc & 0xf;
    }
    const int ticks = spin_ticks + ((int)(xcc & 0xf) == slow_xcc ? extra_ticks : 0);
    if (ticks > 0) {
        while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 1) lds[0] = 1.f;  // (touch the LDS allocation)
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int wgs = p.multiProcessorCount;  // one per CU, as kq_rows
    const int launches = 40;
    unsigned long long *rec;
    hipMalloc(&rec, (size_t)launches * wgs * 2 * 8);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    // slow: XCC whose workgroups spin extra_us longer (-1: none). If a launch's dispatch
    // waited for the previous launch per XCC rather than for all of it, the next launch
    // would start later on that XCC only.
    struct Cfg {
        int spin_us, lds_kb, graph, slow, extra_us, gap_us = 0;
    } cfgs[] = {{5, 0, 0, -1, 0, 10}, {5, 0, 0, -1, 0, 30}, {5, 96, 0, -1, 0, 30}, {5, 0, 0, -1, 0, 100}, {0, 0, 0, -1, 0}, {2, 0, 0, -1, 0}, {5, 0, 0, -1, 0}, {10, 0, 0, -1, 0}, {2, 64, 0, -1, 0},
                {5, 96, 0, -1, 0}, {2, 0, 1, -1, 0}, {5, 0, 1, -1, 0}, {5, 96, 1, -1, 0}, {5, 0, 0, 4, 3},
                {5, 0, 1, 4, 3}, {5, 0, 0, 0, 3}};
    std::vector<unsigned long long> h((size_t)launches * wgs * 2);
    for (const Cfg &c : cfgs) {
        const int ticks = c.spin_us * 100;  // 100 MHz
        const size_t lds = (size_t)c.lds_kb << 10;
        auto issue = [&]() {
            for (int l = 0; l < launches; ++l) {
                hipLaunchKernelGGL(probe, dim3(wgs), dim3(768), lds, s, rec + (size_t)l * wgs * 2, ticks, c.slow,
                                   c.extra_us * 100);
                if (c.gap_us) {  // host-side gap: the GPU goes idle between launches (as eager Python launches do)
                    const auto t = std::chrono::steady_clock::now();
                    while (std::chrono::steady_clock::now() - t < std::chrono::microseconds(c.gap_us)) {
                    }
                }
            }
        };
        if (c.graph) {
            hipGraph_t g;
            hipGraphExec_t ge;
            hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
            issue();
            hipStreamEndCapture(s, &g);
            hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
            for (int r = 0; r < 3; ++r) hipGraphLaunch(ge, s);
            hipStreamSynchronize(s);
            hipGraphExecDestroy(ge);
            hipGraphDestroy(g);
        } else {
            for (int r = 0; r < 3; ++r) issue();
            hipStreamSynchronize(s);
        }
        hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost);
        // per XCC: median over the last 20 launches of (entry - launch's first entry), in us
        std::vector<double> per[8], spread;
        std::vector<int> order_votes(8, 0);
        for (int l = launches - 20; l < launches; ++l) {
            const unsigned long long *r = h.data() + (size_t)l * wgs * 2;
            unsigned long long mn = ~0ull, mx = 0;
            for (int b = 0; b < wgs; ++b) mn = std::min(mn, r[2 * b]), mx = std::max(mx, r[2 * b]);
            spread.push_back((mx - mn) / 100.0);
            std::vector<double> xmed[8];
            for (int b = 0; b < wgs; ++b) xmed[r[2 * b + 1] & 7].push_back((r[2 * b] - mn) / 100.0);
            for (int x = 0; x < 8; ++x) {
                if (xmed[x].empty()) continue;
                std::sort(xmed[x].begin(), xmed[x].end());
                per[x].push_back(xmed[x][xmed[x].size() / 2]);
            }
        }
        std::sort(spread.begin(), spread.end());
        printf("gap %3d us spin %2d us lds %3d KB %s slow xcc %2d +%d us: launch start spread med %.2f us | per-XCC median entry (us):",
               c.gap_us, c.spin_us, c.lds_kb, c.graph ? "graph" : "eager", c.slow, c.extra_us, spread[spread.size() / 2]);
        for (int x = 0; x < 8; ++x) {
            if (per[x].empty()) {
                printf("  x%d -", x);
                continue;
            }
            std::sort(per[x].begin(), per[x].end());
            printf("  x%d %.2f", x, per[x][per[x].size() / 2]);
        }
        // block -> XCC map of the last launch (first 16 blocks)
        const unsigned long long *r = h.data() + (size_t)(launches - 1) * wgs * 2;
        printf("  | blocks 0..15 on XCC:");
        for (int b = 0; b < 16; ++b) printf(" %llu", r[2 * b + 1]);
        printf("\n");
    }
    return 0;
}
