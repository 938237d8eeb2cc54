// wave_placement_probe.hip -- diagnostic only (not part of the product):
// which SIMD each wave of a workgroup lands on.  Every wave reads HW_ID
// (SIMD_ID bits [5:4], CU_ID bits [11:8]) and holds its CU for a while so
// workgroups co-reside as they do in the hashing kernels; the host prints,
// per workgroup size, how often wave w sits on SIMD (simd(wave 0) + d) % 4.
//   hipcc --offload-arch=gfx950 -O3 tools/wave_placement_probe.hip -o tools/wave_placement_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__global__ void placement(uint32_t* out, int spin) {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * (blockDim.x >> 6) + wave] = hw;
    // keep the workgroup resident so later workgroups share CUs with it
    uint64_t t0 = __builtin_readcyclecounter();
    while (__builtin_readcyclecounter() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(1);
}

// XCD spread of a launch: XCC_ID and (SE, SH, CU) of every workgroup's wave 0
__global__ void xcd_spread(uint32_t* out, int spin) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc & 0xf;
        out[2 * blockIdx.x + 1] = hw;
    }
    uint64_t t0 = __builtin_readcyclecounter();
    while (__builtin_readcyclecounter() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(1);
}

static void spread(int groups, int threads) {
    uint32_t* d;
    CHECK(hipMalloc(&d, groups * 8));
    hipLaunchKernelGGL(xcd_spread, dim3(groups), dim3(threads), 0, 0, d, 400000);
    CHECK(hipDeviceSynchronize());
    std::vector<uint32_t> h(2 * groups);
    CHECK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    CHECK(hipFree(d));
    int per_xcc[16] = {0};
    std::vector<uint32_t> cus;  // (xcc, se, sh, cu) keys
    for (int g = 0; g < groups; ++g) {
        const uint32_t x = h[2 * g], hw = h[2 * g + 1];
        per_xcc[x]++;
        cus.push_back((x << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15));
    }
    std::sort(cus.begin(), cus.end());
    const long distinct = std::unique(cus.begin(), cus.end()) - cus.begin();
    printf("{\"xcd_spread\": {\"workgroups\": %d, \"threads\": %d, \"distinct_cus\": %ld, \"per_xcc\": [", groups,
           threads, distinct);
    for (int x = 0; x < 8; ++x) printf("%s%d", x ? ", " : "", per_xcc[x]);
    printf("]}}\n");
}

int main() {
    spread(64, 256);    // config 2: 4096 chunks, the one-group split kernel
    spread(256, 512);   // 32768 chunks: the 8-wave two-group kernel
    spread(256, 256);   // 16384 chunks
    const int sizes[] = {2, 3, 4, 6, 8};
    for (int nw : sizes) {
        for (int groups : {256, 512}) {
            uint32_t* d;
            CHECK(hipMalloc(&d, groups * nw * 4));
            hipLaunchKernelGGL(placement, dim3(groups), dim3(64 * nw), 0, 0, d, 200000);
            CHECK(hipDeviceSynchronize());
            std::vector<uint32_t> h(groups * nw);
            CHECK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
            CHECK(hipFree(d));
            // hist[w][delta]: wave w on SIMD simd(wave0)+delta
            std::vector<int> hist(nw * 4, 0);
            int same_cu = 0;
            for (int g = 0; g < groups; ++g) {
                const uint32_t s0 = (h[g * nw] >> 4) & 3, cu0 = (h[g * nw] >> 8) & 15;
                for (int w = 0; w < nw; ++w) {
                    const uint32_t s = (h[g * nw + w] >> 4) & 3, cu = (h[g * nw + w] >> 8) & 15;
                    hist[w * 4 + ((s - s0) & 3)]++;
                    same_cu += cu == cu0;
                }
            }
            printf("{\"waves_per_group\": %d, \"groups\": %d, \"same_cu_frac\": %.3f, \"simd_delta_hist\": [", nw,
                   groups, same_cu / (double)(groups * nw));
            for (int w = 0; w < nw; ++w)
                printf("%s[%d, %d, %d, %d]", w ? ", " : "", hist[w * 4], hist[w * 4 + 1], hist[w * 4 + 2],
                       hist[w * 4 + 3]);
            printf("]}\n");
        }
    }
    return 0;
}
