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

int main() {
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
