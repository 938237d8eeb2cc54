// sim_probe.hip -- shader cycles per job of the mixed planner's own
// dispatch simulation (sim_xcd, compiled from sha1_kernels.hip) on one
// candidate (8 lanes: one per XCD, as in the planner's first pass), in a
// 64-thread workgroup and in the planner's 1024-thread one (the other waves
// waiting at a barrier).  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I congestion-control-with-bittorren_amd/csrc tools/sim_probe.hip -o tools/sim_probe
#include "sha1_kernels.hip"

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(1024) void sim_probe(const uint32_t* gblocks, const uint8_t* grun, uint32_t G, uint32_t H,
                                                  uint32_t F, uint32_t ncand, uint64_t* cyc, float* out) {
    __shared__ uint32_t blocks[kSimMaxG];  // as the planner keeps them: the run in bits 28-31
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) blocks[g] = gblocks[g] | (uint32_t)grun[g] << 28;
    __syncthreads();
    __shared__ uint32_t longest;
    if (threadIdx.x == 0) longest = 0;
    __syncthreads();
    const uint32_t t = threadIdx.x, c = t / kSimXcds, x = t % kSimXcds;
    // per-lane runtime mode and F, as in the planner (gblocks[G + c] = 0 / 8)
    const uint32_t mode = gblocks[G] & 0u, f = c & 1u ? F : F;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    float mk = 0.0f;
    if (c < ncand) mk = sim_xcd(blocks, G, mode, H - 8u + c, f, x, kSimCus);
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    if (c < ncand && (t & 63u) == 0u) atomicMax(&longest, static_cast<uint32_t>(c1 - c0));
    __syncthreads();
    out[t] = mk;
    if (t == 0) *cyc = longest;
}

int main() {
    const uint32_t G = 2048, H = 191, F = 4;
    std::vector<uint32_t> b(G);
    std::vector<uint8_t> r(G, 0);
    for (uint32_t g = 0; g < G; ++g) b[g] = 16385u - g * 7u;
    uint32_t* db;
    uint8_t* dr;
    uint64_t* cyc;
    float* out;
    (void)hipMalloc(&db, (G + 1) * 4);
    (void)hipMalloc(&dr, G);
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&out, 1024 * 4);
    b.push_back(0u);
    (void)hipMemcpy(db, b.data(), (G + 1) * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dr, r.data(), G, hipMemcpyHostToDevice);
    const uint32_t J = H + (G - H + F - 1) / F;
    for (int threads : {64, 1024}) {
        for (uint32_t nc : {1u, 8u, 16u, 28u, 44u}) {
            if (nc * 8 > (uint32_t)threads) continue;
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(sim_probe, 1, threads, 0, 0, db, dr, G, H, F, nc, cyc, out);
                uint64_t c = 0;
                (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
                if (rep == 2)
                    printf("{\"threads\": %d, \"candidates\": %u, \"jobs_per_lane\": %u, \"cycles\": %llu, "
                           "\"cycles_per_job\": %.1f}\n",
                           threads, nc, (J + 7) / 8, (unsigned long long)c, (double)c / ((J + 7) / 8));
            }
        }
    }
    return 0;
}
