// coop_probe.hip -- in a scattered chunk layout, is it the number of chunks
// one load instruction touches that thrashes the CU's translation cache
// (tools/tlb_probe.sh), or the number of chunks resident per CU?  Reads N
// chunks of L bytes, each exactly once, in three patterns, with chunk c at
// byte offset off[c] (in place: c * L; scattered: a random permutation):
//
//   lane    lane = chunk (the hash kernels' pattern): 16-byte loads, 128
//           bytes per lane per stage, so one dwordx4 instruction touches 64
//           chunks
//   coop8   8 lanes per chunk: one instruction reads 128 bytes of each of 8
//           chunks (8 chunks per instruction)
//   coop64  64 lanes per chunk: one instruction reads 1 KiB of one chunk
//
// Layouts: in place, permuted at random, and permuted in runs of 4
// adjacent chunks.  Every wave owns 64 chunks and every pattern reads the same bytes; 256
// threads per workgroup, N / 256 workgroups (N = 65536: one per CU, four
// waves = 256 resident chunks per CU, the fused kernel's F = 4 shape).
// XOR/add-folded into one dword per lane so nothing is dead.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/coop_probe tools/coop_probe.hip
// run:   tools/coop_probe [chunks] [chunk_bytes]  -> one JSON line per (layout, pattern)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

__device__ __forceinline__ void fold(uint32_t& a, uint32_t& b, const uint4& v) {
    a ^= v.x ^ v.z;
    b += v.y + v.w;
}

// lane = chunk
__global__ __launch_bounds__(256) void read_lane(const uint8_t* __restrict__ base,
                                                 const uint64_t* __restrict__ off, uint32_t L,
                                                 uint32_t* __restrict__ out) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    const uint4* p = reinterpret_cast<const uint4*>(base + off[c]);
    uint32_t a = 0, b = 0;
    for (uint32_t s = 0; s < L / 128u; ++s) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = p[8 * s + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) fold(a, b, v[j]);
    }
    out[c] = a ^ b;
}

// 8 lanes per chunk: instruction i of a stage reads chunks 8i .. 8i+7 of the wave
__global__ __launch_bounds__(256) void read_coop8(const uint8_t* __restrict__ base,
                                                  const uint64_t* __restrict__ off, uint32_t L,
                                                  uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w0 = (blockIdx.x * 256u + threadIdx.x) & ~63u;  // first chunk of this wave
    const uint4* p[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = reinterpret_cast<const uint4*>(base + off[w0 + 8 * i + lane / 8]) + (lane & 7u);
    uint32_t a = 0, b = 0;
    for (uint32_t s = 0; s < L / 128u; ++s) {
        uint4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = p[i][8 * s];
#pragma unroll
        for (int i = 0; i < 8; ++i) fold(a, b, v[i]);
    }
    out[w0 + lane] = a ^ b;
}

// 64 lanes per chunk: instruction i of a super-stage reads 1 KiB of chunk i of the wave
__global__ __launch_bounds__(256) void read_coop64(const uint8_t* __restrict__ base,
                                                   const uint64_t* __restrict__ off, uint32_t L,
                                                   uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w0 = (blockIdx.x * 256u + threadIdx.x) & ~63u;
    uint32_t a = 0, b = 0;
    for (uint32_t s = 0; s < L / 1024u; ++s) {
        for (uint32_t i0 = 0; i0 < 64; i0 += 8) {
            uint4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
                v[i] = reinterpret_cast<const uint4*>(base + off[w0 + i0 + i] + 1024ull * s)[lane];
#pragma unroll
            for (int i = 0; i < 8; ++i) fold(a, b, v[i]);
        }
    }
    out[w0 + lane] = a ^ b;
}

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536u;
    const uint32_t L = argc > 2 ? (uint32_t)atoi(argv[2]) : 524288u;
    if (N % 256u || L % 1024u) {
        fprintf(stderr, "chunks must be a multiple of 256, chunk bytes of 1024\n");
        return 1;
    }
    uint8_t* base;
    uint64_t* d_off;
    uint32_t* out;
    CHECK(hipMalloc(&base, (size_t)N * L));
    CHECK(hipMalloc(&d_off, N * sizeof(uint64_t)));
    CHECK(hipMalloc(&out, N * sizeof(uint32_t)));
    CHECK(hipMemset(base, 0x5a, (size_t)N * L));
    std::vector<uint64_t> off(N);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int layout = 0; layout < 3; ++layout) {
        std::vector<uint32_t> perm(N);
        for (uint32_t i = 0; i < N; ++i) perm[i] = i;
        if (layout == 1) std::shuffle(perm.begin(), perm.end(), std::mt19937(1));
        if (layout == 2) {  // runs of 4 adjacent chunks, the runs permuted
            std::vector<uint32_t> runs(N / 4);
            for (uint32_t r = 0; r < N / 4; ++r) runs[r] = r;
            std::shuffle(runs.begin(), runs.end(), std::mt19937(1));
            for (uint32_t i = 0; i < N; ++i) perm[i] = runs[i / 4] * 4 + i % 4;
        }
        for (uint32_t i = 0; i < N; ++i) off[i] = (uint64_t)perm[i] * L;
        CHECK(hipMemcpy(d_off, off.data(), N * sizeof(uint64_t), hipMemcpyHostToDevice));
        for (int pat = 0; pat < 3; ++pat) {
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                CHECK(hipEventRecord(e0));
                if (pat == 0) hipLaunchKernelGGL(read_lane, dim3(N / 256), dim3(256), 0, 0, base, d_off, L, out);
                if (pat == 1) hipLaunchKernelGGL(read_coop8, dim3(N / 256), dim3(256), 0, 0, base, d_off, L, out);
                if (pat == 2) hipLaunchKernelGGL(read_coop64, dim3(N / 256), dim3(256), 0, 0, base, d_off, L, out);
                CHECK(hipGetLastError());
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) best = std::min(best, ms);
            }
            static const char* names[] = {"lane", "coop8", "coop64"};
            printf("{\"layout\": \"%s\", \"pattern\": \"%s\", \"chunks\": %u, \"chunk_bytes\": %u, \"ms\": %.3f, "
                   "\"GBps\": %.1f}\n",
                   layout == 1 ? "scattered" : layout == 2 ? "runs_of_4" : "in_place", names[pat], N, L, best, (double)N * L / (best * 1e-3) / 1e9);
            fflush(stdout);
        }
    }
    CHECK(hipFree(base));
    CHECK(hipFree(d_off));
    CHECK(hipFree(out));
    return 0;
}
