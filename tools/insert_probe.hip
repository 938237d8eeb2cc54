// insert_probe.hip -- shader cycles per job of the mixed planner's
// dispatch simulation (sha1_kernels.hip sim_xcd) for several forms of its
// sorted insert, one wave alone on the chip (8 lanes active, as in the
// planner's first pass, and all 64).  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 tools/insert_probe.hip -o tools/insert_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kCus = 32;

template <int V>
__device__ __forceinline__ void insert(float (&t)[kCus], uint32_t (&u)[kCus], float d) {
    if constexpr (V == 0) {  // product: med3 chain
        const float nx = t[0] + d;
#pragma unroll
        for (int i = 0; i + 1 < kCus; ++i) t[i] = __builtin_amdgcn_fmed3f(t[i], nx, t[i + 1]);
        t[kCus - 1] = fmaxf(t[kCus - 1], nx);
    } else if constexpr (V == 1) {  // u32 min then max, interleaved by the compiler
        const uint32_t nx = __float_as_uint(__uint_as_float(u[0]) + d);
#pragma unroll
        for (int i = 0; i + 1 < kCus; ++i) u[i] = max(u[i], min(nx, u[i + 1]));
        u[kCus - 1] = max(u[kCus - 1], nx);
    } else if constexpr (V == 2) {  // u32: every min first, then every max
        const uint32_t nx = __float_as_uint(__uint_as_float(u[0]) + d);
        uint32_t m[kCus];
#pragma unroll
        for (int i = 0; i + 1 < kCus; ++i) m[i] = min(nx, u[i + 1]);
        m[kCus - 1] = nx;
#pragma unroll
        for (int i = 0; i < kCus; ++i) u[i] = max(u[i], m[i]);
    } else if constexpr (V == 3) {  // u32 med3
        const uint32_t nx = __float_as_uint(__uint_as_float(u[0]) + d);
#pragma unroll
        for (int i = 0; i + 1 < kCus; ++i) {
            uint32_t r;
            asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(u[i]), "v"(nx), "v"(u[i + 1]));
            u[i] = r;
        }
        u[kCus - 1] = max(u[kCus - 1], nx);
    }
}

template <int V>
__global__ void probe(const float* dur, int jobs, int active, uint64_t* cyc, float* out) {
    const int lane = threadIdx.x;
    float t[kCus];
    uint32_t u[kCus];
#pragma unroll
    for (int i = 0; i < kCus; ++i) {
        t[i] = 0.0f;
        u[i] = 0u;
    }
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    if (lane < active) {
        float d = dur[lane];
        for (int j = 0; j < jobs; ++j) {
            const float dn = dur[(j + 1) & 1023];
            insert<V>(t, u, d);
            d = dn;
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    float s = 0;
#pragma unroll
    for (int i = 0; i < kCus; ++i) s += t[i] + __uint_as_float(u[i]);
    out[lane] = s;
    if (lane == 0) *cyc = c1 - c0;
}

int main() {
    float* dur;
    uint64_t* cyc;
    float* out;
    (void)hipMalloc(&dur, 1024 * 4);
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&out, 64 * 4);
    float h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = 100.0f - 0.05f * i;
    (void)hipMemcpy(dur, h, sizeof h, hipMemcpyHostToDevice);
    const char* names[] = {"f32_med3", "u32_min_max", "u32_mins_then_maxes", "u32_med3"};
    for (int active : {8, 64}) {
        for (int v = 0; v < 4; ++v) {
            for (int rep = 0; rep < 3; ++rep) {
                const int jobs = 2000;
                switch (v) {
                case 0: hipLaunchKernelGGL(probe<0>, 1, 64, 0, 0, dur, jobs, active, cyc, out); break;
                case 1: hipLaunchKernelGGL(probe<1>, 1, 64, 0, 0, dur, jobs, active, cyc, out); break;
                case 2: hipLaunchKernelGGL(probe<2>, 1, 64, 0, 0, dur, jobs, active, cyc, out); break;
                case 3: hipLaunchKernelGGL(probe<3>, 1, 64, 0, 0, dur, jobs, active, cyc, out); break;
                }
                uint64_t c = 0;
                (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
                if (rep == 2)
                    printf("{\"variant\": \"%s\", \"active_lanes\": %d, \"cycles_per_job\": %.1f}\n", names[v], active,
                           (double)c / jobs);
            }
        }
    }
    return 0;
}
