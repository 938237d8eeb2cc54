// sort_probe.hip -- what the mixed path's longest-first sort costs at the
// config-5 law's sizes: rocPRIM radix_sort_pairs_desc
// on the 32-bit lengths (the product), on lengths with only bits 6..31
// (block granularity), and on 16-bit block-count keys.  Not part of the
// product.  Build: hipcc --offload-arch=gfx950 -O3 tools/sort_probe.hip -o tools/sort_probe
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void to_blocks16(const uint32_t* len, uint16_t* key, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t b = (len[i] + 9u + 63u) / 64u;
        key[i] = (uint16_t)(b > 65535u ? 65535u : b);
    }
}

template <typename K>
float time_sort(const K* keys, K* kout, uint32_t* vout, uint32_t n, int bits0, int bits1, void* temp, size_t tb,
                hipStream_t st, const uint32_t* len32 = nullptr, uint16_t* k16 = nullptr) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const rocprim::counting_iterator<uint32_t> ids(0u);
    for (int w = 0; w < 3; ++w)
        (void)rocprim::radix_sort_pairs_desc(temp, tb, keys, kout, ids, vout, n, bits0, bits1, st);
    (void)hipEventRecord(a, st);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
        if (len32) hipLaunchKernelGGL(to_blocks16, dim3((n + 255) / 256), dim3(256), 0, st, len32, k16, n);
        (void)rocprim::radix_sort_pairs_desc(temp, tb, keys, kout, ids, vout, n, bits0, bits1, st);
    }
    (void)hipEventRecord(b, st);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / reps;
}

int main() {
    for (uint32_t n : {16384u, 65536u, 131072u, 262144u}) {
        std::vector<uint32_t> h(n);
        std::mt19937_64 g(1);
        for (auto& x : h) x = (4096u + (uint32_t)(g() % 4096)) << (g() % 8);
        uint32_t *len, *kout, *vout;
        uint16_t *k16, *k16o;
        CK(hipMalloc(&len, n * 4));
        CK(hipMalloc(&kout, n * 4));
        CK(hipMalloc(&vout, n * 4));
        CK(hipMalloc(&k16, n * 2));
        CK(hipMalloc(&k16o, n * 2));
        CK(hipMemcpy(len, h.data(), n * 4, hipMemcpyHostToDevice));
        hipStream_t st;
        CK(hipStreamCreate(&st));
        const rocprim::counting_iterator<uint32_t> ids(0u);
        size_t tb32 = 0, tb16 = 0;
        CK(rocprim::radix_sort_pairs_desc(nullptr, tb32, len, kout, ids, vout, n, 0, 32, st));
        CK(rocprim::radix_sort_pairs_desc(nullptr, tb16, k16, k16o, ids, vout, n, 0, 16, st));
        void* temp;
        CK(hipMalloc(&temp, std::max(tb32, tb16)));
        hipLaunchKernelGGL(to_blocks16, dim3((n + 255) / 256), dim3(256), 0, st, len, k16, n);
        const float t32 = time_sort(len, kout, vout, n, 0, 32, temp, tb32, st);
        const float t26 = time_sort(len, kout, vout, n, 6, 32, temp, tb32, st);
        const float t16 = time_sort(k16, k16o, vout, n, 0, 16, temp, tb16, st);
        const float t16k = time_sort(k16, k16o, vout, n, 0, 16, temp, tb16, st, len, k16);
        printf("{\"n\": %u, \"u32_bits0_32_us\": %.1f, \"u32_bits6_32_us\": %.1f, \"u16_blocks_us\": %.1f, "
               "\"u16_blocks_with_key_kernel_us\": %.1f}\n", n, t32, t26, t16, t16k);
        (void)hipFree(len); (void)hipFree(kout); (void)hipFree(vout); (void)hipFree(k16); (void)hipFree(k16o);
        (void)hipFree(temp);
        (void)hipStreamDestroy(st);
    }
    return 0;
}
