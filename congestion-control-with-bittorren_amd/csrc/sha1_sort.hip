// sha1_sort.hip -- longest-first ordering of a ragged device batch.
//
// A wave runs as long as its longest lane (SHA-1 is serial per chunk), so a
// mixed-length batch (BASELINE config 5: received chunks of 4 KiB .. 1 MiB)
// is hashed in descending-length order: the 64 lanes of a wave get similar
// lengths and the hardware dispatcher starts the heaviest groups first.
// rocPRIM radix sort (via hipCUB) on the device, temporaries from the
// stream-ordered allocator so concurrent calls on different streams do not
// share scratch.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "sha1_kernels.h"

namespace {

__global__ void iota_kernel(uint32_t* v, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

hipError_t sort_by_length_desc(const uint32_t* d_len, uint32_t n, const uint32_t** d_order,
                               const uint32_t** d_sorted_len, uint32_t** d_plan, void** scratch,
                               hipStream_t st) {
    *d_order = nullptr;
    *d_sorted_len = nullptr;
    *d_plan = nullptr;
    *scratch = nullptr;
    size_t temp_bytes = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(
        nullptr, temp_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
        (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0, 32, st);
    if (e != hipSuccess) return e;
    const size_t arr = align256(size_t(n) * sizeof(uint32_t));
    void* base = nullptr;
    e = hipMallocAsync(&base, 3 * arr + 256 + align256(temp_bytes), st);
    if (e != hipSuccess) return e;
    uint8_t* b = static_cast<uint8_t*>(base);
    uint32_t* keys_out = reinterpret_cast<uint32_t*>(b);
    uint32_t* vals_in = reinterpret_cast<uint32_t*>(b + arr);
    uint32_t* vals_out = reinterpret_cast<uint32_t*>(b + 2 * arr);
    uint32_t* plan = reinterpret_cast<uint32_t*>(b + 3 * arr);
    void* temp = b + 3 * arr + 256;
    hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, st, vals_in, n);
    if ((e = hipGetLastError()) != hipSuccess) {
        (void)hipFreeAsync(base, st);
        return e;
    }
    e = hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, d_len, keys_out, vals_in,
                                                     vals_out, n, 0, 32, st);
    if (e != hipSuccess) {
        (void)hipFreeAsync(base, st);
        return e;
    }
    *d_order = vals_out;
    *d_sorted_len = keys_out;
    *d_plan = plan;
    *scratch = base;
    return hipSuccess;
}
