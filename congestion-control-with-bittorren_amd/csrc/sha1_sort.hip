// sha1_sort.hip -- longest-first ordering of a ragged device batch.
//
// A wave runs as long as its longest lane (SHA-1 is serial per chunk), so a
// mixed-length batch (BASELINE config 5: received chunks of 4 KiB .. 1 MiB)
// is hashed in descending-length order: the 64 lanes of a wave get similar
// lengths and the hardware dispatcher starts the heaviest groups first.
// rocPRIM's native device radix sort (stable, so equal lengths keep caller
// order), values straight from a counting iterator (no iota pass);
// temporaries from the stream-ordered allocator so concurrent calls on
// different streams do not share scratch.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <stdint.h>

#include "sha1_kernels.h"

namespace {
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }
}  // namespace

hipError_t sort_by_length_desc(const uint32_t* d_len, uint32_t n, const uint32_t** d_order,
                               const uint32_t** d_sorted_len, uint32_t** d_plan, void** scratch,
                               hipStream_t st) {
    *d_order = nullptr;
    *d_sorted_len = nullptr;
    *d_plan = nullptr;
    *scratch = nullptr;
    const rocprim::counting_iterator<uint32_t> ids(0u);
    size_t temp_bytes = 0;
    hipError_t e = rocprim::radix_sort_pairs_desc(nullptr, temp_bytes, d_len, (uint32_t*)nullptr, ids,
                                                  (uint32_t*)nullptr, n, 0, 32, st);
    if (e != hipSuccess) return e;
    const size_t arr = align256(size_t(n) * sizeof(uint32_t));
    void* base = nullptr;
    const size_t planb = mixed_plan_bytes(n);
    e = hipMallocAsync(&base, 2 * arr + planb + align256(temp_bytes), st);
    if (e != hipSuccess) return e;
    uint8_t* b = static_cast<uint8_t*>(base);
    uint32_t* keys_out = reinterpret_cast<uint32_t*>(b);
    uint32_t* vals_out = reinterpret_cast<uint32_t*>(b + arr);
    uint32_t* plan = reinterpret_cast<uint32_t*>(b + 2 * arr);
    void* temp = b + 2 * arr + planb;
    e = rocprim::radix_sort_pairs_desc(temp, temp_bytes, d_len, keys_out, ids, vals_out, n, 0, 32, st);
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
