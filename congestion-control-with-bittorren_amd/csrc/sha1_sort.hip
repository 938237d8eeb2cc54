// sha1_sort.hip -- longest-first ordering of a ragged device batch.
//
// A wave runs as long as its longest lane (SHA-1 is serial per chunk), so a
// mixed-length batch (BASELINE config 5: received chunks of 4 KiB .. 1 MiB)
// is hashed in descending order of its chunks' SHA-1 block counts (the
// length of each serial chain): the 64 lanes of a wave get equal chains and
// the hardware dispatcher starts the heaviest groups first.  Stable: chunks
// of equal block counts keep caller order, so the order is a function of
// the lengths alone.
//
// Keys are 16-bit block counts, ceil((len + 9) / 64) clamped at 65535
// (chunks of 4 MiB and more tie at the top in caller order; the planner then
// prices such a group by its first chunk, the hashing is unaffected).
//
// Up to kSortMaxTiles tiles of 4096 chunks (1 Mi chunks) an LSD radix sort
// of two 8-bit digits in three launches of its own:
//   sort_keys_hist   keys, and each tile's low-digit histogram
//   sort_scatter<1>  stable scatter by the low digit; the high-digit
//                    histograms of the tiles it writes into (atomics)
//   sort_scatter<2>  stable scatter by the high digit: the order, and the
//                    sorted lengths the planner reads
// A tile's start for digit d is the count of d in the tiles before it plus
// every larger digit's total, each workgroup summing the histogram columns
// itself (T loads per thread), so no scan launch.  Inside a tile, rank =
// (earlier (item, wave) slices' count of d) + (lanes of the wave below this
// one with the same digit, from 8 ballots).  rocPRIM's radix sort took
// ~51 us at 131072 chunks (a block sort and seven merge passes on 32-bit
// lengths; onesweep on these 16-bit keys 58 us, profiles/sort_probe_r05.log).
// Beyond 1 Mi chunks the columns grow with T, and rocPRIM's onesweep sorts
// the same keys (same order: both stable).
// Temporaries come from the stream-ordered allocator so concurrent calls on
// different streams do not share scratch.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <stdint.h>

#include "sha1_kernels.h"

namespace {
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

constexpr uint32_t kSortThreads = 256, kSortItems = 16, kSortWaves = kSortThreads / 64;
constexpr uint32_t kSortTile = kSortThreads * kSortItems;  // 4096 chunks
constexpr uint32_t kSortMaxTiles = 256;

__device__ __forceinline__ uint16_t block_key(uint32_t len) {
    const uint32_t b = (uint32_t)(((uint64_t)len + 9u + 63u) / 64u);
    return (uint16_t)(b > 65535u ? 65535u : b);
}

// Descending order as ascending "slots": slot 0 is the largest digit.
template <int PASS>
__device__ __forceinline__ uint32_t key_slot(uint32_t k) {
    return 255u - (PASS == 1 ? (k & 255u) : (k >> 8));
}
}  // namespace

// Tile t: keys[i] for its chunks, hist1[t][slot] of their low digits, and
// hist2[t][*] zeroed for sort_scatter<1>'s atomics.
__global__ __launch_bounds__(kSortThreads) void sort_keys_hist(const uint32_t* len, uint16_t* keys, uint32_t* hist1,
                                                               uint32_t* hist2, uint32_t n) {
    __shared__ uint32_t h[256];
    const uint32_t tid = threadIdx.x;
    h[tid] = 0u;
    __syncthreads();
    const uint32_t base = blockIdx.x * kSortTile;
#pragma unroll
    for (uint32_t it = 0; it < kSortItems; ++it) {
        const uint32_t i = base + it * kSortThreads + tid;
        if (i < n) {
            const uint16_t k = block_key(len[i]);
            keys[i] = k;
            atomicAdd(&h[key_slot<1>(k)], 1u);
        }
    }
    __syncthreads();
    hist1[blockIdx.x * 256u + tid] = h[tid];
    hist2[blockIdx.x * 256u + tid] = 0u;
}

// One stable counting-sort pass over 8-bit digit PASS of tile blockIdx.x's
// keys (keys_in / ids_in in the previous pass's order; ids_in null = the
// chunk index).  PASS 1 writes keys_out / ids_out and counts the high digit
// of what lands in each output tile into hist_next; PASS 2 writes the final
// order and sorted lengths.
template <int PASS>
__global__ __launch_bounds__(kSortThreads) void sort_scatter(const uint16_t* keys_in, const uint32_t* ids_in,
                                                             const uint32_t* hist, uint32_t tiles, uint32_t n,
                                                             uint16_t* keys_out, uint32_t* ids_out,
                                                             uint32_t* hist_next, const uint32_t* len,
                                                             uint32_t* sorted_len) {
    __shared__ uint32_t start[256];                         // the tile's first position per slot
    __shared__ uint32_t scan[256];
    __shared__ uint16_t cnt[kSortItems * kSortWaves][256];  // per (item, wave) slice, then its prefix
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    const uint32_t tile = blockIdx.x;

    // this slot's count over all tiles and over the tiles before this one
    uint32_t tot = 0, pre = 0;
    {
        uint32_t t = 0;
        for (; t + 8u <= tiles; t += 8u) {
            uint32_t v[8];
#pragma unroll
            for (uint32_t u = 0; u < 8u; ++u) v[u] = hist[(t + u) * 256u + tid];
#pragma unroll
            for (uint32_t u = 0; u < 8u; ++u) {
                tot += v[u];
                pre += t + u < tile ? v[u] : 0u;
            }
        }
        for (; t < tiles; ++t) {
            const uint32_t v = hist[t * 256u + tid];
            tot += v;
            pre += t < tile ? v : 0u;
        }
    }
    // exclusive scan of the slot totals (inclusive Hillis-Steele, minus own)
    scan[tid] = tot;
    __syncthreads();
    for (uint32_t off = 1; off < 256u; off <<= 1) {
        const uint32_t v = tid >= off ? scan[tid - off] : 0u;
        __syncthreads();
        scan[tid] += v;
        __syncthreads();
    }
    start[tid] = scan[tid] - tot + pre;
    {
        uint32_t* c32 = reinterpret_cast<uint32_t*>(&cnt[0][0]);
        for (uint32_t w = tid; w < kSortItems * kSortWaves * 128u; w += kSortThreads) c32[w] = 0u;
    }
    __syncthreads();

    // rank inside the wave: valid lanes below this one with the same slot
    const uint32_t base = tile * kSortTile;
    uint32_t key_rank[kSortItems];  // key | rank in wave << 16
    uint32_t id[kSortItems];
#pragma unroll
    for (uint32_t it = 0; it < kSortItems; ++it) {
        const uint32_t i = base + it * kSortThreads + tid;
        const bool valid = i < n;
        const uint32_t k = valid ? keys_in[i] : 0u;
        id[it] = valid ? (ids_in ? ids_in[i] : i) : 0u;
        const uint32_t s = key_slot<PASS>(k);
        uint64_t m = __ballot(valid);
#pragma unroll
        for (uint32_t b = 0; b < 8u; ++b) {
            const uint64_t bal = __ballot((s >> b) & 1u);
            m &= ((s >> b) & 1u) ? bal : ~bal;
        }
        const uint32_t below =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (valid && below == 0u) cnt[it * kSortWaves + wave][s] = (uint16_t)__popcll(m);
        key_rank[it] = k | (below << 16);
    }
    __syncthreads();
    // per slot: the slices' exclusive prefix inside the tile, in (item, wave) order
    {
        uint32_t run = 0;
        for (uint32_t q = 0; q < kSortItems * kSortWaves; ++q) {
            const uint32_t c = cnt[q][tid];
            cnt[q][tid] = (uint16_t)run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t it = 0; it < kSortItems; ++it) {
        const uint32_t i = base + it * kSortThreads + tid;
        if (i < n) {
            const uint32_t k = key_rank[it] & 0xffffu;
            const uint32_t s = key_slot<PASS>(k);
            const uint32_t dst = start[s] + cnt[it * kSortWaves + wave][s] + (key_rank[it] >> 16);
            if constexpr (PASS == 1) {
                keys_out[dst] = (uint16_t)k;
                ids_out[dst] = id[it];
                atomicAdd(&hist_next[(dst / kSortTile) * 256u + key_slot<2>(k)], 1u);
            } else {
                ids_out[dst] = id[it];
                sorted_len[dst] = len[id[it]];
            }
        }
    }
}

// Batches beyond kSortMaxTiles tiles: rocPRIM onesweep on the same keys.
__global__ void block_keys16(const uint32_t* len, uint16_t* key, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) key[i] = block_key(len[i]);
}

// sorted_len[i] = len[order[i]]: the planner's view of the sorted batch.
__global__ void gather_lengths(const uint32_t* len, const uint32_t* order, uint32_t* out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = len[order[i]];
}

hipError_t sort_by_length_desc(const uint32_t* d_len, uint32_t n, const uint32_t** d_order,
                               const uint32_t** d_sorted_len, uint32_t** d_plan, void** scratch,
                               hipStream_t st) {
    *d_order = nullptr;
    *d_sorted_len = nullptr;
    *d_plan = nullptr;
    *scratch = nullptr;
    const uint32_t tiles = (uint32_t)((uint64_t(n) + kSortTile - 1u) / kSortTile);
    const bool own = tiles <= kSortMaxTiles;
    const rocprim::counting_iterator<uint32_t> ids(0u);
    const size_t hb = align256(size_t(tiles) * 256u * sizeof(uint32_t));
    size_t temp_bytes = 0;
    hipError_t e = hipSuccess;
    if (own) {
        temp_bytes = 2 * hb + align256(size_t(n) * sizeof(uint32_t));
    } else {
        e = rocprim::radix_sort_pairs_desc(nullptr, temp_bytes, (const uint16_t*)nullptr, (uint16_t*)nullptr, ids,
                                           (uint32_t*)nullptr, n, 0, 16, st);
        if (e != hipSuccess) return e;
    }
    // [sorted lengths][order][plan][keys][keys'][temporaries]
    const size_t arr = align256(size_t(n) * sizeof(uint32_t));
    const size_t arr16 = align256(size_t(n) * sizeof(uint16_t));
    const size_t planb = mixed_plan_bytes(n);
    void* mem = nullptr;
    e = hipMallocAsync(&mem, 2 * arr + planb + 2 * arr16 + align256(temp_bytes), st);
    if (e != hipSuccess) return e;
    uint8_t* b = static_cast<uint8_t*>(mem);
    uint32_t* sorted_len = reinterpret_cast<uint32_t*>(b);
    uint32_t* order = reinterpret_cast<uint32_t*>(b + arr);
    uint32_t* plan = reinterpret_cast<uint32_t*>(b + 2 * arr);
    uint16_t* keys = reinterpret_cast<uint16_t*>(b + 2 * arr + planb);
    uint16_t* keys2 = reinterpret_cast<uint16_t*>(b + 2 * arr + planb + arr16);
    uint8_t* temp = b + 2 * arr + planb + 2 * arr16;
    if (own) {
        uint32_t* hist1 = reinterpret_cast<uint32_t*>(temp);
        uint32_t* hist2 = reinterpret_cast<uint32_t*>(temp + hb);
        uint32_t* ids2 = reinterpret_cast<uint32_t*>(temp + 2 * hb);
        hipLaunchKernelGGL(sort_keys_hist, dim3(tiles), dim3(kSortThreads), 0, st, d_len, keys, hist1, hist2, n);
        hipLaunchKernelGGL(sort_scatter<1>, dim3(tiles), dim3(kSortThreads), 0, st, keys, (const uint32_t*)nullptr,
                           hist1, tiles, n, keys2, ids2, hist2, (const uint32_t*)nullptr, (uint32_t*)nullptr);
        hipLaunchKernelGGL(sort_scatter<2>, dim3(tiles), dim3(kSortThreads), 0, st, keys2, ids2, hist2, tiles, n,
                           (uint16_t*)nullptr, order, (uint32_t*)nullptr, d_len, sorted_len);
        e = hipGetLastError();
    } else {
        const dim3 grid((n + 255u) / 256u);
        hipLaunchKernelGGL(block_keys16, grid, dim3(256), 0, st, d_len, keys, n);
        e = rocprim::radix_sort_pairs_desc(temp, temp_bytes, keys, keys2, ids, order, n, 0, 16, st);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(gather_lengths, grid, dim3(256), 0, st, d_len, order, sorted_len, n);
            e = hipGetLastError();
        }
    }
    if (e != hipSuccess) {
        (void)hipFreeAsync(mem, st);
        return e;
    }
    *d_order = order;
    *d_sorted_len = sorted_len;
    *d_plan = plan;
    *scratch = mem;
    return hipSuccess;
}
