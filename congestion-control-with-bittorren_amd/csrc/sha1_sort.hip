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
// Keys are 16-bit block counts, ceil((len + 9) / 64) clamped at 65535:
// chunks of 4 MiB and more tie at the top in caller order.  For the mixed
// path the sort also records them (per-tile counts, their lengths and ids,
// BigFix) and the layout kernel re-ranks up to kBigExact of them by exact
// block count before the planner prices the groups (round 6, no extra
// launch); beyond that they stay in caller order.  The hashing is
// unaffected either way.
//
// An LSD radix sort of two 8-bit digits in four launches of its own:
//   sort_hist<1>     keys, and each tile's low-digit histogram
//   sort_scatter<1>  stable scatter by the low digit
//   sort_hist<2>     each tile's high-digit histogram of that order (its
//                    own launch: global atomics from the scatter serialised,
//                    40 against 24 us at 131072 chunks in arrival order)
//   sort_scatter<2>  stable scatter by the high digit: the order, and the
//                    sorted lengths the planner reads (each group's first)
// A tile's start for digit d is the count of d in the tiles before it plus
// every larger digit's total, each workgroup summing the histogram columns
// itself (T / 4 loads per thread), so no scan launch.  Inside a tile, rank =
// (earlier (item, wave) slices' count of d) + (lanes of the wave below this
// one with the same digit, from 8 ballots).  rocPRIM's radix sort took
// ~51 us at 131072 chunks (a block sort and seven merge passes on 32-bit
// lengths; onesweep on these 16-bit keys 58 us, profiles/sort_probe_r05.log).
// Beyond kSortMaxTiles tiles (1 Mi chunks) the columns grow with T, so each
// histogram launch is followed by hist_scan (one workgroup per slot: every
// tile's start and the slot's total), and the scatters read those instead
// of summing columns: six launches, the same order (round 6; rounds 5 sent
// these batches to rocPRIM's onesweep).
// Temporaries come from the stream-ordered allocator so concurrent calls on
// different streams do not share scratch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sha1_kernels.h"

namespace {
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// A tile of 4096 chunks per workgroup of 16 waves, 4 chunks per lane
// (chunk base + item * 1024 + thread): 16 waves keep each lane's chains of
// dependent loads and LDS steps short (4 waves of 16 items each: 21-40 us
// per scatter at 131072 chunks, profiles/fixed_cost_r05.log).
constexpr uint32_t kSortThreads = 1024, kSortItems = 4, kSortWaves = kSortThreads / 64;
constexpr uint32_t kSortTile = kSortThreads * kSortItems;  // 4096 chunks
constexpr uint32_t kSortSlices = kSortItems * kSortWaves;  // (item, wave) slices of a tile, in chunk order
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

// The valid lanes of the wave whose slot equals this lane's (8 ballots).
__device__ __forceinline__ uint64_t slot_peers(bool valid, uint32_t s) {
    uint64_t m = __ballot(valid);
#pragma unroll
    for (uint32_t b = 0; b < 8u; ++b) {
        const uint64_t bal = __ballot((s >> b) & 1u);
        m &= ((s >> b) & 1u) ? bal : ~bal;
    }
    return m;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
}  // namespace

// Tile blockIdx.x's slot histogram of digit PASS: PASS 1 from the lengths
// (writing the keys), PASS 2 from the first scatter's keys.  One LDS atomic
// per run of equal slots in a wave (a tile of equal keys otherwise
// serialises 4096 atomics on one bin).
// PASS 1 also counts the tile's chunks whose key clamped (big_cnt, if set).
template <int PASS>
__global__ __launch_bounds__(kSortThreads) void sort_hist(const uint32_t* len, const uint16_t* keys_in,
                                                          uint16_t* keys_out, uint32_t* hist, uint32_t n,
                                                          uint32_t* big_cnt) {
    __shared__ uint32_t h[256];
    __shared__ uint32_t nbig;
    const uint32_t tid = threadIdx.x;
    if (tid < 256u) h[tid] = 0u;
    if (tid == 0u) nbig = 0u;
    __syncthreads();
    const uint32_t base = blockIdx.x * kSortTile;
#pragma unroll
    for (uint32_t it = 0; it < kSortItems; ++it) {
        const uint32_t i = base + it * kSortThreads + tid;
        const bool valid = i < n;
        uint32_t k = 0;
        if (valid) {
            if constexpr (PASS == 1) {
                k = block_key(len[i]);
                keys_out[i] = (uint16_t)k;
            } else {
                k = keys_in[i];
            }
        }
        const uint32_t s = key_slot<PASS>(k);
        const uint64_t m = slot_peers(valid, s);
        if (valid && lanes_below(m) == 0u) atomicAdd(&h[s], (uint32_t)__popcll(m));
        if constexpr (PASS == 1) {
            const uint64_t big = __ballot(valid && k == 0xffffu);
            if (big && (tid & 63u) == 0u) atomicAdd(&nbig, (uint32_t)__popcll(big));
        }
    }
    __syncthreads();
    if (tid < 256u) hist[blockIdx.x * 256u + tid] = h[tid];
    if (PASS == 1 && big_cnt && tid == 0u) big_cnt[blockIdx.x] = nbig;
}

// Batches of more than kSortMaxTiles tiles: slot blockIdx.x's count in the
// tiles before each tile (pre[tile * 256 + slot]) and in all of them
// (tot[slot]), an exclusive scan down the histogram column.
constexpr uint32_t kScanThreads = 256;
__global__ __launch_bounds__(kScanThreads) void hist_scan(const uint32_t* hist, uint32_t tiles, uint32_t* pre,
                                                          uint32_t* tot) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    const uint32_t s = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t per = (tiles + kScanThreads - 1u) / kScanThreads;
    const uint32_t t0 = min(tiles, tid * per), t1 = min(tiles, t0 + per);
    uint32_t sum = 0;
    for (uint32_t t = t0; t < t1; ++t) sum += hist[t * 256u + s];
    uint32_t inc = sum;
#pragma unroll
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint32_t v = __shfl_up(inc, d);
        if (lane >= d) inc += v;
    }
    if (lane == 63u) wsum[wave] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (uint32_t w = 0; w < wave; ++w) run += wsum[w];
    for (uint32_t t = t0; t < t1; ++t) {
        const uint32_t v = hist[t * 256u + s];
        pre[t * 256u + s] = run;
        run += v;
    }
    if (tid == kScanThreads - 1u) tot[s] = run;
}

// One stable counting-sort pass over digit PASS of tile blockIdx.x (keys_in
// / ids_in in the previous pass's order; ids_in null = the chunk index):
// PASS 1 writes keys_out / ids_out, PASS 2 the order and sorted lengths.
// pre_in / tot_in (batches of more than kSortMaxTiles tiles): the tile's
// per-slot starts and the slot totals from hist_scan; null: summed here.
template <int PASS>
__global__ __launch_bounds__(kSortThreads) void sort_scatter(const uint16_t* keys_in, const uint32_t* ids_in,
                                                             const uint32_t* hist, uint32_t tiles, uint32_t n,
                                                             uint16_t* keys_out, uint32_t* ids_out,
                                                             const uint32_t* len, uint32_t* sorted_len,
                                                             const uint32_t* pre_in, const uint32_t* tot_in,
                                                             uint32_t* big_len, uint32_t* big_id) {
    __shared__ uint32_t start[256];                   // the tile's first position per slot
    __shared__ uint32_t part_tot[4][256], part_pre[4][256], wsum[4];
    __shared__ uint16_t cnt[kSortSlices][256];        // per (item, wave) slice, then its prefix
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t tile = blockIdx.x;

    // slot s = tid % 256 over a quarter q = tid / 256 of the tiles: its
    // count in all of them and in those before this one
    {
        const uint32_t s = tid & 255u, q = tid >> 8, per = (tiles + 3u) / 4u;
        const uint32_t t0 = pre_in ? tiles : min(tiles, q * per), t1 = pre_in ? tiles : min(tiles, t0 + per);
        uint32_t tot = 0, pre = 0, t = t0;
        if (pre_in && q == 0u) {
            tot = tot_in[s];
            pre = pre_in[tile * 256u + s];
        }
        for (; t + 8u <= t1; t += 8u) {
            uint32_t v[8];
#pragma unroll
            for (uint32_t u = 0; u < 8u; ++u) v[u] = hist[(t + u) * 256u + s];
#pragma unroll
            for (uint32_t u = 0; u < 8u; ++u) {
                tot += v[u];
                pre += t + u < tile ? v[u] : 0u;
            }
        }
        for (; t < t1; ++t) {
            const uint32_t v = hist[t * 256u + s];
            tot += v;
            pre += t < tile ? v : 0u;
        }
        part_tot[q][s] = tot;
        part_pre[q][s] = pre;
        uint32_t* c32 = reinterpret_cast<uint32_t*>(&cnt[0][0]);
        for (uint32_t w = tid; w < kSortSlices * 128u; w += kSortThreads) c32[w] = 0u;
    }
    __syncthreads();
    // slots' exclusive scan of their totals (waves 0-3, a slot per lane)
    if (tid < 256u) {
        const uint32_t tot = part_tot[0][tid] + part_tot[1][tid] + part_tot[2][tid] + part_tot[3][tid];
        const uint32_t pre = part_pre[0][tid] + part_pre[1][tid] + part_pre[2][tid] + part_pre[3][tid];
        uint32_t inc = tot;
#pragma unroll
        for (uint32_t d = 1; d < 64u; d <<= 1) {
            const uint32_t v = __shfl_up(inc, d);
            if (lane >= d) inc += v;
        }
        if (lane == 63u) wsum[wave] = inc;
        part_tot[0][tid] = inc - tot + pre;  // exclusive within the wave, plus earlier tiles
    }
    __syncthreads();
    if (tid < 256u) {
        uint32_t off = 0;
        for (uint32_t w = 0; w < wave; ++w) off += wsum[w];
        start[tid] = part_tot[0][tid] + off;
    }

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
        const uint64_t m = slot_peers(valid, s);
        const uint32_t below = lanes_below(m);
        if (valid && below == 0u) cnt[it * kSortWaves + wave][s] = (uint16_t)__popcll(m);
        key_rank[it] = k | (below << 16);
    }
    __syncthreads();
    // per slot: the slices' exclusive prefix inside the tile, in (item, wave)
    // order; thread (q, s) takes slices 16q .. 16q+15
    {
        const uint32_t s = tid & 255u, q = tid >> 8;
        uint32_t c[16], sum = 0;
#pragma unroll
        for (uint32_t u = 0; u < 16u; ++u) {
            c[u] = cnt[16u * q + u][s];
            sum += c[u];
        }
        part_pre[q][s] = sum;
        __syncthreads();
        uint32_t run = 0;
        for (uint32_t w = 0; w < q; ++w) run += part_pre[w][s];
#pragma unroll
        for (uint32_t u = 0; u < 16u; ++u) {
            cnt[16u * q + u][s] = (uint16_t)run;
            run += c[u];
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
            } else {
                ids_out[dst] = id[it];
                // the planner reads a group's first length only (group_blocks):
                // one gather in 64, not every chunk's
                if ((dst & 63u) == 0u) sorted_len[dst] = len[id[it]];
                // a clamped key (>= 65535 blocks) lands in [0, m) in caller
                // order: its length and id for the exact re-ranking (BigFix)
                if (big_len && k == 0xffffu && dst < kBigExact) {
                    big_len[dst] = len[id[it]];
                    big_id[dst] = id[it];
                }
            }
        }
    }
}

// sorted_len[i] = len[order[i]]: the planner's view of the sorted batch.
__global__ void gather_lengths(const uint32_t* len, const uint32_t* order, uint32_t* out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = len[order[i]];
}

hipError_t sort_by_length_desc(const uint32_t* d_len, uint32_t n, const uint32_t** d_order,
                               const uint32_t** d_sorted_len, uint32_t** d_plan, void** scratch, BigFix* big,
                               hipStream_t st) {
    *d_order = nullptr;
    *d_sorted_len = nullptr;
    *d_plan = nullptr;
    *scratch = nullptr;
    const uint32_t tiles = (uint32_t)((uint64_t(n) + kSortTile - 1u) / kSortTile);
    const bool scan = tiles > kSortMaxTiles;  // starts from hist_scan, not summed per workgroup
    const size_t hb = align256(size_t(tiles) * 256u * sizeof(uint32_t));
    const size_t tb = align256(256u * sizeof(uint32_t));
    // temporaries: hist1, hist2, ids2 [, pre1, pre2, tot1, tot2] [, big_cnt, big_len, big_id]
    const size_t bigb = big ? align256(size_t(tiles) * sizeof(uint32_t)) + 2 * align256(kBigExact * sizeof(uint32_t))
                            : 0;
    const size_t temp_bytes =
        2 * hb + align256(size_t(n) * sizeof(uint32_t)) + (scan ? 2 * hb + 2 * tb : 0) + bigb;
    // [sorted lengths][order][plan][keys][keys'][temporaries]
    const size_t arr = align256(size_t(n) * sizeof(uint32_t));
    const size_t arr16 = align256(size_t(n) * sizeof(uint16_t));
    const size_t planb = mixed_plan_bytes(n);
    void* mem = nullptr;
    hipError_t e = hipMallocAsync(&mem, 2 * arr + planb + 2 * arr16 + temp_bytes, st);
    if (e != hipSuccess) return e;
    uint8_t* b = static_cast<uint8_t*>(mem);
    uint32_t* sorted_len = reinterpret_cast<uint32_t*>(b);
    uint32_t* order = reinterpret_cast<uint32_t*>(b + arr);
    uint32_t* plan = reinterpret_cast<uint32_t*>(b + 2 * arr);
    uint16_t* keys = reinterpret_cast<uint16_t*>(b + 2 * arr + planb);
    uint16_t* keys2 = reinterpret_cast<uint16_t*>(b + 2 * arr + planb + arr16);
    uint8_t* temp = b + 2 * arr + planb + 2 * arr16;
    uint32_t* hist1 = reinterpret_cast<uint32_t*>(temp);
    uint32_t* hist2 = reinterpret_cast<uint32_t*>(temp + hb);
    uint32_t* ids2 = reinterpret_cast<uint32_t*>(temp + 2 * hb);
    uint8_t* extra = temp + 2 * hb + align256(size_t(n) * sizeof(uint32_t));
    uint32_t* pre1 = scan ? reinterpret_cast<uint32_t*>(extra) : nullptr;
    uint32_t* pre2 = scan ? reinterpret_cast<uint32_t*>(extra + hb) : nullptr;
    uint32_t* tot1 = scan ? reinterpret_cast<uint32_t*>(extra + 2 * hb) : nullptr;
    uint32_t* tot2 = scan ? reinterpret_cast<uint32_t*>(extra + 2 * hb + tb) : nullptr;
    uint8_t* bigm = extra + (scan ? 2 * hb + 2 * tb : 0);
    uint32_t* big_cnt = big ? reinterpret_cast<uint32_t*>(bigm) : nullptr;
    uint32_t* big_len = big ? reinterpret_cast<uint32_t*>(bigm + align256(size_t(tiles) * sizeof(uint32_t))) : nullptr;
    uint32_t* big_id = big ? big_len + align256(kBigExact * sizeof(uint32_t)) / sizeof(uint32_t) : nullptr;
    hipLaunchKernelGGL(sort_hist<1>, dim3(tiles), dim3(kSortThreads), 0, st, d_len, (const uint16_t*)nullptr, keys,
                       hist1, n, big_cnt);
    if (scan) hipLaunchKernelGGL(hist_scan, dim3(256), dim3(kScanThreads), 0, st, hist1, tiles, pre1, tot1);
    hipLaunchKernelGGL(sort_scatter<1>, dim3(tiles), dim3(kSortThreads), 0, st, keys, (const uint32_t*)nullptr, hist1,
                       tiles, n, keys2, ids2, (const uint32_t*)nullptr, (uint32_t*)nullptr, pre1, tot1,
                       (uint32_t*)nullptr, (uint32_t*)nullptr);
    hipLaunchKernelGGL(sort_hist<2>, dim3(tiles), dim3(kSortThreads), 0, st, (const uint32_t*)nullptr, keys2,
                       (uint16_t*)nullptr, hist2, n, (uint32_t*)nullptr);
    if (scan) hipLaunchKernelGGL(hist_scan, dim3(256), dim3(kScanThreads), 0, st, hist2, tiles, pre2, tot2);
    hipLaunchKernelGGL(sort_scatter<2>, dim3(tiles), dim3(kSortThreads), 0, st, keys2, ids2, hist2, tiles, n,
                       (uint16_t*)nullptr, order, d_len, sorted_len, pre2, tot2, big_len, big_id);
    e = hipGetLastError();
    if (e != hipSuccess) {
        (void)hipFreeAsync(mem, st);
        return e;
    }
    *d_order = order;
    *d_sorted_len = sorted_len;
    *d_plan = plan;
    if (big) *big = BigFix{big_cnt, tiles, big_len, big_id, order, sorted_len};
    *scratch = mem;
    return hipSuccess;
}

hipError_t gather_sorted_lengths(const uint32_t* d_len, const uint32_t* d_order, uint32_t* d_out, uint32_t n,
                                 hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_lengths, dim3((n + 255u) / 256u), dim3(256), 0, st, d_len, d_order, d_out, n);
    return hipGetLastError();
}
