// sha1_kernels.h -- kernel arguments and launchers (internal to libsha1chunk).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// One batch of independent messages.  Message e (0 <= e < n) is chunk
// id = order ? order[e] : e, bytes base[off[id] .. off[id] + len[id]),
// with off/len replaced by id*ulen / ulen when the arrays are null.
struct BatchArgs {
    const uint8_t* base;
    const uint64_t* off;
    const uint32_t* len;
    uint32_t ulen;
    uint32_t n;
    const uint32_t* order;
    uint8_t* dig;  // n x 20 digest bytes (finalising mode), 4-byte aligned
    // Streaming extras (null/0 for plain batches).  init_state/out_state:
    // every kernel; prefix_bytes (finalising a stream): lane kernel only.
    const uint32_t* init_state;  // 5 words per message instead of the IV
    uint64_t prefix_bytes;       // bytes already hashed before this call
    uint32_t* out_state;         // non-null: no padding, write raw state
    // Mixed-batch kernel only: its device-side plan {mode, H, F}
    // (plan_mixed_kernel, sha1_kernels.hip).
    const uint32_t* plan;
};

hipError_t launch_lane(const BatchArgs& A, hipStream_t st);
hipError_t launch_fused(const BatchArgs& A, hipStream_t st);
// Split-kernel shapes (sha1_kernels.hip launch_split): 1 (1-block units), 4
// (4-block units, two producers: <= 1 group per CU), 11 (8-wave workgroup of
// two pairs: <= 2 groups per CU).  The A/B library (`make ab`,
// -DSHA1CHUNK_AB_VARIANTS) also builds the study's other shapes and variant
// flags (2, 3, 8-10, 12, 13, 10*U+V, 500+V, 569, 577-585, 86, 87, 590).
bool split_unit_built(int unit_blocks);
hipError_t launch_split(const BatchArgs& A, int unit_blocks, hipStream_t st);
// The other shapes of the split-kernel study: weak stubs in the product
// (no such shape), defined by tools/ab_kernels.hip in the A/B library.
bool split_unit_study_built(int unit_blocks);
hipError_t launch_split_study(const BatchArgs& A, int unit_blocks, hipStream_t st);
// Sorted ragged batch of more groups than CUs (A.order set, sorted_len =
// the lengths in that order): a device-side plan splits the groups between
// the one-group split shape (longest first) and the fused kernel, or runs
// them all in the 8-wave split shape (sha1_kernels.hip, mixed).  `plan`:
// 3 device words; forced (or null): {mode, H, F} instead of the planner's.
uint32_t mixed_grid(uint32_t groups, int cus, uint32_t* hcap);
// Exact order of the chunks whose 16-bit sort keys clamp (>= 65535 SHA-1
// blocks: 4 MiB and more).  The sort leaves them at the front in caller
// order; the mixed path's layout kernel re-ranks up to kBigExact of them by
// their exact block counts (stable) before the planner and the hash kernel
// read the order (sha1_kernels.hip plan_layout_kernel).  More than that
// keep caller order among themselves (digests unaffected).
constexpr uint32_t kBigExact = 4096;
struct BigFix {
    const uint32_t* cnt;   // per sort tile: its chunks whose key clamped (sort_hist<1>)
    uint32_t tiles;
    const uint32_t* len;   // positions [0, min(m, kBigExact)) of the sort's output:
    const uint32_t* id;    //   their lengths and chunk ids (sort_scatter<2>)
    uint32_t* order;       // the sort's order and (group-head) sorted lengths,
    uint32_t* sorted_len;  //   rewritten for positions < m
};
// big (or null: no re-ranking): the sort's BigFix.
hipError_t launch_mixed(const BatchArgs& A, const uint32_t* sorted_len, const BigFix* big, uint32_t* plan, int cus,
                        const int* forced, hipStream_t st);
// The layout summary alone (its re-ranking included): the diagnostics of
// s1be_mixed_order_async.
hipError_t launch_plan_layout(const BatchArgs& A, const uint32_t* sorted_len, const BigFix* big, uint32_t* plan,
                              hipStream_t st);
// Persistent verify-queue drain (sha1_kernels.hip, vq drain; host side in
// sha1_runtime.hip, the persistent sha1chunk_vq).  The queue's rings live in
// coherent pinned host memory, which the kernel reads over PCIe (no copy
// engine, no launch per batch); results go back to host memory.
struct VqDrainArgs {
    const uint8_t* data;     // host: chunk bytes (ring)
    const uint64_t* off;     // host: per slot, byte offset into data
    const uint32_t* len;     // host: per slot, chunk length
    const uint8_t* exp;      // host: per slot, expected digest (20 B)
    const uint32_t* grp;     // host: per group ring entry {first slot, count}
    const uint32_t* pub;     // host: groups published so far
    const uint32_t* stop;    // host: nonzero = exit once nothing is claimable
    uint8_t* alive;          // host: per workgroup, 1 while it may still claim
    uint8_t* res;            // host: per slot, 0 match / 1 mismatch
    uint32_t* done;          // host: per group ring entry, group index + 1 when done
    uint32_t* last_done;     // host: the last group finished (index + 1), any order
    uint8_t* dig;            // device: per slot, digest scratch
    uint32_t* claim;         // device: groups claimed so far
    uint32_t grp_ring;       // group ring entries
    uint32_t pad;
    uint64_t idle_ticks;     // 100 MHz ticks without work before a workgroup exits
    uint64_t life_ticks;     // 100 MHz ticks after which a workgroup exits even under load
};
hipError_t launch_vq_drain(const VqDrainArgs& Q, uint32_t grid, hipStream_t st);

hipError_t launch_synth(uint8_t* dst, const uint64_t* off, const uint32_t* lens, uint32_t ulen,
                        uint64_t first, uint64_t count, uint64_t seed, hipStream_t st);
hipError_t launch_compare(const uint8_t* dig, const uint8_t* exp, uint32_t n, uint8_t* mismatch,
                          hipStream_t st);

// Longest-first order of a ragged batch (sha1_sort.hip): *d_order receives n
// indices in descending order of SHA-1 block count (stable), *d_sorted_len
// the lengths in that order at each group's first position (64g; the
// planner reads no other) and *d_plan the mixed kernel's plan area of the
// same allocation
// (mixed_plan_bytes(n): 256 bytes of plan words, then the planner's layout
// summary); release *scratch with hipFreeAsync on the same stream after the
// consuming kernel has been enqueued.
inline size_t mixed_plan_bytes(uint32_t n) {
    const size_t words = ((size_t(n) + 63) / 64 + 31) / 32;  // one per 32 groups of 64 chunks
    return 256 + ((words * 12 + words * 32 * 4 + 255) & ~size_t(255));  // + a block count per group
}
// big (or null): receives the clamped chunks' re-ranking inputs (BigFix).
hipError_t sort_by_length_desc(const uint32_t* d_len, uint32_t n, const uint32_t** d_order,
                               const uint32_t** d_sorted_len, uint32_t** d_plan, void** scratch, BigFix* big,
                               hipStream_t st);
// out[i] = len[order[i]] for every i (diagnostics: s1be_sort_order_async).
hipError_t gather_sorted_lengths(const uint32_t* d_len, const uint32_t* d_order, uint32_t* d_out, uint32_t n,
                                 hipStream_t st);
