// sha1_split.hpp -- the device-side building blocks of the gfx950 SHA-1
// kernels: per-lane entries and loads, the split kernel (consumer +
// producer waves over an LDS W+K ring) as a template over its shape, the
// fused and shared-load (coop) bodies.  Included by sha1_kernels.hip (the
// product's kernels and launchers) and by tools/ab_kernels.hip (the other
// split shapes of the round-1..3 study, built only into the A/B library).
// Everything here is a template or internal to the including file.
#ifndef SHA1_SPLIT_HPP
#define SHA1_SPLIT_HPP

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sha1_device.hpp"
#include "sha1_kernels.h"

using namespace s1;

namespace {

struct Entry {
    uint32_t id;
    const uint8_t* p;
    uint32_t len;
};

#ifdef SHA1CHUNK_CHECKED
// The bounds-checked backend (`make checked`): every
// entry index and every A.order value is checked against the batch; a
// violation is counted here (read by s1be_checked_violations, sha1_kernels.hip),
// the first few printed, and the index clamped so the access stays inside
// the batch -- the run reports the bug instead of faulting the GPU.
__device__ unsigned int g_checked_oob;

__device__ __forceinline__ uint32_t checked_index(uint32_t i, uint32_t n, const char* what) {
    if (i < n) return i;
    if (atomicAdd(&g_checked_oob, 1u) < 8u)
        printf("sha1chunk checked: %s %u >= n %u (block %u, thread %u)\n", what, i, n, blockIdx.x, threadIdx.x);
    return n ? n - 1u : 0u;
}
#endif

__device__ __forceinline__ Entry fetch_entry(const BatchArgs& A, uint32_t e) {
    Entry r;
#ifdef SHA1CHUNK_CHECKED
    e = checked_index(e, A.n, "entry index");
    r.id = A.order ? checked_index(A.order[e], A.n, "A.order value") : e;
#else
    r.id = A.order ? A.order[e] : e;
#endif
    const uint64_t off = A.off ? A.off[r.id] : (uint64_t)r.id * A.ulen;
    r.p = A.base + off;
    r.len = A.len ? A.len[r.id] : A.ulen;
    return r;
}

// The entry a lane past the batch reads instead of its own (its loads are
// valid and unused): the group's first chunk, or -- for a group wholly past
// the batch (the empty second pair of a split workgroup when the group count
// is odd) -- the batch's last entry, never group*64, which indexes past
// A.order (round 5's fault, gpurun_out/pytest_sort16_r05.log; fixed in
// 2705501).  SHA1CHUNK_AB_UNCLAMPED puts the unclamped index back: only for
// the checked build's negative test (`make checked-unclamped`).
__device__ __forceinline__ uint32_t fallback_entry(const BatchArgs& A, uint32_t group) {
#ifdef SHA1CHUNK_AB_UNCLAMPED
    return group * 64u;
#else
    return min(group * 64u, A.n - 1u);
#endif
}

__device__ __forceinline__ void load_init(const BatchArgs& A, uint32_t id, uint32_t (&h)[5]) {
    if (A.init_state) {
#pragma unroll
        for (int i = 0; i < 5; ++i) h[i] = A.init_state[5 * id + i];
    } else {
        init_state(h);
    }
}

__device__ __forceinline__ void emit(const BatchArgs& A, uint32_t id, const uint32_t (&h)[5]) {
    if (A.out_state) {
#pragma unroll
        for (int i = 0; i < 5; ++i) A.out_state[5 * id + i] = h[i];
    } else {
        store_digest(A.dig + 20ull * id, h);
    }
}

// Blocks [k0, nfull) of one lane straight from global memory (one block
// prefetched), then the padded tail (unless the batch is in update mode).
__device__ __forceinline__ void lane_loop(const Entry& en, uint32_t k0, uint32_t (&h)[5]) {
    const uint32_t nfull = en.len >> 6;
    uint32_t cur[16];
    if (k0 < nfull) load_block16(en.p + 64ull * k0, cur);
    for (uint32_t k = k0; k < nfull; ++k) {
        // swap into the schedule window first (other registers), then
        // refill `cur` with the next block in flight during the compression
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap_fresh(cur[j]);
        if (k + 1 < nfull) load_block16(en.p + 64ull * (k + 1), cur);
        compress(h, w);
    }
}

__device__ __forceinline__ bool wave_all(bool x) { return __ballot(!x) == 0; }
__device__ __forceinline__ bool wave_any(bool x) { return __ballot(x) != 0; }

__device__ __forceinline__ void lane_blocks(const BatchArgs& A, const Entry& en, uint32_t k0,
                                            uint32_t (&h)[5]) {
    lane_loop(en, k0, h);
    const uint32_t nfull = en.len >> 6;
    if (!A.out_state)
        finish_message(h, en.p + 64ull * nfull, en.len & 63u, A.prefix_bytes + en.len);
}

__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x = min(x, (uint32_t)__shfl_xor(x, m));
    return x;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x = max(x, (uint32_t)__shfl_xor(x, m));
    return x;
}

// Bulk stages every lane has: the wave's fewest whole 128-byte stages.
__device__ __forceinline__ uint32_t bulk_stages(const Entry& en, bool valid) {
    return wave_any(valid) ? __builtin_amdgcn_readfirstlane(wave_min(valid ? (en.len >> 7) : 0xffffffffu)) : 0u;
}

}  // namespace

// --------------------------------------------------------------- split ----
// Workgroup = consumer wave (wave 0) + producer wave (wave 1) on the same 64
// chunks.  The producer streams the wave's blocks from HBM (two blocks or
// stages in flight in registers; in the product shapes with loads shared
// across the wave, kVCoop), byte-swaps them and
// expands the 80-word schedule into an LDS ring; the consumer runs only the
// 80 rounds, so each chunk's serial instruction stream (the bound when
// there are too few chunks to fill the SIMDs) drops from ~630 to ~440
// instructions per block.
//
// The ring has 2 slots of U blocks (U*20 KiB each).  W slot layout: group q
// (q = 0..19) of four schedule words of block j of lane r at
// j*20K + q*1K + r*16, so every ds_write_b128 / ds_read_b128 touches one
// contiguous KiB (conflict-free).  Protocol, one s_barrier per unit of U
// blocks (each wave executes ceil(Tmax/U)+1 of them):
//   producer: write unit m (blocks mU..mU+U-1) into slot m&1 -> B_m
//   consumer: B_0, read W(0); per block k: [if k+1 starts unit m+1: B_{m+1}]
//             stream W(k+1) into the spare register set, rounds of block k.
//   RAW: unit m+1 is complete before B_{m+1}; its reads come after it.
//   WAR: the producer rewrites slot m&1 (unit m+2) only after B_{m+1}; every
//        read of unit m was issued before B_{m+1} and drained by its lgkmcnt(0).
// Fewer barriers per block (U > 1) is worth ~10% at low occupancy (U = 4,
// the whole 160 KiB LDS, is ~1.5% ahead of U = 3); U = 1 keeps LDS at 40 KiB
// for higher occupancy.
constexpr int kWBlockBytes = 20 * 1024;

// The lgkmcnt(0) goes through the builtin so hipcc knows every LDS access
// before the barrier has completed (it then stops waiting for them later);
// the barrier itself is asm with a memory clobber so no LDS access moves
// across it.
__device__ __forceinline__ void split_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only (gfx9 encoding)
    asm volatile("s_barrier" ::: "memory");
}

// Study probe (A/B library only, kVProbe): the same barrier, with the
// shader-clock cycles the wave spends in it added to `acc`.
__device__ __forceinline__ void split_barrier_timed(uint64_t& acc) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_barrier" ::: "memory");
    acc += __builtin_amdgcn_s_memtime() - t0;
}

// Producer: the 80-word schedule of one block, plus K, into its W block slot.
template <int T, bool WK>
struct SchedWrite {
    __device__ __forceinline__ static void run(uint32_t (&w)[16], uint8_t* slot, int lane) {
        if constexpr (T < 80) {
            if constexpr (T >= 16) sched_step<T>(w);
            if constexpr ((T & 3) == 3) {
                // ship W + K (K is constant over each group of 4: the round
                // ranges 0/20/40/60 are multiples of 4)
                constexpr int j = (T - 3) & 15;
                constexpr uint32_t k = WK ? round_k<T>() : 0u;
                *reinterpret_cast<uint4*>(slot + (T >> 2) * 1024 + lane * 16) =
                    make_uint4(w[j] + k, w[j + 1] + k, w[j + 2] + k, w[j + 3] + k);
            }
            SchedWrite<T + 1, WK>::run(w, slot, lane);
        }
    }
};

__device__ __forceinline__ uint32_t total_blocks(uint32_t len) {
    // nfull data blocks + 1 padded block (+1 more when len % 64 >= 56)
    return (len >> 6) + (((len & 63u) < 56u) ? 1u : 2u);
}

// Message words of block k for the producer's tail region (any block of any
// lane: full, partial+pad, length-only), big-endian, padding applied.
__device__ __forceinline__ void tail_block_words(const Entry& en, uint32_t k, uint32_t (&w)[16]) {
    const uint32_t nfull = en.len >> 6, rem = en.len & 63u;
    const uint64_t bits = (uint64_t)en.len * 8ull;
    if (k < nfull) {
        load_block16(en.p + 64ull * k, w);
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
    } else if (k == nfull) {
        if (rem) {
            load_block_partial(en.p + 64ull * k, rem, w);
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) w[j] = 0u;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = pad_word(bswap(w[j]), j, (int)rem);
        if (rem < 56u) {
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 14; ++j) w[j] = 0u;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
    }
}

// NPROD producer waves share a unit's blocks.  NPROD = 2 (U = 4): each
// producer owns one stage (2 blocks) per unit and ends the unit with its
// barrier after that stage's odd block.  NPROD = U = 2: each producer owns
// one block per unit and ends the unit after it.  A single producer ends the
// unit after block U-1.
template <int U, bool WK, int NPROD = 1>
__device__ __forceinline__ void produce_block(uint32_t k, uint32_t (&w)[16], uint8_t* ring, int lane,
                                              uint64_t* bw = nullptr) {
    const uint32_t m = k / U, j = k - m * U;
    SchedWrite<0, WK>::run(w, ring + ((m & 1u) * U + j) * kWBlockBytes, lane);
    // U == NPROD: each producer writes one block of every unit
    if (NPROD == 1 ? j == U - 1 : (U == NPROD || (k & 1u) == 1u)) {
        if (bw)
            split_barrier_timed(*bw);
        else
            split_barrier();
    }
}


// Two blocks (128 contiguous bytes) of one lane's chunk, loaded per lane.
struct Stage {
    uint32_t w[32];
};
// V: uint4 when every lane's chunk is 16-byte aligned (hipcc then keeps
// the stage in 64-bit register pairs: 8 fewer moves per block in the fused
// loop), u32x4u at any alignment.
template <typename V = u32x4u>
__device__ __forceinline__ void load_stage(const uint8_t* p, Stage& st) {
    const V* q = reinterpret_cast<const V*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const V x = q[j];
        st.w[4 * j + 0] = x.x;
        st.w[4 * j + 1] = x.y;
        st.w[4 * j + 2] = x.z;
        st.w[4 * j + 3] = x.w;
    }
}

// ------------------------------------------------------- shared loads ----
// Bulk loads shared across the wave: instruction i
// (i = 0..7) of a 128-byte stage reads 128 bytes of each of the group's
// chunks 8i .. 8i+7 (lane l: chunk 8i + l/8, 16-byte piece l%8), so one load
// instruction touches 8 chunks instead of 64, and an LDS transpose hands
// each lane its own chunk's 128 bytes.  The loads take chunks at any byte
// alignment (u32x4u, sha1_device.hpp).  The lane-per-chunk pattern makes
// each load instruction translate 64 addresses; with chunks far apart that
// thrashes the CU's translation cache: scattered 512 KiB chunks read at
// 1183 GB/s lane-per-chunk and 5954 GB/s 8 chunks per instruction (5036 /
// 5980 in place; tools/coop_probe.hip).  In the hash kernels: 65536 x
// 512 KiB with permuted offsets in 11.1 ms (fused tail) and 24.3 (one-group
// split) against 28.7 and 29.3 lane-per-chunk; 32768 in the 8-wave split
// 6.62 ms against 14.8; and in place the split shapes get ~1 % faster
// (config 2: 6.019 vs 6.067 ms; profiles/mixed_r02.json "coop").
// Swizzle: piece p of chunk c at c*128 + ((p + c/2) & 7)*16, conflict-free
// for the b128 stores (8 contiguous lanes write one chunk) and for the b128
// reads (each of ds_read_b128's 16-lane groups sees 16 distinct 16-byte
// bank groups).
constexpr uint32_t kCoopStageBytes = 64u * 128u;
// A fused wave's LDS in the mixed kernel: five 4 KiB block buffers of the
// LDS-DMA loop below (eight fused waves fill the workgroup's 160 KiB).
constexpr uint32_t kCoopBlockBytes = 64u * 64u;
constexpr uint32_t kCoopBlockBufs = 5u;
constexpr uint32_t kCoopWaveBytes = kCoopBlockBufs * kCoopBlockBytes;

// Orders one wave's LDS accesses across a transpose: lane-to-lane exchange
// through LDS (coop_store -> coop_read, and the reads of a buffer before its
// next stores).  The hardware completes a wave's LDS ops in order; this pins
// the program order in the compiler too (a wavefront-scope fence and the
// wave barrier pseudo-op: neither emits an instruction).
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t coop_slot(uint32_t c, uint32_t piece) {
    return c * 128u + ((piece + (c >> 1)) & 7u) * 16u;
}

// (the in-flight stage lives in plain 32-bit words: an array of uint4
// stays in scratch memory)
__device__ __forceinline__ void coop_load(const u32x4u* const (&src)[8], uint32_t s, uint32_t (&v)[32]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u32x4u x = src[i][8u * s];
        v[4 * i + 0] = x.x;
        v[4 * i + 1] = x.y;
        v[4 * i + 2] = x.z;
        v[4 * i + 3] = x.w;
    }
}

__device__ __forceinline__ void coop_store(uint8_t* buf, const uint32_t (&v)[32], uint32_t lane) {
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i)
        *reinterpret_cast<uint4*>(buf + coop_slot(8u * i + lane / 8u, lane & 7u)) =
            make_uint4(v[4 * i + 0], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}

__device__ __forceinline__ void coop_read(const uint8_t* buf, uint32_t lane, uint32_t (&w)[32]) {
#pragma unroll
    for (uint32_t p = 0; p < 8; ++p) {
        const uint4 x = *reinterpret_cast<const uint4*>(buf + coop_slot(lane, p));
        w[4 * p + 0] = x.x;
        w[4 * p + 1] = x.y;
        w[4 * p + 2] = x.z;
        w[4 * p + 3] = x.w;
    }
}


// The same for one 64-byte block of the wave's 64 chunks (the split
// producers that own one block per unit): instruction i (i = 0..3) reads
// block k of chunks 16i .. 16i+15 (lane l: chunk 16i + l/4, 16-byte piece
// l%4), staged through 4 KiB of LDS.  Piece p of chunk c at
// c*64 + ((p + c/4) & 3)*16: conflict-free b128 stores and reads, and a
// lane's store address is the same for every i but for an i*1024 offset.
__device__ __forceinline__ void coop4_load(const u32x4u* const (&src)[4], uint32_t k, uint32_t (&v)[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const u32x4u x = src[i][4u * k];
        v[4 * i + 0] = x.x;
        v[4 * i + 1] = x.y;
        v[4 * i + 2] = x.z;
        v[4 * i + 3] = x.w;
    }
}

__device__ __forceinline__ void coop4_store(uint8_t* buf, const uint32_t (&v)[16], uint32_t lane) {
    const uint32_t at = (lane >> 2) * 64u + (((lane & 3u) + (lane >> 4)) & 3u) * 16u;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i)
        *reinterpret_cast<uint4*>(buf + i * 1024u + at) =
            make_uint4(v[4 * i + 0], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}

__device__ __forceinline__ void coop4_read(const uint8_t* buf, uint32_t lane, uint32_t (&w)[16]) {
#pragma unroll
    for (uint32_t p = 0; p < 4; ++p) {
        const uint4 x = *reinterpret_cast<const uint4*>(buf + lane * 64u + ((p + (lane >> 2)) & 3u) * 16u);
        w[4 * p + 0] = x.x;
        w[4 * p + 1] = x.y;
        w[4 * p + 2] = x.z;
        w[4 * p + 3] = x.w;
    }
}

// Per-lane source pointers of the shared-load pattern with `lanes` lanes per
// chunk: slot i is chunk group*64 + (64/lanes)*i + lane/lanes, piece
// lane%lanes; a slot past the batch reads the group's first chunk (valid,
// and at least as long as the wave's bulk region).  A group wholly past the
// batch (the second pair of a split workgroup when the group count is odd)
// takes the batch's last entry instead: never group*64, which indexes past
// A.order, and its blocks are never loaded (no bulk region).
template <int LANES>
__device__ __forceinline__ void coop_sources(const BatchArgs& A, uint32_t group, uint32_t lane,
                                             const u32x4u* (&src)[LANES]) {
#pragma unroll
    for (uint32_t i = 0; i < (uint32_t)LANES; ++i) {
        const uint32_t ej = group * 64u + (64u / LANES) * i + lane / LANES;
        src[i] = reinterpret_cast<const u32x4u*>(fetch_entry(A, ej < A.n ? ej : fallback_entry(A, group)).p) + (lane % LANES);
    }
}

// Producer side of one bulk stage: blocks 2s, 2s+1 from `cur`; once the
// second block's words are taken, `cur` is refilled with this producer's
// stage after next, s + 2 NPROD.
template <int U, bool WK, int NPROD = 1>
__device__ __forceinline__ void produce_stage(const Entry& en, uint32_t s, uint32_t S, Stage& cur,
                                              uint8_t* ring, int lane) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap(cur.w[16 * half + j]);
        if (half == 1 && s + 2 * NPROD < S) load_stage(en.p + 128ull * (s + 2 * NPROD), cur);
        produce_block<U, WK, NPROD>(2 * s + half, w, ring, lane);
    }
}

// Shared-load producers (kVCoop): the raw 128 bytes (stage) or 64 bytes
// (own block) of the wave's 64 chunks go through the first bytes of the W
// slot they are about to fill (free at that point, as for the W writes that
// follow; the wave's LDS accesses complete in order, so the transposing
// reads precede the W writes over them).
template <int U, bool WK, int NPROD = 1>
__device__ __forceinline__ void produce_stage_coop(const u32x4u* const (&src)[8], uint32_t s, uint32_t S,
                                                   uint32_t (&cur)[32], uint8_t* ring, uint32_t lane) {
    const uint32_t k0 = 2 * s, m = k0 / U, j = k0 - m * U;
    uint8_t* raw = ring + ((m & 1u) * U + j) * kWBlockBytes;
    coop_store(raw, cur, lane);
    if (s + 2 * NPROD < S) coop_load(src, s + 2 * NPROD, cur);
    uint32_t x[32];
    wave_lds_order();
    coop_read(raw, lane, x);
    wave_lds_order();  // the W writes below overwrite what was just read
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) w[q] = bswap(x[16 * half + q]);
        produce_block<U, WK, NPROD>(k0 + half, w, ring, (int)lane);
    }
}

template <int U, bool WK, int NPROD>
__device__ __forceinline__ void produce_own_block_coop(const u32x4u* const (&src)[4], uint32_t k, uint32_t K,
                                                       uint32_t (&cur)[16], uint8_t* ring, uint32_t lane,
                                                       uint64_t* bw = nullptr) {
    const uint32_t m = k / U, j = k - m * U;
    uint8_t* raw = ring + ((m & 1u) * U + j) * kWBlockBytes;
    coop4_store(raw, cur, lane);
    if (k + 2 * NPROD < K) coop4_load(src, k + 2 * NPROD, cur);
    uint32_t w[16];
    wave_lds_order();
    coop4_read(raw, lane, w);
    wave_lds_order();  // the W writes below overwrite what was just read
#pragma unroll
    for (int q = 0; q < 16; ++q) w[q] = bswap(w[q]);
    produce_block<U, WK, NPROD>(k, w, ring, (int)lane, bw);
}

// Producer that owns one block per unit (U == NPROD): block k from `cur`,
// which is then refilled with this producer's block after next, k + 2 NPROD.
template <int U, bool WK, int NPROD>
__device__ __forceinline__ void produce_own_block(const Entry& en, uint32_t k, uint32_t K,
                                                  uint32_t (&cur)[16], uint8_t* ring, int lane,
                                                  uint64_t* bw = nullptr) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap(cur[j]);
    if (k + 2 * NPROD < K) load_block16(en.p + 64ull * (k + 2 * NPROD), cur);
    produce_block<U, WK, NPROD>(k, w, ring, lane, bw);
}

template <int P>
__device__ __forceinline__ void read_w_group(const uint8_t* slot, uint32_t (&W)[80]) {
#pragma unroll
    for (int q = 5 * P; q < 5 * P + 5; ++q) {
        const uint4 x = *reinterpret_cast<const uint4*>(slot + q * 1024);
        W[4 * q + 0] = x.x;
        W[4 * q + 1] = x.y;
        W[4 * q + 2] = x.z;
        W[4 * q + 3] = x.w;
    }
}

// Consumer: rounds of block k from Wc while W(k+1) streams into Wn.  All of
// it is straight-line (the barrier position is a compile-time function of
// the unrolled block index), so hipcc inserts no waits inside the rounds.
// Split-kernel shape flags (defaults in kSplitV).  The study that chose them
// (rounds 1-3) also built variants that lost and were removed from the
// source in round 4 (their code is in git history before that round; results
// in profiles/): the slot address computed at run time, the consumer at
// s_setprio 3, all 20 schedule reads in one burst, the W+K ring in global
// memory instead of LDS, wave 1 left empty instead of wave 2, the 8-wave
// layout split over the LDS store-path halves, and variants in which the
// consumer skipped its LDS reads or one side idled at the barriers (wrong
// digests by design); round 4: one schedule read every 4 rounds instead of
// bursts (6.49 against 6.03 ms at 4096 chunks in the one-group shape, 6.60
// against 6.31 at 32768 in the 8-wave one: spread_read_ab_r04.json).  profiles/issue_r01.json, split_variants_r01.json,
// split_2prod_sweep_r01.json, split_prio_read_r02.json, global_w_ab_r02.json,
// halves_ab_r03.json, spread_read_ab_r04.json.  Shapes other than the product's 1 / 4 / 11 are built
// only into the A/B library (tools/ab_kernels.hip, `make ab`).
constexpr int kVWK = 1;      // producer ships W+K (consumer: one VOP2 add)
constexpr int kVUnmask = 4;  // unmasked commit while every lane is live
constexpr int kVRead10 = 8;  // schedule reads in two bursts of 10 instead of four of 5
// With two producers, launch 4 waves and leave wave 2 empty, so both
// producers (waves 1, 3) sit on the other LDS store-path half than the
// consumer (a workgroup's waves alternate halves, SIMDs {0,1} / {2,3}):
// measured 2-3% faster than 3 waves (profiles/split_2prod_sweep_r01.json).
constexpr int kVSkipWave2 = 64;
// Two pairs per workgroup with two producers each, 2-block units (one
// block per producer per unit), 8 waves: a workgroup's waves w and w + 4
// share a SIMD and waves 0-3 sit on four different SIMDs
// (tools/wave_placement_probe), so the consumers go on waves 0 and 2 with
// waves 4 and 6 left empty (each consumer alone on its SIMD), and each
// pair's producers share one of the other two SIMDs: waves 1 + 5 and 3 + 7.
// kVCross swaps which producer SIMD serves which consumer.
constexpr int kVLayout8 = 128;
constexpr int kVCross = 256;
// Producers load with shared loads (4 or 8 lanes per chunk, staged through
// the W slot): one load instruction touches 16 or 8 chunks instead of 64
// (see `shared loads`).
constexpr int kVCoop = 8192;
// Round-5 study flag: two 4-wave one-pair workgroups per CU (80 KiB of LDS
// each, 2-block units, two producers) with roles taken from the SIMD each
// wave landed on, so the two consumers sit on different SIMDs (0 and 2) and
// the producers share SIMDs 1 and 3, as in the 8-wave layout, but each pair
// has its own s_barrier.  Without the SIMD roles the dispatcher put both
// consumers on one SIMD on many CUs (10.67 ms at 32768 chunks,
// profiles/split_unit_ab_r03.json).  cu_turn(): a per-CU counter in device
// memory orders the workgroups that land on one CU (its parity picks SIMD 0
// or 2 for the consumer).
constexpr int kVSimdRole = 8192 * 2;
__device__ uint32_t g_cu_turn[4096];
__device__ __forceinline__ uint32_t cu_turn(uint32_t hw) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3u << 11) | (0u << 6) | 20u) & 15u;  // HW_REG_XCC_ID
    const uint32_t cu = (((xcc * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u + ((hw >> 8) & 15u)) & 4095u;
    return atomicAdd(&g_cu_turn[cu], 1u);
}
template <int PAIRS, int V, int NPROD>
constexpr int kSplitThreads = (V & kVLayout8) ? 512 : (V & kVSimdRole) ? 256 : 64 * PAIRS * (1 + NPROD) + ((V & kVSkipWave2) ? 64 : 0);
// Why W+K matters: the consumer's x = e + W + K as a VOP3 v_add3 (K in an
// SGPR or a VGPR alike) runs the one-wave round stream at ~4.98 cycles per
// instruction, the VOP2 v_add on a shipped W+K at the 4-cycle issue floor
// (tools/consumer_probe, profiles/issue_r01.json).  With ONE producer the
// extra 80 adds per block make the producer the slower wave (1878 vs 1757
// cycles per block), so single-producer kernels with 3- and 4-block units
// keep K in the consumer; the 4-block default has TWO producers (kSplitNProd)
// and ships W+K.  Measured on MI355X (profiles/split_variants_r01.json):
// 2-block units W+K ~5% ahead; unmasked commit helps every shape.
template <int U>
constexpr int kSplitV = U == 4 ? (kVWK | kVUnmask | kVSkipWave2 | kVRead10 | kVCoop)
                               : U == 3 ? kVUnmask : (kVWK | kVUnmask);
template <int U>
constexpr int kSplitNProd = U == 4 ? 2 : 1;

// Round-5 study flag (the 8-wave two-pair shape): the second pair's
// consumer issues its schedule-read bursts half a burst interval later than
// the first's.  Both pairs pass the workgroup's shared s_barrier together,
// so without it their read bursts (each 5 or 10 ds_read_b128 of 1 KiB) hit
// the CU's one LDS pipe at the same moments.
constexpr int kVPhase = 512;
// Round-5 study flag: the consumer times its barrier waits and its whole
// loop (shader clock) and writes them over its group's first digest rows
// instead of digests (wrong digests by design; A/B library only).
constexpr int kVProbe = 2048;
// Round-5 study flag: the pairs' read bursts both off the barrier, at
// rounds 10 / 50 (first pair) and 30 / 70 (second pair), with kVRead10.
constexpr int kVPhase2 = 4096;
template <int V>
__device__ __forceinline__ void split_barrier_or_timed(uint64_t& acc) {
    if constexpr ((V & kVProbe) != 0)
        split_barrier_timed(acc);
    else
        split_barrier();
}
// Round-5 study flag: all 20 schedule reads of the next block in one burst
// (before round 0, or before round 40 for the second pair under kVPhase).
constexpr int kVRead20 = 1024;

template <int U, int J, int V, bool MASK, int PH = 0>
__device__ __forceinline__ void consume_block(uint32_t k, uint32_t T, uint32_t (&h)[5],
                                              const uint32_t (&Wc)[80], uint32_t (&Wn)[80],
                                              const uint8_t* ring, int lane, uint64_t& bw) {
    // Block k+1 (k = k0 + J, k0 a multiple of 2U) is unit (k0/U + (J+1)/U),
    // whose parity is that of (J+1)/U since k0/U is even, and sub-block
    // (J+1) % U: the slot address is a compile-time offset.  A barrier goes
    // in front of the first read of every new unit.
    constexpr bool WK = (V & kVWK) != 0;
    constexpr int jn = (J + 1) % U;
    constexpr int slot_idx = (((J + 1) / U) & 1) * U + jn;
    const uint8_t* slot = ring + slot_idx * kWBlockBytes + lane * 16;
    uint32_t v[5] = {h[0], h[1], h[2], h[3], h[4]};
    if constexpr ((V & kVRead20) != 0) {
        constexpr int R = PH != 0 ? 40 : 0;
        if constexpr (jn == 0) split_barrier_or_timed<V>(bw);
        RoundsW<0, R, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<0>(slot, Wn);
        read_w_group<1>(slot, Wn);
        read_w_group<2>(slot, Wn);
        read_w_group<3>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<R, 80, WK>::run(v, Wc);
    } else if constexpr ((V & kVRead10) != 0) {
        // two bursts of 10 reads, before rounds 10 PH and 10 PH + 40
        constexpr int R = 10 * PH;
        if constexpr (jn == 0) split_barrier_or_timed<V>(bw);
        RoundsW<0, R, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<0>(slot, Wn);
        read_w_group<1>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<R, R + 40, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<2>(slot, Wn);
        read_w_group<3>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<R + 40, 80, WK>::run(v, Wc);
    } else {
        // four bursts of 5 reads, before rounds R, R + 20, R + 40, R + 60
        constexpr int R = PH != 0 ? 10 : 0;
        if constexpr (jn == 0) split_barrier_or_timed<V>(bw);
        RoundsW<0, R, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<0>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<R, R + 20, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<1>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<R + 20, R + 40, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<2>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<R + 40, R + 60, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<3>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<R + 60, 80, WK>::run(v, Wc);
    }
    if constexpr (MASK) {
        const bool live = k < T;
#pragma unroll
        for (int i = 0; i < 5; ++i) h[i] = live ? h[i] + v[i] : h[i];
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) h[i] += v[i];
    }
}

// 2U blocks (two units) per consumer iteration, unrolled, so Wa/Wb keep
// their parity and every barrier position is a compile-time constant.
template <int U, int J, int V, bool MASK, int PH = 0>
struct ConsumeUnits {
    __device__ __forceinline__ static void run(uint32_t k0, uint32_t T, uint32_t (&h)[5],
                                               uint32_t (&Wa)[80], uint32_t (&Wb)[80],
                                               const uint8_t* ring, int lane, uint64_t& bw) {
        if constexpr (J < 2 * U) {
            consume_block<U, J, V, MASK, PH>(k0 + J, T, h, Wa, Wb, ring, lane, bw);
            ConsumeUnits<U, J + 1, V, MASK, PH>::run(k0, T, h, Wb, Wa, ring, lane, bw);
        }
    }
};

// The consumer wave of a split pair: every block's 80 rounds, W+K from the
// ring (see split_body).
template <int U, int V, int PH>
__device__ __forceinline__ void consume_all(const BatchArgs& A, const Entry& en, bool valid, uint32_t T,
                                            uint32_t units, const uint8_t* ring, int lane) {
    uint32_t h[5];
    load_init(A, en.id, h);
    uint32_t Wa[80], Wb[80];
    split_barrier();  // B_0
    read_w_group<0>(ring + lane * 16, Wa);
    read_w_group<1>(ring + lane * 16, Wa);
    read_w_group<2>(ring + lane * 16, Wa);
    read_w_group<3>(ring + lane * 16, Wa);
    // Iterations in which every valid lane is still inside its chunk
    // commit without the per-lane select (all of them for equal lengths).
    const uint32_t Tmin = __builtin_amdgcn_readfirstlane(wave_min(valid ? T : 0xffffffffu));
    const uint32_t full = (V & kVUnmask) ? min(Tmin, units * U) / (2 * U) * (2 * U) : 0u;
    uint32_t k = 0;
    uint64_t bw = 0;
    const uint64_t t0 = (V & kVProbe) ? __builtin_amdgcn_s_memtime() : 0;
    for (; k < full; k += 2 * U) {
        ConsumeUnits<U, 0, V, false, PH>::run(k, T, h, Wa, Wb, ring, lane, bw);
    }
    for (; k < units * U; k += 2 * U) {
        ConsumeUnits<U, 0, V, true, PH>::run(k, T, h, Wa, Wb, ring, lane, bw);
    }
    if constexpr ((V & kVProbe) != 0) {
        const uint64_t tot = __builtin_amdgcn_s_memtime() - t0;
        if (lane == 0) {  // over the group's first digest row
            uint32_t* o = reinterpret_cast<uint32_t*>(A.dig + 20ull * (en.id & ~63u));
            o[0] = (uint32_t)bw;
            o[1] = (uint32_t)(bw >> 32);
            o[2] = (uint32_t)tot;
            o[3] = (uint32_t)(tot >> 32);
            o[4] = units * U;
        }
        return;
    }
    if (valid) emit(A, en.id, h);
}

// PAIRS consumer/producer pairs per workgroup: waves 0..PAIRS-1 consume,
// waves PAIRS..2*PAIRS-1 produce, pair p = (wave p, wave p+PAIRS).  Waves of
// a workgroup are dealt to the CU's SIMDs cyclically, so with PAIRS = 4 each
// SIMD hosts exactly one consumer and its own producer (the consumer keeps
// the SIMD's issue slots it needs; the producer fills the rest).  All waves
// share one s_barrier sequence, so the unit count is the workgroup maximum.
//
// NPROD = 2 (one pair, U = 4): wave 0 consumes, waves 1 and 2 produce,
// each writing one of the unit's two stages.  The producer's schedule work
// per block (byte swap, 64-word expansion, W+K, 20 ds_write_b128) is then
// half as long as the consumer's rounds, so the W+K hand-off, whose
// VOP2-add consumer issues at the 4-cycle floor, is no longer producer-bound
// (tools/consumer_probe, tools/replay_probe).
// The body of one split workgroup `wg` (groups wg*PAIRS ..) over the LDS
// array `lds` (PAIRS * 2 * U * kWBlockBytes bytes): sha1_split_kernel runs
// it on blockIdx.x, the mixed-batch kernel on the workgroups its plan gives
// to this shape.
template <int U, int PAIRS, int V, int NPROD>
__device__ __forceinline__ void split_body(const BatchArgs& A, uint8_t* lds, uint32_t wg) {
    constexpr bool WK = (V & kVWK) != 0;
    static_assert(PAIRS * 2 * U * kWBlockBytes <= 160 * 1024, "LDS");
    // Two producers for 2-block units (each owning one block per unit) were
    // measured slower at two groups per CU: 6 waves on 4 SIMDs put producers
    // on the consumers' SIMDs (profiles/split_2prod_sweep_r01.json).
    static_assert(NPROD == 1 || (PAIRS == 1 && (U == 2 * NPROD || U == NPROD)) ||
                      (PAIRS == 2 && U == NPROD && (V & kVLayout8) != 0),
                  "two producers: one stage (U = 4) or one block (U = 2, 8-wave layout) each per unit");
    int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr ((V & kVSimdRole) != 0) {
        // Roles by the SIMD each wave actually landed on (two 4-wave
        // workgroups per CU, see kVSimdRole): the first workgroup of a CU
        // puts its consumer on SIMD 0, the second on SIMD 2; producers on
        // SIMDs 1 and 3; the wave on the other even SIMD leaves.  Every wave
        // derives the same assignment from the table of all four waves'
        // SIMDs, so exactly one consumer and two producers exist however
        // the waves were placed.
        static_assert(PAIRS == 1 && NPROD == 2 && U == 2, "SIMD roles: one pair, two producers, 2-block units");
        uint32_t* slots = reinterpret_cast<uint32_t*>(lds);
        const uint32_t hw = __builtin_amdgcn_s_getreg((31u << 11) | (0u << 6) | 4u);  // HW_REG_HW_ID, bits 0..31
        if ((threadIdx.x & 63u) == 0) slots[1 + wave] = (hw >> 4) & 3u;
        if (threadIdx.x == 0) slots[0] = cu_turn(hw);
        __syncthreads();
        const uint32_t cs = (__builtin_amdgcn_readfirstlane(slots[0]) & 1u) ? 2u : 0u;
        int wc = -1, wi = -1;
        for (int w = 0; w < 4; ++w)
            if (wc < 0 && slots[1 + w] == cs) wc = w;
        if (wc < 0) wc = 0;
        for (int w = 0; w < 4; ++w)
            if (wi < 0 && w != wc && slots[1 + w] == (cs ^ 2u)) wi = w;
        if (wi < 0) wi = wc == 3 ? 2 : 3;
        int rank = 0;  // producer index: order among the two remaining waves
        for (int w = 0; w < wave; ++w) rank += (w != wc && w != wi) ? 1 : 0;
        __syncthreads();  // the table is read before the ring is written
        if (wave == wi) return;  // never joins a barrier
        wave = wave == wc ? 0 : 1 + rank;
    }
    if constexpr ((V & kVSkipWave2) != 0) {
        static_assert(NPROD == 2 && PAIRS == 1, "skip-wave layout is for two producers");
        if (wave == 2) return;  // never joins a barrier: an ended wave is not waited for
        if (wave > 2) wave -= 1;
    }
    int pair = wave % PAIRS;
    bool producer = wave >= PAIRS;
    uint32_t pidx = producer ? (uint32_t)(wave - PAIRS) / PAIRS : 0u;  // producer index
    if constexpr ((V & kVLayout8) != 0) {
        static_assert(PAIRS == 2 && NPROD == 2, "8-wave layout: two pairs, two producers each");
        if (wave == 4 || wave == 6) return;  // never joins a barrier
        producer = (wave & 1) != 0;
        pair = producer ? (((wave >> 1) & 1) ^ ((V & kVCross) ? 1 : 0)) : (wave >> 1);
        pidx = producer ? (uint32_t)(wave >> 2) : 0u;
    }
    const int lane = threadIdx.x & 63;
    uint8_t* ring = lds + pair * (2 * U * kWBlockBytes);
    const uint32_t group = wg * PAIRS + (uint32_t)pair;
    const uint32_t e = group * 64u + (uint32_t)lane;
    const bool valid = e < A.n;
    Entry en = fetch_entry(A, valid ? e : fallback_entry(A, group));
    if (!valid) en.len = 0;
    // update mode (A.out_state): whole blocks only, no padding
    const uint32_t T = valid ? (A.out_state ? (en.len >> 6) : total_blocks(en.len)) : 0u;
    uint32_t Tmax = __builtin_amdgcn_readfirstlane(wave_max(T));
    if constexpr (PAIRS > 1) {
        // workgroup max through the (not yet used) ring; the second barrier
        // keeps producers from overwriting it before every wave has read it
        uint32_t* slots = reinterpret_cast<uint32_t*>(lds);
        if (!producer && lane == 0) slots[pair] = Tmax;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PAIRS; ++q) Tmax = max(Tmax, slots[q]);
        Tmax = __builtin_amdgcn_readfirstlane(Tmax);
        __syncthreads();
    }
    // Both waves run whole units (2U blocks per consumer iteration); blocks
    // past a lane's T are computed on stale data and never committed.
    const uint32_t units = (Tmax + 2 * U - 1) / (2 * U) * 2;

    if (producer) {
        // ----------------------------- producer -------------------------
        // Bulk: stages (2 full blocks) that every lane has, with
        // branch-free loads hipcc can count (of any alignment); registers
        // hold the current stage and the next one in flight.
        const uint32_t S = bulk_stages(en, valid);
        if constexpr (U == NPROD) {
            // this producer's blocks: k = pidx, pidx + NPROD, ... (one per unit);
            // bulk over the full blocks every lane has, then tail/padding
            const uint32_t K = S * 2u;
            uint32_t B0[16], B1[16];
            uint32_t k = pidx;
            uint64_t pbw = 0;
            uint64_t* const pb = (V & kVProbe) ? &pbw : nullptr;
            const uint64_t pt0 = (V & kVProbe) ? __builtin_amdgcn_s_memtime() : 0;
            if constexpr ((V & kVCoop) != 0) {
                const u32x4u* src[4];
                coop_sources<4>(A, group, (uint32_t)lane, src);
                if (pidx < K) coop4_load(src, pidx, B0);
                if (pidx + NPROD < K) coop4_load(src, pidx + NPROD, B1);
                for (; k + NPROD < K; k += 2 * NPROD) {
                    produce_own_block_coop<U, WK, NPROD>(src, k, K, B0, ring, (uint32_t)lane, pb);
                    produce_own_block_coop<U, WK, NPROD>(src, k + NPROD, K, B1, ring, (uint32_t)lane, pb);
                }
                if (k < K) {
                    produce_own_block_coop<U, WK, NPROD>(src, k, K, B0, ring, (uint32_t)lane, pb);
                    k += NPROD;
                }
            } else {
                if (pidx < K) load_block16(en.p + 64ull * pidx, B0);
                if (pidx + NPROD < K) load_block16(en.p + 64ull * (pidx + NPROD), B1);
                for (; k + NPROD < K; k += 2 * NPROD) {
                    produce_own_block<U, WK, NPROD>(en, k, K, B0, ring, lane, pb);
                    produce_own_block<U, WK, NPROD>(en, k + NPROD, K, B1, ring, lane, pb);
                }
                if (k < K) {
                    produce_own_block<U, WK, NPROD>(en, k, K, B0, ring, lane, pb);
                    k += NPROD;
                }
            }
            for (; k < units * U; k += NPROD) {
                uint32_t w[16];
                if (k < T) tail_block_words(en, k, w);
                produce_block<U, WK, NPROD>(k, w, ring, lane, pb);
            }
            if constexpr ((V & kVProbe) != 0) {
                const uint64_t tot = __builtin_amdgcn_s_memtime() - pt0;
                if (lane == 0) {  // over the group's digest row 1 + pidx
                    uint32_t* o = reinterpret_cast<uint32_t*>(A.dig + 20ull * (group * 64u + 1u + pidx));
                    o[0] = (uint32_t)pbw;
                    o[1] = (uint32_t)(pbw >> 32);
                    o[2] = (uint32_t)tot;
                    o[3] = (uint32_t)(tot >> 32);
                    o[4] = units * U;
                }
            }
            split_barrier();  // matches the consumer's last (unused) read
            return;
        }
        // this producer's stages: s = pidx, pidx + NPROD, ...
        uint32_t s = pidx;
        if constexpr ((V & kVCoop) != 0) {
            const u32x4u* src[8];
            coop_sources<8>(A, group, (uint32_t)lane, src);
            uint32_t C0[32], C1[32];
            if (pidx < S) coop_load(src, pidx, C0);
            if (pidx + NPROD < S) coop_load(src, pidx + NPROD, C1);
            for (; s + NPROD < S; s += 2 * NPROD) {
                produce_stage_coop<U, WK, NPROD>(src, s, S, C0, ring, (uint32_t)lane);
                produce_stage_coop<U, WK, NPROD>(src, s + NPROD, S, C1, ring, (uint32_t)lane);
            }
            if (s < S) {
                produce_stage_coop<U, WK, NPROD>(src, s, S, C0, ring, (uint32_t)lane);
                s += NPROD;
            }
        } else {
            Stage A0, A1;
            if (pidx < S) load_stage(en.p + 128ull * pidx, A0);
            if (pidx + NPROD < S) load_stage(en.p + 128ull * (pidx + NPROD), A1);
            for (; s + NPROD < S; s += 2 * NPROD) {
                produce_stage<U, WK, NPROD>(en, s, S, A0, ring, lane);
                produce_stage<U, WK, NPROD>(en, s + NPROD, S, A1, ring, lane);
            }
            if (s < S) {
                produce_stage<U, WK, NPROD>(en, s, S, A0, ring, lane);
                s += NPROD;
            }
        }
        // tail and padding stages (whole units: blocks past a lane's T are
        // never committed by the consumer)
        for (; 2 * s < units * U; s += NPROD) {
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const uint32_t k = 2 * s + half;
                uint32_t w[16];
                if (k < T) tail_block_words(en, k, w);
                produce_block<U, WK, NPROD>(k, w, ring, lane);
            }
        }
        split_barrier();  // matches the consumer's last (unused) read
    } else {
        // ----------------------------- consumer -------------------------
        if constexpr ((V & kVPhase2) != 0) {
            if (pair == 1)
                consume_all<U, V, 3>(A, en, valid, T, units, ring, lane);
            else
                consume_all<U, V, 1>(A, en, valid, T, units, ring, lane);
            return;
        }
        if constexpr ((V & kVPhase) != 0) {
            if (pair == 1) {
                consume_all<U, V, 2>(A, en, valid, T, units, ring, lane);
                return;
            }
        }
        consume_all<U, V, 0>(A, en, valid, T, units, ring, lane);
    }
}

// The 8-wave two-pair shape (product case 11, the mixed kernel's mode 1).
constexpr int kSplit8V = kVWK | kVUnmask | kVLayout8 | kVCross | kVCoop;

template <int U, int PAIRS, int V = kSplitV<U>, int NPROD = 1>
__global__ __launch_bounds__((kSplitThreads<PAIRS, V, NPROD>)) void sha1_split_kernel(
    BatchArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[PAIRS * 2 * U * kWBlockBytes];
    split_body<U, PAIRS, V, NPROD>(A, lds, blockIdx.x);
}


// --------------------------------------------------------------- fused ----
// One wave, 64 chunks, schedule and rounds in registers (~630 VALU per
// block).  Best once there are enough chunks for two or more waves per SIMD:
// then the SIMD, not one wave's issue rate, is the limit and the split
// kernel's LDS hand-off is pure overhead.  Each lane streams its own chunk
// with 16-byte loads (dword loads shifted at use when the wave's chunks are
// not all 16-byte aligned), two 128-byte stages (4 blocks) in flight in VGPRs so
// HBM latency under full load stays covered.
template <typename V>
__device__ __forceinline__ void fused_stage(uint32_t s, uint32_t S, const Entry& en, Stage& cur,
                                            uint32_t (&h)[5]) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap_fresh(cur.w[16 * half + j]);
        if (half == 1 && s + 2 < S) load_stage<V>(en.p + 128ull * (s + 2), cur);
        compress(h, w);
    }
}

// Stages 0 .. S-1 of every lane's chunk, each lane loading its own.
template <typename V>
__device__ __forceinline__ void fused_lane_stages_v(const Entry& en, uint32_t S, uint32_t (&h)[5]) {
    Stage A0, A1;
    if (S > 0) load_stage<V>(en.p, A0);
    if (S > 1) load_stage<V>(en.p + 128, A1);
    uint32_t s = 0;
    for (; s + 1 < S; s += 2) {
        fused_stage<V>(s, S, en, A0, h);
        fused_stage<V>(s + 1, S, en, A1, h);
    }
    if (s < S) fused_stage<V>(s, S, en, A0, h);
}

// The same for a wave whose chunks are not all 16-byte aligned: dword loads
// (RawSpan, from p & ~3) two stages ahead, funnel-shifted by p & 3 at use.
// Lane-per-chunk byte-unaligned 16-byte loads were slower here (65536 x
// 512 KiB 1..15 bytes off: 13.6 ms against 11.2; profiles/misaligned_r02.json).
__device__ __forceinline__ void fused_stage_any(uint32_t s, uint32_t S, const Entry& en, RawSpan<32>& cur,
                                                uint32_t (&h)[5]) {
    const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(en.p) & 3u);
    uint32_t w[16];
    shift_raw<32, 0, 16>(cur, sh, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap_fresh(w[j]);
    compress(h, w);
    shift_raw<32, 16, 16>(cur, sh, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap_fresh(w[j]);
    if (s + 2 < S) load_raw<32>(en.p + 128ull * (s + 2), cur);
    compress(h, w);
}

__device__ __forceinline__ void fused_lane_stages_any(const Entry& en, uint32_t S, uint32_t (&h)[5]) {
    RawSpan<32> A0, A1;
    if (S > 0) load_raw<32>(en.p, A0);
    if (S > 1) load_raw<32>(en.p + 128, A1);
    uint32_t s = 0;
    for (; s + 1 < S; s += 2) {
        fused_stage_any(s, S, en, A0, h);
        fused_stage_any(s + 1, S, en, A1, h);
    }
    if (s < S) fused_stage_any(s, S, en, A0, h);
}

__device__ __forceinline__ void fused_lane_stages(const Entry& en, bool valid, uint32_t S, uint32_t (&h)[5]) {
    if (wave_all(!valid || (reinterpret_cast<uintptr_t>(en.p) & 15u) == 0))
        fused_lane_stages_v<uint4>(en, S, h);
    else
        fused_lane_stages_any(en, S, h);
}

// The body of one fused wave: message e's lane (group e / 64).
__device__ __forceinline__ void fused_body(const BatchArgs& A, uint32_t e) {
    const uint32_t group = e / 64u;
    const bool valid = e < A.n;
    Entry en = fetch_entry(A, valid ? e : fallback_entry(A, group));
    if (!valid) en.len = 0;
    uint32_t h[5];
    load_init(A, en.id, h);
    const uint32_t S = bulk_stages(en, valid);
    fused_lane_stages(en, valid, S, h);
    if (valid) {
        lane_blocks(A, en, 2u * S, h);
        emit(A, en.id, h);
    }
}


// ---------------------------------------------------------- coop fused ----
// The fused wave with its stage loads shared across the wave
// (coop_load / coop_store / coop_read, above the split kernel).  Used by the
// mixed kernel, whose workgroups own the CU's LDS anyway (16 KiB per wave:
// two stage buffers).
__device__ __forceinline__ void coop_compress(const uint32_t (&cur)[32], uint32_t (&h)[5]) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap_fresh(cur[16 * half + j]);
        compress(h, w);
    }
}

// LDS-DMA (global_load_lds_dwordx4): each lane's 16 bytes from its own
// global address land at the wave-uniform LDS byte address `lds_dst` +
// 16 x lane, with no VGPR and no ds_write.  M0 carries the LDS address and is
// saved and restored in the same statement (hipcc reserves it).  hipcc does
// not count these loads: the caller waits for them with an explicit
// s_waitcnt vmcnt (and drains them before any load hipcc counts).
typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ uint32_t lds_addr(const uint8_t* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const lds_u8*)p));
}
__device__ __forceinline__ void glds16(const void* src, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_dst)
                 : "memory");
}

// Block k of the group's 64 chunks into the 4 KiB buffer at LDS address
// `buf`: instruction i reads block k of chunks 16i .. 16i+15 (4 lanes per
// chunk), lane l writing buf + i KiB + 16 l.  p[i] is lane l's source in
// chunk 16i + l/4 at byte 16 x ((l%4 - l/16) & 3) of the block, so the LDS
// image is coop4_store's swizzled one (piece q of chunk c at
// c*64 + ((q + c/4) & 3)*16) and coop4_read hands each lane its chunk.
__device__ __forceinline__ void glds_block(const uint8_t* const (&p)[4], uint32_t k, uint32_t buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(p[i] + 64ull * k, buf + 1024u * (uint32_t)i);
}

// Block k of the LDS-DMA fused loop: `cur` holds block k (its LDS read
// issued during block k-1); block k+1's read is issued into `nxt` once its
// DMA has landed, block k+4's DMA goes into block k-1's buffer (read during
// block k-2, consumed during block k-1), then block k is compressed while
// block k+1's read is in flight.  At the start of block k the DMAs of
// blocks k+1..k+3 are outstanding (12 loads): vmcnt(8) retires block k+1.
__device__ __forceinline__ void glds_stage_step(const uint8_t* const (&p)[4], uint32_t k, uint32_t K,
                                                const uint8_t* lds, uint32_t base, uint32_t lane, uint32_t& b,
                                                const uint32_t (&cur)[16], uint32_t (&nxt)[16],
                                                uint32_t (&h)[5]) {
    const uint32_t b1 = b + 1u == kCoopBlockBufs ? 0u : b + 1u;      // block k+1's buffer
    const uint32_t bp = b == 0u ? kCoopBlockBufs - 1u : b - 1u;      // block k-1's buffer
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    coop4_read(lds + b1 * kCoopBlockBytes, lane, nxt);
    glds_block(p, min(k + kCoopBlockBufs - 1u, K - 1u), base + bp * kCoopBlockBytes);
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap_fresh(cur[j]);
    compress(h, w);
    b = b1;
}

// lds: this wave's kCoopWaveBytes.  Same contract as fused_body.  The
// wave's LDS accesses complete in order, so a stage's stores precede its
// reads and the reads of a buffer precede its next stores; hipcc keeps the
// program order of these lane-dependent accesses it cannot prove disjoint.
// One stage in flight in registers: a second (as fused_body keeps) was
// slower -- hipcc moved its loads next to their LDS stores (65536 x 512 KiB
// 13.1 against 10.4 ms, profiles/coop_split_ab_r02.json).
__device__ __forceinline__ void fused_coop_body(const BatchArgs& A, uint32_t e, uint8_t* lds) {
    const uint32_t group = e / 64u, lane = e & 63u;
    const bool valid = e < A.n;
    Entry en = fetch_entry(A, valid ? e : fallback_entry(A, group));
    if (!valid) en.len = 0;
    uint32_t h[5];
    load_init(A, en.id, h);
    const uint32_t S = bulk_stages(en, valid);
    // A group whose chunks lie together (in place, or permuted within a
    // span of about their own bytes) streams lane-per-chunk: no UTCL1
    // thrash to avoid there, and the shared loads' LDS round trip costs
    // 1-4 % (profiles/coop_split_ab_r02.json).
    uint64_t lo = valid ? reinterpret_cast<uint64_t>(en.p) : ~0ull;
    uint64_t hi = valid ? reinterpret_cast<uint64_t>(en.p) + en.len : 0ull;
    uint64_t bytes = valid ? en.len : 0ull;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        lo = min(lo, (uint64_t)__shfl_xor(lo, m));
        hi = max(hi, (uint64_t)__shfl_xor(hi, m));
        bytes += (uint64_t)__shfl_xor(bytes, m);
    }
    const bool together = hi - lo <= 2 * bytes + (2ull << 20);
    if (S > 0 && together && wave_all(!valid || (reinterpret_cast<uintptr_t>(en.p) & 15u) == 0)) {
        fused_lane_stages_v<uint4>(en, S, h);
    } else if (S > 0) {  // scattered or not 16-byte aligned: shared loads (any alignment)
        // Block loads shared across the wave go straight to LDS
        // (global_load_lds), four blocks ahead in five 4 KiB buffers; each
        // lane then reads its own chunk's block back (coop4_read).  Round 4
        // staged 128-byte stages through VGPRs (8 global loads + 8
        // ds_write_b128 per stage) with one stage in flight: this wave IS its
        // chunks' chain (alone on its SIMD at F = 4), so a scattered load that
        // had not landed one stage (~4900 cycles) later stalled it, and a
        // second register stage did not fit the mixed kernel's 256 VGPRs
        // (65536 uniform chunks permuted: 11.4 ms against 10.1 in place).
        const uint32_t K = 2u * S;
        const uint8_t* p[4];
        const uint32_t piece = ((lane & 3u) - (lane >> 4)) & 3u;
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t ej = group * 64u + 16u * i + (lane >> 2);
            p[i] = fetch_entry(A, ej < A.n ? ej : fallback_entry(A, group)).p + 16u * piece;
        }
        const uint32_t base = lds_addr(lds);
        // blocks 0..3 in flight (past the bulk region: the last block again,
        // a harmless repeat that keeps the count of loads in flight fixed)
#pragma unroll
        for (uint32_t d = 0; d < kCoopBlockBufs - 1u; ++d) glds_block(p, min(d, K - 1u), base + d * kCoopBlockBytes);
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // block 0 landed
        uint32_t wa[16], wb[16];
        coop4_read(lds, lane, wa);
        uint32_t b = 0;  // buffer of block k
        uint32_t k = 0;
        for (; k + 1 < K; k += 2) {
            glds_stage_step(p, k, K, lds, base, lane, b, wa, wb, h);
            glds_stage_step(p, k + 1, K, lds, base, lane, b, wb, wa, h);
        }
        if (k < K) glds_stage_step(p, k, K, lds, base, lane, b, wa, wb, h);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing of ours in flight past the loop
    }
    if (valid) {
        lane_blocks(A, en, 2u * S, h);
        emit(A, en.id, h);
    }
}

#endif
