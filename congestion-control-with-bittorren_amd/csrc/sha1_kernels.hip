// sha1_kernels.hip -- gfx950 kernels of the SHA-1 chunk engine.
//
// The reference hashes one chunk at a time on one CPU core (make_chunks loop
// chunk.c:22-24 -> shahash chunk.c:35-51 -> SHA1Update sha.c:453-527 ->
// SHA1Guts sha.c:176-451).  Here every lane owns one chunk and a wave hashes
// 64 chunks in lockstep.  SHA-1 is serial inside a message (Merkle-Damgard:
// sha.c:518 carries sc->hash from block to block), so the only parallelism
// is across chunks; the kernels differ in how a lane gets its 64-byte blocks
// and who computes the message schedule:
//
//   sha1_lane_kernel   each lane loads its own blocks from HBM (any byte
//                      alignment, any length); also the streaming kernel
//                      behind SHA1Update/SHA1Final (init state + no-final).
//   sha1_fused_kernel  one wave per 64 chunks, schedule + rounds in VGPRs
//                      (~627 instructions per block), two 128-byte stages of
//                      each chunk prefetched per lane.  The high-occupancy
//                      kernel: > 2 groups of 64 chunks per CU.
//   sha1_split_kernel  workgroup = consumer wave + producer wave(s) on the
//                      same 64 chunks.  Producers stream and byte-swap the
//                      blocks and expand the 80-word schedule (+K) into an
//                      LDS ring; the consumer runs only the 80 rounds (~428
//                      instructions per block instead of ~627), which is the
//                      bound when there are too few chunks to fill the
//                      SIMDs (BASELINE config 2: 4096 chunks = 64 waves).
//                      One wave's 20 ds_write_b128 per block cost ~28 cycles
//                      each on top of its VALU (tools/gen_producer_probe.py),
//                      so one producer is as slow as the consumer: each
//                      consumer gets two producers, laid out so that it has a
//                      SIMD to itself (a workgroup's waves 0-3 land on four
//                      different SIMDs, wave w + 4 on wave w's:
//                      tools/wave_placement_probe.hip).
//   sha1_mixed_kernel  ragged batches sorted longest-first with more groups
//                      than CUs: one launch whose workgroups run the split
//                      body (longest groups) or the fused body, per a
//                      device-side plan (plan_mixed_kernel) -- see `mixed`.
//
// Measured on MI355X (tools/issue_probe.hip, tools/gen_consumer_probe.py,
// DESIGN.md section 5): one wave issues at most one instruction per 4.0
// cycles; its round stream reaches that with x = e + (W+K) as a VOP2 add and
// runs at ~5 cycles per VALU with a VOP3 add3 of K; at several waves per SIMD
// v_alignbit/v_add3/v_perm cost ~1.9 ns of SIMD time per wave-instruction vs
// ~1.1 ns for v_add/v_xor/v_bitop3.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "sha1_device.hpp"
#include "sha1_kernels.h"

using namespace s1;

namespace {

struct Entry {
    uint32_t id;
    const uint8_t* p;
    uint32_t len;
};

__device__ __forceinline__ Entry fetch_entry(const BatchArgs& A, uint32_t e) {
    Entry r;
    r.id = A.order ? A.order[e] : e;
    const uint64_t off = A.off ? A.off[r.id] : (uint64_t)r.id * A.ulen;
    r.p = A.base + off;
    r.len = A.len ? A.len[r.id] : A.ulen;
    return r;
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
    uint32_t cur[16], nxt[16];
    if (k0 < nfull) load_block16(en.p + 64ull * k0, cur);
    for (uint32_t k = k0; k < nfull; ++k) {
        if (k + 1 < nfull) load_block16(en.p + 64ull * (k + 1), nxt);
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap(cur[j]);
        compress(h, w);
#pragma unroll
        for (int j = 0; j < 16; ++j) cur[j] = nxt[j];
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

// ---------------------------------------------------------------- lane ----
__global__ __launch_bounds__(256) void sha1_lane_kernel(BatchArgs A) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= A.n) return;
    const Entry en = fetch_entry(A, e);
    uint32_t h[5];
    load_init(A, en.id, h);
    lane_blocks(A, en, 0, h);
    emit(A, en.id, h);
}

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

// Global-memory W ring (A/B flag kVGlobalW, defined with the variant flags).
typedef uint32_t gw_u4 __attribute__((ext_vector_type(4)));
struct GRing {
    __amdgpu_buffer_rsrc_t r;
    uint32_t base;  // byte offset of this group's ring
};
__device__ __forceinline__ void gw_barrier() {
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0) (gfx9 encoding)
    asm volatile("s_barrier" ::: "memory");
}
template <int T, bool WK>
struct SchedWriteG {
    __device__ __forceinline__ static void run(uint32_t (&w)[16], const GRing& g, uint32_t off, int lane) {
        if constexpr (T < 80) {
            if constexpr (T >= 16) sched_step<T>(w);
            if constexpr ((T & 3) == 3) {
                constexpr int j = (T - 3) & 15;
                constexpr uint32_t k = WK ? round_k<T>() : 0u;
                gw_u4 x = {w[j] + k, w[j + 1] + k, w[j + 2] + k, w[j + 3] + k};
                __builtin_amdgcn_raw_buffer_store_b128(x, g.r, (int)(g.base + off + (T >> 2) * 1024 + lane * 16), 0,
                                                       16);
            }
            SchedWriteG<T + 1, WK>::run(w, g, off, lane);
        }
    }
};
template <int P>
__device__ __forceinline__ void read_w_group_g(const GRing& g, uint32_t off, uint32_t lane, uint32_t (&W)[80]) {
#pragma unroll
    for (int q = 5 * P; q < 5 * P + 5; ++q) {
        // one voffset VGPR (lane + group); the slot and quad go in soffset
        // (a constant) + the 12-bit immediate
        const gw_u4 x = __builtin_amdgcn_raw_buffer_load_b128(g.r, (int)(g.base + lane * 16 + (q & 3) * 1024),
                                                              (int)(off + (q >> 2) * 4096), 16);
        W[4 * q + 0] = x.x;
        W[4 * q + 1] = x.y;
        W[4 * q + 2] = x.z;
        W[4 * q + 3] = x.w;
    }
}

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
__device__ __forceinline__ void produce_block(uint32_t k, uint32_t (&w)[16], uint8_t* ring, int lane) {
    const uint32_t m = k / U, j = k - m * U;
    SchedWrite<0, WK>::run(w, ring + ((m & 1u) * U + j) * kWBlockBytes, lane);
    // U == NPROD: each producer writes one block of every unit
    if (NPROD == 1 ? j == U - 1 : (U == NPROD || (k & 1u) == 1u)) split_barrier();
}

template <int U, bool WK, int NPROD = 1>
__device__ __forceinline__ void produce_block_g(uint32_t k, uint32_t (&w)[16], const GRing& g, int lane) {
    const uint32_t m = k / U, j = k - m * U;
    SchedWriteG<0, WK>::run(w, g, ((m & 1u) * U + j) * kWBlockBytes, lane);
    if (NPROD == 1 ? j == U - 1 : (U == NPROD || (k & 1u) == 1u)) gw_barrier();
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
constexpr uint32_t kCoopWaveBytes = 2u * kCoopStageBytes;

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
// and at least as long as the wave's bulk region).
template <int LANES>
__device__ __forceinline__ void coop_sources(const BatchArgs& A, uint32_t group, uint32_t lane,
                                             const u32x4u* (&src)[LANES]) {
#pragma unroll
    for (uint32_t i = 0; i < (uint32_t)LANES; ++i) {
        const uint32_t ej = group * 64u + (64u / LANES) * i + lane / LANES;
        src[i] = reinterpret_cast<const u32x4u*>(fetch_entry(A, ej < A.n ? ej : group * 64u).p) + (lane % LANES);
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

// kVGlobalW: the same, W+K to the global ring (the LDS slot still stages the
// shared loads' transpose)
template <int U, bool WK, int NPROD = 1>
__device__ __forceinline__ void produce_stage_coop_g(const u32x4u* const (&src)[8], uint32_t s, uint32_t S,
                                                     uint32_t (&cur)[32], uint8_t* ring, const GRing& g,
                                                     uint32_t lane) {
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
        produce_block_g<U, WK, NPROD>(k0 + half, w, g, (int)lane);
    }
}

template <int U, bool WK, int NPROD>
__device__ __forceinline__ void produce_own_block_coop(const u32x4u* const (&src)[4], uint32_t k, uint32_t K,
                                                       uint32_t (&cur)[16], uint8_t* ring, uint32_t lane) {
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
    produce_block<U, WK, NPROD>(k, w, ring, (int)lane);
}

// Producer that owns one block per unit (U == NPROD): block k from `cur`,
// which is then refilled with this producer's block after next, k + 2 NPROD.
template <int U, bool WK, int NPROD>
__device__ __forceinline__ void produce_own_block(const Entry& en, uint32_t k, uint32_t K,
                                                  uint32_t (&cur)[16], uint8_t* ring, int lane) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap(cur[j]);
    if (k + 2 * NPROD < K) load_block16(en.p + 64ull * (k + 2 * NPROD), cur);
    produce_block<U, WK, NPROD>(k, w, ring, lane);
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
// Split-kernel variant flags (A/B switches, defaults in kSplitV).
constexpr int kVWK = 1;      // producer ships W+K (consumer: one VOP2 add)
constexpr int kVRtSlot = 2;  // slot address computed at run time
constexpr int kVUnmask = 4;  // unmasked commit while every lane is live
constexpr int kVRead10 = 8;  // schedule reads in two bursts of 10 instead of four of 5
// (The timing study behind these defaults also used variants in which the
// consumer skipped its LDS reads or one side idled at the barriers; their
// digests are wrong by design, so they are not built into the library.
// Results: profiles/issue_r01.json, profiles/split_2prod_sweep_r01.json.)
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
constexpr int kVSkipWave1 = 512;  // with kVSkipWave2: leave wave 1 empty instead of wave 2 (A/B)
constexpr int kVCross = 256;
// Round-3 A/B (A/B library only): the 8-wave layout with the consumers on
// waves 0 and 1 (different halves of the LDS store path, SIMDs {0,1} / {2,3})
// and the producers on waves 2 + 6 and 3 + 7 (waves 4, 5 empty), so each half
// carries one consumer's reads and two producers' stores; with kVCross each
// consumer's producers sit on the other half.
constexpr int kVHalves = 32768;
// Round-2 A/B flags (A/B library only): consumer at s_setprio 3; all 20
// schedule reads of the next block in one burst before round 0.
constexpr int kVPrio = 2048;
constexpr int kVRead20 = 4096;
// Producers load with shared loads (4 or 8 lanes per chunk, staged through
// the W slot): one load instruction touches 16 or 8 chunks instead of 64
// (see `shared loads`).
constexpr int kVCoop = 8192;
// Round-2 A/B (A/B library only): the W+K ring in global memory (L2) instead
// of LDS -- producers buffer-store it, the consumer buffer-loads it at device
// scope (sc1: misses the CU's L1, hits the XCD's L2), with vmcnt(0) at the
// barriers.  Tests whether a vector-memory load of the schedule costs the
// consumer's issue stream less than a ds_read_b128 (~6 cycles).
constexpr int kVGlobalW = 16384;
template <int PAIRS, int V, int NPROD>
constexpr int kSplitThreads = (V & kVLayout8) ? 512 : 64 * PAIRS * (1 + NPROD) + ((V & kVSkipWave2) ? 64 : 0);
// Why W+K matters: the consumer's x = e + W + K as a VOP3 v_add3 (K in an
// SGPR or a VGPR alike) runs the one-wave round stream at ~4.98 cycles per
// instruction, the VOP2 v_add on a shipped W+K at the 4-cycle issue floor
// (tools/consumer_probe, profiles/issue_r01.json).  With ONE producer the
// extra 80 adds per block make the producer the slower wave (1878 vs 1757
// cycles per block), so single-producer kernels with 3- and 4-block units
// keep K in the consumer; the 4-block default has TWO producers (kSplitNProd)
// and ships W+K.  Measured on MI355X (profiles/split_variants_r01.json):
// 2-block units W+K ~5% ahead, the slot-address form neutral there; unmasked
// commit helps every shape.
template <int U>
constexpr int kSplitV = U == 4 ? (kVWK | kVUnmask | kVSkipWave2 | kVRead10 | kVCoop)
                               : U == 3 ? (kVRtSlot | kVUnmask) : (kVWK | kVUnmask);
template <int U>
constexpr int kSplitNProd = U == 4 ? 2 : 1;

template <int U, int J, int V, bool MASK>
__device__ __forceinline__ void consume_block(uint32_t k, uint32_t T, uint32_t (&h)[5],
                                              const uint32_t (&Wc)[80], uint32_t (&Wn)[80],
                                              const uint8_t* ring, const GRing& g, int lane) {
    // Block k+1 (k = k0 + J, k0 a multiple of 2U) is unit (k0/U + (J+1)/U),
    // whose parity is that of (J+1)/U since k0/U is even, and sub-block
    // (J+1) % U: the slot address is a compile-time offset.  A barrier goes
    // in front of the first read of every new unit.
    constexpr bool WK = (V & kVWK) != 0;
    constexpr int jn = (J + 1) % U;
    constexpr int slot_idx = (((J + 1) / U) & 1) * U + jn;
    const uint8_t* slot;
    if constexpr ((V & kVRtSlot) != 0) {
        const uint32_t mn = (k + 1) / U;
        slot = ring + ((mn & 1u) * U + jn) * kWBlockBytes + lane * 16;
    } else {
        slot = ring + slot_idx * kWBlockBytes + lane * 16;
    }
    uint32_t v[5] = {h[0], h[1], h[2], h[3], h[4]};
    if constexpr ((V & kVGlobalW) != 0) {
        static_assert((V & (kVRtSlot | kVRead20)) == 0 && (V & kVRead10) != 0, "global W: the product's read order");
        // this block's W (loaded during the previous block) in one wait, so
        // hipcc adds none per quad
        if constexpr (jn == 0)
            gw_barrier();
        else
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        constexpr uint32_t off = slot_idx * kWBlockBytes;
        read_w_group_g<0>(g, off, lane, Wn);
        read_w_group_g<1>(g, off, lane, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<0, 40, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group_g<2>(g, off, lane, Wn);
        read_w_group_g<3>(g, off, lane, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<40, 80, WK>::run(v, Wc);
    } else if constexpr ((V & kVRead20) != 0) {
        if constexpr (jn == 0) split_barrier();
        read_w_group<0>(slot, Wn);
        read_w_group<1>(slot, Wn);
        read_w_group<2>(slot, Wn);
        read_w_group<3>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<0, 80, WK>::run(v, Wc);
    } else if constexpr ((V & kVRead10) != 0) {
        if constexpr (jn == 0) split_barrier();
        // two bursts of 10 reads (before rounds 0 and 40)
        read_w_group<0>(slot, Wn);
        read_w_group<1>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<0, 40, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<2>(slot, Wn);
        read_w_group<3>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<40, 80, WK>::run(v, Wc);
    } else {
        if constexpr (jn == 0) split_barrier();
        read_w_group<0>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<0, 20, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<1>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<20, 40, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<2>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<40, 60, WK>::run(v, Wc);
        __builtin_amdgcn_sched_barrier(0);
        read_w_group<3>(slot, Wn);
        __builtin_amdgcn_sched_barrier(0);
        RoundsW<60, 80, WK>::run(v, Wc);
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
template <int U, int J, int V, bool MASK>
struct ConsumeUnits {
    __device__ __forceinline__ static void run(uint32_t k0, uint32_t T, uint32_t (&h)[5],
                                               uint32_t (&Wa)[80], uint32_t (&Wb)[80],
                                               const uint8_t* ring, const GRing& g, int lane) {
        if constexpr (J < 2 * U) {
            consume_block<U, J, V, MASK>(k0 + J, T, h, Wa, Wb, ring, g, lane);
            ConsumeUnits<U, J + 1, V, MASK>::run(k0, T, h, Wb, Wa, ring, g, lane);
        }
    }
};

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
__device__ __forceinline__ void split_body(const BatchArgs& A, uint8_t* lds, uint32_t wg,
                                           uint8_t* wring = nullptr) {
    constexpr bool WK = (V & kVWK) != 0;
    constexpr bool GW = (V & kVGlobalW) != 0;
    static_assert(!GW || (U == 4 && PAIRS == 1 && NPROD == 2 && (V & kVCoop) != 0), "global W: the config-2 shape");
    static_assert(PAIRS * 2 * U * kWBlockBytes <= 160 * 1024, "LDS");
    // Two producers for 2-block units (each owning one block per unit) were
    // measured slower at two groups per CU: 6 waves on 4 SIMDs put producers
    // on the consumers' SIMDs (profiles/split_2prod_sweep_r01.json).
    static_assert(NPROD == 1 || (PAIRS == 1 && (U == 2 * NPROD || U == NPROD)) ||
                      (PAIRS == 2 && U == NPROD && (V & kVLayout8) != 0),
                  "two producers: one stage (U = 4) or one block (U = 2, 8-wave layout) each per unit");
    int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr ((V & kVSkipWave2) != 0) {
        static_assert(NPROD == 2 && PAIRS == 1, "skip-wave layout is for two producers");
        // kVSkipWave1 (A/B): wave 1 stays empty instead, producers on waves 2 and 3
        constexpr int skip = (V & kVSkipWave1) ? 1 : 2;
        if (wave == skip) return;  // never joins a barrier: an ended wave is not waited for
        if (wave > skip) wave -= 1;
    }
    int pair = wave % PAIRS;
    bool producer = wave >= PAIRS;
    uint32_t pidx = producer ? (uint32_t)(wave - PAIRS) / PAIRS : 0u;  // producer index
    if constexpr ((V & kVLayout8) != 0) {
        static_assert(PAIRS == 2 && NPROD == 2, "8-wave layout: two pairs, two producers each");
        if constexpr ((V & kVHalves) != 0) {
            if (wave == 4 || wave == 5) return;  // never joins a barrier
            producer = wave >= 2;
            pair = producer ? ((wave & 1) ^ ((V & kVCross) ? 1 : 0)) : wave;
        } else {
            if (wave == 4 || wave == 6) return;  // never joins a barrier
            producer = (wave & 1) != 0;
            pair = producer ? (((wave >> 1) & 1) ^ ((V & kVCross) ? 1 : 0)) : (wave >> 1);
        }
        pidx = producer ? (uint32_t)(wave >> 2) : 0u;
    }
    const int lane = threadIdx.x & 63;
    uint8_t* ring = lds + pair * (2 * U * kWBlockBytes);
    const uint32_t group = wg * PAIRS + (uint32_t)pair;
    GRing g{};
    if constexpr (GW) g = GRing{__builtin_amdgcn_make_buffer_rsrc(wring, 0, 0x7fffffff, 0x00020000),
                                group * (2u * U * kWBlockBytes)};
    const uint32_t e = group * 64u + (uint32_t)lane;
    const bool valid = e < A.n;
    Entry en = fetch_entry(A, valid ? e : min(group * 64u, A.n - 1u));
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
            if constexpr ((V & kVCoop) != 0) {
                const u32x4u* src[4];
                coop_sources<4>(A, group, (uint32_t)lane, src);
                if (pidx < K) coop4_load(src, pidx, B0);
                if (pidx + NPROD < K) coop4_load(src, pidx + NPROD, B1);
                for (; k + NPROD < K; k += 2 * NPROD) {
                    produce_own_block_coop<U, WK, NPROD>(src, k, K, B0, ring, (uint32_t)lane);
                    produce_own_block_coop<U, WK, NPROD>(src, k + NPROD, K, B1, ring, (uint32_t)lane);
                }
                if (k < K) {
                    produce_own_block_coop<U, WK, NPROD>(src, k, K, B0, ring, (uint32_t)lane);
                    k += NPROD;
                }
            } else {
                if (pidx < K) load_block16(en.p + 64ull * pidx, B0);
                if (pidx + NPROD < K) load_block16(en.p + 64ull * (pidx + NPROD), B1);
                for (; k + NPROD < K; k += 2 * NPROD) {
                    produce_own_block<U, WK, NPROD>(en, k, K, B0, ring, lane);
                    produce_own_block<U, WK, NPROD>(en, k + NPROD, K, B1, ring, lane);
                }
                if (k < K) {
                    produce_own_block<U, WK, NPROD>(en, k, K, B0, ring, lane);
                    k += NPROD;
                }
            }
            for (; k < units * U; k += NPROD) {
                uint32_t w[16];
                if (k < T) tail_block_words(en, k, w);
                produce_block<U, WK, NPROD>(k, w, ring, lane);
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
            if constexpr (GW) {
                for (; s + NPROD < S; s += 2 * NPROD) {
                    produce_stage_coop_g<U, WK, NPROD>(src, s, S, C0, ring, g, (uint32_t)lane);
                    produce_stage_coop_g<U, WK, NPROD>(src, s + NPROD, S, C1, ring, g, (uint32_t)lane);
                }
                if (s < S) {
                    produce_stage_coop_g<U, WK, NPROD>(src, s, S, C0, ring, g, (uint32_t)lane);
                    s += NPROD;
                }
            } else {
                for (; s + NPROD < S; s += 2 * NPROD) {
                    produce_stage_coop<U, WK, NPROD>(src, s, S, C0, ring, (uint32_t)lane);
                    produce_stage_coop<U, WK, NPROD>(src, s + NPROD, S, C1, ring, (uint32_t)lane);
                }
                if (s < S) {
                    produce_stage_coop<U, WK, NPROD>(src, s, S, C0, ring, (uint32_t)lane);
                    s += NPROD;
                }
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
                if constexpr (GW)
                    produce_block_g<U, WK, NPROD>(k, w, g, lane);
                else
                    produce_block<U, WK, NPROD>(k, w, ring, lane);
            }
        }
        if constexpr (GW)
            gw_barrier();
        else
            split_barrier();  // matches the consumer's last (unused) read
    } else {
        // ----------------------------- consumer -------------------------
        uint32_t h[5];
        load_init(A, en.id, h);
        uint32_t Wa[80], Wb[80];
        if constexpr ((V & kVPrio) != 0) __builtin_amdgcn_s_setprio(3);
        if constexpr (GW) {
            gw_barrier();  // B_0
            read_w_group_g<0>(g, 0, lane, Wa);
            read_w_group_g<1>(g, 0, lane, Wa);
            read_w_group_g<2>(g, 0, lane, Wa);
            read_w_group_g<3>(g, 0, lane, Wa);
        } else {
            split_barrier();  // B_0
            read_w_group<0>(ring + lane * 16, Wa);
            read_w_group<1>(ring + lane * 16, Wa);
            read_w_group<2>(ring + lane * 16, Wa);
            read_w_group<3>(ring + lane * 16, Wa);
        }
        // Iterations in which every valid lane is still inside its chunk
        // commit without the per-lane select (all of them for equal lengths).
        const uint32_t Tmin = __builtin_amdgcn_readfirstlane(wave_min(valid ? T : 0xffffffffu));
        const uint32_t full = (V & kVUnmask) ? min(Tmin, units * U) / (2 * U) * (2 * U) : 0u;
        uint32_t k = 0;
        for (; k < full; k += 2 * U) {
            ConsumeUnits<U, 0, V, false>::run(k, T, h, Wa, Wb, ring, g, lane);
        }
        for (; k < units * U; k += 2 * U) {
            ConsumeUnits<U, 0, V, true>::run(k, T, h, Wa, Wb, ring, g, lane);
        }
        if (valid) emit(A, en.id, h);
    }
}

template <int U, int PAIRS, int V = kSplitV<U>, int NPROD = 1>
__global__ __launch_bounds__((kSplitThreads<PAIRS, V, NPROD>)) void sha1_split_kernel(
    BatchArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[PAIRS * 2 * U * kWBlockBytes];
    split_body<U, PAIRS, V, NPROD>(A, lds, blockIdx.x);
}

#ifdef SHA1CHUNK_AB_VARIANTS
// kVGlobalW A/B: the config-2 shape with its W+K ring in `wring` (groups x
// 2 x U x 20 KiB of device memory)
template <int V>
__global__ __launch_bounds__((kSplitThreads<1, V, 2>)) void sha1_split_gw_kernel(BatchArgs A, uint8_t* wring) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 4 * kWBlockBytes];
    split_body<4, 1, V, 2>(A, lds, blockIdx.x, wring);
}
#endif

// --------------------------------------------------------------- fused ----
// One wave, 64 chunks, schedule and rounds in registers (~630 VALU per
// block).  Best once there are enough chunks for two or more waves per SIMD:
// then the SIMD, not one wave's issue rate, is the limit and the split
// kernel's LDS hand-off is pure overhead.  Each lane streams its own chunk
// with 16-byte loads (dword loads shifted at use when the wave's chunks are
// not all 16-byte aligned), two 128-byte stages (4 blocks) in flight in VGPRs so
// HBM latency under full load stays covered.
template <int RV, typename V>
__device__ __forceinline__ void fused_stage(uint32_t s, uint32_t S, const Entry& en, Stage& cur,
                                            uint32_t (&h)[5]) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap(cur.w[16 * half + j]);
        if (half == 1 && s + 2 < S) load_stage<V>(en.p + 128ull * (s + 2), cur);
        compress<RV>(h, w);
    }
}

// Stages 0 .. S-1 of every lane's chunk, each lane loading its own.
template <int RV, typename V>
__device__ __forceinline__ void fused_lane_stages_v(const Entry& en, uint32_t S, uint32_t (&h)[5]) {
    Stage A0, A1;
    if (S > 0) load_stage<V>(en.p, A0);
    if (S > 1) load_stage<V>(en.p + 128, A1);
    uint32_t s = 0;
    for (; s + 1 < S; s += 2) {
        fused_stage<RV, V>(s, S, en, A0, h);
        fused_stage<RV, V>(s + 1, S, en, A1, h);
    }
    if (s < S) fused_stage<RV, V>(s, S, en, A0, h);
}

// The same for a wave whose chunks are not all 16-byte aligned: dword loads
// (RawSpan, from p & ~3) two stages ahead, funnel-shifted by p & 3 at use.
// Lane-per-chunk byte-unaligned 16-byte loads were slower here (65536 x
// 512 KiB 1..15 bytes off: 13.6 ms against 11.2; profiles/misaligned_r02.json).
template <int RV>
__device__ __forceinline__ void fused_stage_any(uint32_t s, uint32_t S, const Entry& en, RawSpan<32>& cur,
                                                uint32_t (&h)[5]) {
    const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(en.p) & 3u);
    uint32_t w[16];
    shift_raw<32, 0, 16>(cur, sh, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
    compress<RV>(h, w);
    shift_raw<32, 16, 16>(cur, sh, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
    if (s + 2 < S) load_raw<32>(en.p + 128ull * (s + 2), cur);
    compress<RV>(h, w);
}

template <int RV>
__device__ __forceinline__ void fused_lane_stages_any(const Entry& en, uint32_t S, uint32_t (&h)[5]) {
    RawSpan<32> A0, A1;
    if (S > 0) load_raw<32>(en.p, A0);
    if (S > 1) load_raw<32>(en.p + 128, A1);
    uint32_t s = 0;
    for (; s + 1 < S; s += 2) {
        fused_stage_any<RV>(s, S, en, A0, h);
        fused_stage_any<RV>(s + 1, S, en, A1, h);
    }
    if (s < S) fused_stage_any<RV>(s, S, en, A0, h);
}

template <int RV>
__device__ __forceinline__ void fused_lane_stages(const Entry& en, bool valid, uint32_t S, uint32_t (&h)[5]) {
    if (wave_all(!valid || (reinterpret_cast<uintptr_t>(en.p) & 15u) == 0))
        fused_lane_stages_v<RV, uint4>(en, S, h);
    else
        fused_lane_stages_any<RV>(en, S, h);
}

// RV: round-sum form (sha1_device.hpp round_step); the product uses 0, the
// A/B library also builds 1 and 2 (SHA1CHUNK_FUSED_VARIANT).
// The body of one fused wave: message e's lane (group e / 64).
template <int RV>
__device__ __forceinline__ void fused_body(const BatchArgs& A, uint32_t e) {
    const uint32_t group = e / 64u;
    const bool valid = e < A.n;
    Entry en = fetch_entry(A, valid ? e : min(group * 64u, A.n - 1u));
    if (!valid) en.len = 0;
    uint32_t h[5];
    load_init(A, en.id, h);
    const uint32_t S = bulk_stages(en, valid);
    fused_lane_stages<RV>(en, valid, S, h);
    if (valid) {
        lane_blocks(A, en, 2u * S, h);
        emit(A, en.id, h);
    }
}

template <int RV = 0>
__global__ __launch_bounds__(256) void sha1_fused_kernel(BatchArgs A) {
    fused_body<RV>(A, blockIdx.x * 256u + threadIdx.x);
}

// ---------------------------------------------------------- coop fused ----
// The fused wave with its stage loads shared across the wave
// (coop_load / coop_store / coop_read, above the split kernel).  Used by the
// mixed kernel, whose workgroups own the CU's LDS anyway (16 KiB per wave:
// two stage buffers).
template <int RV>
__device__ __forceinline__ void coop_compress(const uint32_t (&cur)[32], uint32_t (&h)[5]) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap(cur[16 * half + j]);
        compress<RV>(h, w);
    }
}

// lds: this wave's kCoopWaveBytes.  Same contract as fused_body.  The
// wave's LDS accesses complete in order, so a stage's stores precede its
// reads and the reads of a buffer precede its next stores; hipcc keeps the
// program order of these lane-dependent accesses it cannot prove disjoint.
// One stage in flight in registers: a second (as fused_body keeps) was
// slower -- hipcc moved its loads next to their LDS stores (65536 x 512 KiB
// 13.1 against 10.4 ms, profiles/coop_split_ab_r02.json).
template <int RV>
__device__ __forceinline__ void fused_coop_body(const BatchArgs& A, uint32_t e, uint8_t* lds) {
    const uint32_t group = e / 64u, lane = e & 63u;
    const bool valid = e < A.n;
    Entry en = fetch_entry(A, valid ? e : min(group * 64u, A.n - 1u));
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
        fused_lane_stages_v<RV, uint4>(en, S, h);
    } else if (S > 0) {  // scattered or not 16-byte aligned: shared loads (any alignment)
        const u32x4u* src[8];
        coop_sources<8>(A, group, lane, src);
        // stage loads run ahead unconditionally (clamped to the last stage:
        // a repeated read at the end, never past a chunk)
        uint32_t v[32];
        coop_load(src, 0, v);
        coop_store(lds, v, lane);
        coop_load(src, min(1u, S - 1u), v);
        for (uint32_t s = 0; s < S; ++s) {
            uint32_t cur[32];
            wave_lds_order();  // stage s stored (previous iteration) -> read
            coop_read(lds + (s & 1u) * kCoopStageBytes, lane, cur);
            wave_lds_order();  // buffer (s+1)&1 was read last iteration -> store
            coop_store(lds + ((s + 1u) & 1u) * kCoopStageBytes, v, lane);
            coop_load(src, min(s + 2u, S - 1u), v);
            coop_compress<RV>(cur, h);
        }
    }
    if (valid) {
        lane_blocks(A, en, 2u * S, h);
        emit(A, en.id, h);
    }
}

// --------------------------------------------------------------- mixed ----
// Ragged batches with more groups of 64 than CUs, sorted longest-first
// (BASELINE config 5's shape beyond 16384 chunks).  A batch of mixed lengths
// ends with its longest chunks' serial chains, so the kernel that has the
// most throughput per CU (fused) is not the one to run them on: at several
// waves per SIMD a fused wave's chain crawls (2.4 us per block at 2 waves
// per SIMD against 0.74 us in the one-group split shape), and a batch of
// log-uniform 4 KiB .. 1 MiB chunks ran 2.5x longer fused than split
// (tools/mixed_bench.py, profiles/mixed_r02.json).  A device-side plan
// (plan_mixed_kernel, from the sorted lengths, no host round trip) splits
// the batch between the shapes; every workgroup of this kernel reserves the
// whole 160 KiB of LDS, so exactly one is resident per CU:
//   mode 0: workgroups 0 .. H-1 hash groups 0 .. H-1 (the longest) one per
//           CU in the one-group split shape (4-block units, two producers,
//           the consumer alone on its SIMD); workgroup H + j hashes groups
//           H + j*F .. H + j*F + F-1 fused, one group per wave (F = 4: one
//           wave per SIMD, chain 1.28 us per block; F = 8: two), each
//           wave loading lane-per-chunk if its chunks lie together and
//           with loads shared across the wave if not (fused_coop_body).
//   mode 1: workgroup w hashes groups 2w, 2w+1 in the 8-wave two-pair split
//           shape (AUTO's shape for C < groups <= 2C on a uniform batch).
// Blocks in dispatch order: the longest groups start first, and the
// hardware dispatcher hands the next workgroup to whichever CU frees up
// (longest-processing-time order).  The grid is one workgroup per group
// (the all-split plan); workgroups past a plan's count exit at once.
//
// Memory locality: with every lane streaming its own chunk, a load
// instruction translates 64 addresses, and when the resident chunks lie far
// apart (a sorted batch whose chunks arrived in random length order) the
// CU's translation cache (UTCL1) thrashes: 98 % misses instead of ~0 on the
// same requests, L2 unchanged (tools/tlb_probe.sh, profiles/tlb_r02.json).
// 65536 x 512 KiB with permuted offsets hashed in 29.2 ms lane-per-chunk
// against 10.4 in place.  Every shape here loads scattered chunks 8 or 16 per
// instruction (see `shared loads`): permuted, the fused tail takes 10.8 ms
// and the one-group split shape 24.3 as in place, so the planner ignores
// layout (profiles/mixed_r02.json, profiles/coop_split_ab_r02.json).
constexpr int kSplit8V = kVWK | kVUnmask | kVLayout8 | kVCross | kVCoop;
constexpr int kMixedThreads = 512;

__global__ __launch_bounds__(kMixedThreads) void sha1_mixed_kernel(BatchArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
    const uint32_t mode = A.plan[0], H = A.plan[1], F = A.plan[2];
    const uint32_t wg = blockIdx.x;
    const uint32_t groups = (A.n + 63u) / 64u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (mode == 1) {
        if (2u * wg >= groups) return;
        split_body<2, 2, kSplit8V, 2>(A, lds, wg);
        return;
    }
    if (wg < H) {
        if (wave >= 4) return;  // the one-group shape is waves 0-3 (wave 2 empty)
        split_body<4, 1, kSplitV<4>, kSplitNProd<4>>(A, lds, wg);
        return;
    }
    const uint32_t g = H + (wg - H) * F + wave;
    if (wave >= F || g >= groups) return;
    fused_coop_body<0>(A, g * 64u + (threadIdx.x & 63u), lds + wave * kCoopWaveBytes);
}

// Persistent-dispatch variant of the mixed kernel (BASELINE config 5 names
// "persistent-kernel dispatch"): one 512-thread
// workgroup per CU (all 160 KiB of LDS each, so one resident per CU) pulls
// the plan's jobs in order from a device counter (plan[3], zeroed by the
// planner on the same stream) until the list is empty.  The job list is the
// plan's: jobs 0 .. H-1 one split group each, then fused jobs of F groups (or
// mode 1: pairs in the 8-wave split shape).  Against the hardware dispatch
// of sha1_mixed_kernel (workgroup i goes to XCD i % 8 and waits for a CU of
// that XCD) any CU that frees takes the next job: one global greedy queue
// instead of eight.  Every wave stays in the loop, so the waves a split job
// does not use pass the same number of workgroup barriers as the job's
// waves (idle_barriers): units + 1 for a split job, plus the two of the
// 8-wave shape's length exchange.
__device__ __forceinline__ uint32_t group_units(const BatchArgs& A, uint32_t group, uint32_t U) {
    const uint32_t e = group * 64u + (threadIdx.x & 63u);
    const bool valid = e < A.n;
    Entry en = fetch_entry(A, valid ? e : min(group * 64u, A.n - 1u));
    const uint32_t T = valid ? total_blocks(en.len) : 0u;
    const uint32_t Tmax = __builtin_amdgcn_readfirstlane(wave_max(T));
    return (Tmax + 2u * U - 1u) / (2u * U) * 2u;
}

__device__ __forceinline__ void idle_barriers(uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) split_barrier();
}

__global__ __launch_bounds__(kMixedThreads) void sha1_mixed_persistent_kernel(BatchArgs A, uint32_t* queue) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
    const uint32_t mode = A.plan[0], H = A.plan[1], F = A.plan[2];
    const uint32_t groups = (A.n + 63u) / 64u;
    const uint32_t jobs = mode == 1 ? (groups + 1u) / 2u : H + (groups - H + F - 1u) / F;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* slot = reinterpret_cast<uint32_t*>(lds);  // free between jobs
    for (;;) {
        if (threadIdx.x == 0) slot[0] = atomicAdd(queue, 1u);
        __syncthreads();
        const uint32_t job = __builtin_amdgcn_readfirstlane(slot[0]);
        __syncthreads();  // every wave has the job before the LDS is reused
        if (job >= jobs) break;
        if (mode == 1) {
            if (wave == 4 || wave == 6) {  // the 8-wave shape's empty waves
                const uint32_t u = max(group_units(A, 2u * job, 2), 2u * job + 1u < groups
                                                                        ? group_units(A, 2u * job + 1u, 2)
                                                                        : 0u);
                idle_barriers(2u + u + 1u);
            } else {
                split_body<2, 2, kSplit8V, 2>(A, lds, job);
            }
        } else if (job < H) {
            if (wave == 0 || wave == 1 || wave == 3)  // the one-group shape (wave 2 empty)
                split_body<4, 1, kSplitV<4>, kSplitNProd<4>>(A, lds, job);
            else
                idle_barriers(group_units(A, job, 4) + 1u);
        } else {
            const uint32_t g = H + (job - H) * F + wave;
            if (wave < F && g < groups) fused_coop_body<0>(A, g * 64u + (threadIdx.x & 63u), lds + wave * kCoopWaveBytes);
        }
    }
}

// ---------------------------------------------------- verify-queue drain ----
// The persistent drain of the received-chunk verify queue (SURVEY 8f rank 2;
// packet_handler.c:469-472 -> job.c:217-228 verify_hash).  One 512-thread
// workgroup per CU loops: lane 0 claims the next published group of <= 64
// chunks (a compare-and-swap on a device counter, below the host's `pub`),
// the workgroup hashes it in the one-group split shape straight out of the
// host ring (coherent pinned memory: every read goes over PCIe, nothing is
// cached), wave 0 compares the 64 digests with the expected ones and
// writes a 0/1 per chunk and the group's completion word to host memory.
// Without work a workgroup sleeps (exponential backoff up to ~50 us) and
// exits once no group has been claimed for `idle_ticks` of 100 MHz time, or
// at once when the host sets `stop`.  Exit handshake (no lost group): the
// workgroup clears its alive word, fences, and re-reads `pub`; the host
// stores `pub`, fences, and reads the alive words.  At least one of them
// sees the other: either the workgroup claims the new group or the host
// launches a new drain.
constexpr uint32_t kVqIdle = 0xffffffffu, kVqExit = 0xfffffffeu;

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Lane 0 only: a claimed group index, kVqIdle or kVqExit.  Idleness is the
// queue's, not the workgroup's: `last` is when the claim counter last moved
// (any workgroup's claim), so under load no workgroup leaves, and after a
// quiet spell the drain's workgroups leave together.
__device__ uint32_t vq_next(const VqDrainArgs& Q, uint64_t& last, uint32_t& seen) {
    for (int round = 0; round < 2; ++round) {
        uint32_t p = ld_sys(Q.pub);
        uint32_t c = __hip_atomic_load(Q.claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c != seen) {
            seen = c;
            last = __builtin_amdgcn_s_memrealtime();
        }
        while (c < p) {
            if (__hip_atomic_compare_exchange_strong(Q.claim, &c, c + 1u, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                seen = c + 1u;
                last = __builtin_amdgcn_s_memrealtime();
                return c;
            }
        }
        if (ld_sys(Q.stop)) return kVqExit;
        if (round == 1 || __builtin_amdgcn_s_memrealtime() - last <= Q.idle_ticks) return kVqIdle;
        // idle too long: leave, unless a group was published meanwhile
        st_sys(Q.alive + blockIdx.x, 0u);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
        if (__hip_atomic_load(Q.claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ld_sys(Q.pub)) return kVqExit;
        st_sys(Q.alive + blockIdx.x, 1u);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
    }
    return kVqIdle;
}

__global__ __launch_bounds__(kMixedThreads) void sha1_vq_drain_kernel(VqDrainArgs Q) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
    uint32_t* slot = reinterpret_cast<uint32_t*>(lds);  // free between jobs
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    uint32_t seen = 0xffffffffu;
    uint32_t backoff = 1;
    for (;;) {
        if (threadIdx.x == 0) slot[0] = vq_next(Q, last, seen);
        __syncthreads();
        const uint32_t g = __builtin_amdgcn_readfirstlane(slot[0]);
        __syncthreads();  // every wave has the command before the LDS is reused
        if (g == kVqExit) break;
        if (g == kVqIdle) {
            for (uint32_t i = 0; i < backoff; ++i) __builtin_amdgcn_s_sleep(127);  // ~3.4 us each
            backoff = min(backoff * 2u, 16u);
            continue;
        }
        backoff = 1;
        const uint32_t gi = g % Q.grp_ring;
        const uint32_t first = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(Q.grp + 2 * gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        const uint32_t count = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(Q.grp + 2 * gi + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        BatchArgs A{};
        A.base = Q.data;
        A.off = Q.off + first;
        A.len = Q.len + first;
        A.n = count;
        A.dig = Q.dig + 20ull * first;
        if (wave == 0 || wave == 1 || wave == 3)  // the one-group split shape (wave 2 empty)
            split_body<4, 1, kSplitV<4>, kSplitNProd<4>>(A, lds, 0);
        else
            idle_barriers(group_units(A, 0, 4) + 1u);
        __syncthreads();
        if (wave == 0) {  // the consumer wave re-reads the digests it wrote
            uint32_t diff = 0;
            if (lane < count) {
                const uint32_t* d = reinterpret_cast<const uint32_t*>(A.dig + 20u * lane);
                const uint32_t* x = reinterpret_cast<const uint32_t*>(Q.exp + 20ull * (first + lane));
#pragma unroll
                for (int i = 0; i < 5; ++i)
                    diff |= d[i] ^ __hip_atomic_load(x + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                Q.res[first + lane] = diff ? 1 : 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (lane == 0) st_sys(Q.done + gi, g + 1u);
        }
    }
}

// Makespan model of a sorted ragged batch, microseconds per 64-byte block of
// a group of 64 chunks, measured on MI355X:
//   chain: time of one group's block when it runs in that shape
//   cu:    CU-time per group-block (the CU's throughput in that shape)
// one-group split: config 2, 6.08 ms / 8193 blocks, one group per CU.
// fused F = 4 (one wave per SIMD): 65536 x 512 KiB, 10.5 ms; F = 8 (two):
// 131072 x 512 KiB, 19.9 ms.  8-wave split: 32768 x 512 KiB, 6.55 ms.
constexpr double kChainSplit4 = 0.742, kCuSplit4 = 0.742;
constexpr double kChainFused4 = 1.28, kCuFused4 = 0.320;
constexpr double kChainFused8 = 2.43, kCuFused8 = 0.304;
constexpr double kChainSplit8 = 0.80, kCuSplit8 = 0.40;

__device__ __forceinline__ uint32_t group_blocks(const uint32_t* sorted_len, uint32_t g) {
    return total_blocks(sorted_len[64ull * g]);  // a group's first lane is its longest
}

// The workgroups of a plan are jobs that the dispatcher starts in index
// order on whichever CU frees first.  Job i of mode 0 (H split groups, then
// fused workgroups of F groups) and of mode 1 (pairs): its duration.
// (blocks: the planner's LDS copy of group_blocks for groups < kSimMaxG)
constexpr uint32_t kSimMaxG = 16384;  // groups whose blocks the planner keeps in LDS

__device__ __forceinline__ uint32_t plan_blocks(const uint32_t* sorted_len, const uint32_t* blocks, uint32_t g) {
    return g < kSimMaxG ? blocks[g] : group_blocks(sorted_len, g);
}

__device__ __forceinline__ double job_time(const uint32_t* sorted_len, const uint32_t* blocks, uint32_t mode,
                                           uint32_t H, uint32_t F, uint32_t i) {
    if (mode == 1) return plan_blocks(sorted_len, blocks, 2u * i) * kChainSplit8;
    if (i < H) return plan_blocks(sorted_len, blocks, i) * kChainSplit4;
    return plan_blocks(sorted_len, blocks, H + (i - H) * F) * (F == 4 ? kChainFused4 : kChainFused8);
}

// Estimated makespan of a plan: the largest of
//   W / C                         total CU-time over C CUs (work bound)
//   p_0, p_H                      the longest split job, the longest fused job
//   (k + 1) p_{kC}, k >= 1        jobs 0 .. kC on C CUs: some CU runs k + 1
//                                 of them back to back (rounds bound; exact
//                                 for equal lengths)
// where W = cu_split4 * P_H + cu_fusedF * (P_G - P_H) in mode 0 and
// cu_split8 * P_G in mode 1 (P_H: blocks of groups 0 .. H-1).
__device__ double makespan(const uint32_t* sorted_len, const uint32_t* blocks, uint32_t G, uint32_t C,
                           uint32_t mode, uint32_t H, uint32_t F, uint64_t PH, uint64_t PG) {
    double W;
    uint32_t J;
    if (mode == 1) {
        W = kCuSplit8 * (double)PG;
        J = (G + 1u) / 2u;
    } else {
        W = kCuSplit4 * (double)PH + (F == 4 ? kCuFused4 : kCuFused8) * (double)(PG - PH);
        J = H + (G - H + F - 1u) / F;
    }
    double m = fmax(W / C, job_time(sorted_len, blocks, mode, H, F, 0));
    if (mode == 0 && H > 0 && H < G) m = fmax(m, job_time(sorted_len, blocks, mode, H, F, H));
    for (uint32_t k = 1; (uint64_t)k * C < J; ++k)
        m = fmax(m, (k + 1) * job_time(sorted_len, blocks, mode, H, F, k * C));
    return m;
}

// The bounds above are lower bounds: with 160 KiB of LDS per workgroup a CU
// runs one job at a time, and a long fused job that a CU picks up late ends
// late (config-5 law at 131072 chunks: bounds 13.0 ms for H = 257, measured
// 17.4, while H = 160 measured 13.8).  So the planner then simulates the
// dispatch of a short list of candidate plans exactly and keeps the
// shortest: workgroup i goes to XCD i % 8 (round-robin), and each XCD starts
// its jobs in index order on whichever of its CUs frees first.  One lane
// per (candidate, XCD) keeps its CUs' free times sorted in 32 registers;
// fp32, restated bit for bit in tests/test_gpu_mixed.py.  Candidates whose
// bounds already exceed the simulated time of the bounds' best plan are not
// simulated.
constexpr uint32_t kSimXcds = 8, kSimCus = 32;      // CUs per XCD the lane tracks at most
constexpr float kChainSplit4f = 0.742f, kChainFused4f = 1.28f, kChainFused8f = 2.43f,
                kChainSplit8f = 0.80f;

__device__ __forceinline__ uint32_t plan_jobs(uint32_t G, uint32_t mode, uint32_t H, uint32_t F) {
    return mode == 1 ? (G + 1u) / 2u : H + (G - H + F - 1u) / F;
}

__device__ __forceinline__ float sim_job(const uint32_t* blocks, uint32_t mode, uint32_t H, uint32_t F,
                                         uint32_t j) {
    if (mode == 1) return (float)blocks[2u * j] * kChainSplit8f;
    if (j < H) return (float)blocks[j] * kChainSplit4f;
    return (float)blocks[H + (j - H) * F] * (F == 4 ? kChainFused4f : kChainFused8f);
}

// Jobs x, x + 8, .. of a plan on one XCD's `per` CUs: the time its last CU
// frees.  t holds the free times in ascending order (+inf past `per`); a
// job starts at t[0] and its end is inserted in order.
__device__ float sim_xcd(const uint32_t* blocks, uint32_t G, uint32_t mode, uint32_t H, uint32_t F,
                         uint32_t x, uint32_t per) {
    float t[kSimCus];
#pragma unroll
    for (uint32_t i = 0; i < kSimCus; ++i) t[i] = i < per ? 0.0f : __builtin_inff();
    const uint32_t J = plan_jobs(G, mode, H, F);
#pragma unroll 4
    for (uint32_t j = x; j < J; j += kSimXcds) {
        const float nx = t[0] + sim_job(blocks, mode, H, F, j);
        // t ascending: the new t[i] is nx clamped to [t[i], t[i+1]]
#pragma unroll
        for (uint32_t i = 0; i + 1 < kSimCus; ++i) t[i] = __builtin_amdgcn_fmed3f(t[i], nx, t[i + 1]);
        t[kSimCus - 1] = fmaxf(t[kSimCus - 1], nx);
    }
    float last = 0.0f;
#pragma unroll
    for (uint32_t i = 0; i < kSimCus; ++i)
        if (i < per) last = fmaxf(last, t[i]);
    return last;
}

// One workgroup, two stages.  Bounds: every mode-0 plan (H in [0, hcap] or
// H = G, F in {4, 8}) gets the makespan bounds above, the smallest wins
// (ties: smaller H).  Simulation (up to kSimMaxG groups on 8 XCDs of <= 32
// CUs): ~80 candidates around it are simulated and the shortest wins, or
// all-split within 0.5 % of it; beyond that, the bounds' plan or mode 1 by
// the same bounds.  The plan depends on the lengths alone: with shared
// loads where the chunks lie no longer changes the choice (see the
// kernel's comment).  forced: write {fmode, fh, ff} as given (tests, A/B).
constexpr int kPlanThreads = 1024;
constexpr uint32_t kPlanMaxH = 4096;  // largest split head the model search considers

__global__ __launch_bounds__(kPlanThreads) void plan_mixed_kernel(BatchArgs A, const uint32_t* sorted_len,
                                                                  uint32_t cus, uint32_t hcap, int forced,
                                                                  uint32_t fmode, uint32_t fh, uint32_t ff,
                                                                  uint32_t* plan) {
    const uint32_t n = A.n;
    const uint32_t t = threadIdx.x;
    if (t == 0) plan[3] = 0u;  // the persistent kernel's job counter
    if (forced) {
        if (t == 0) {
            plan[0] = fmode;
            plan[1] = fh;
            plan[2] = ff;
        }
        return;
    }
    __shared__ uint64_t scan[kPlanThreads];
    __shared__ double best_m[kPlanThreads];
    __shared__ uint32_t best_h[kPlanThreads], best_f[kPlanThreads];
    __shared__ uint64_t prefix[kPlanMaxH + 1];
    const uint32_t G = (n + 63u) / 64u;
    const uint32_t per = (G + kPlanThreads - 1) / kPlanThreads;
    const uint32_t g0 = min(G, t * per), g1 = min(G, g0 + per);
    uint64_t local = 0;
    __shared__ uint32_t blocks[kSimMaxG];  // group_blocks of groups < kSimMaxG, for the simulation
    for (uint32_t g = g0; g < g1; ++g) {
        const uint32_t b = group_blocks(sorted_len, g);
        if (g < kSimMaxG) blocks[g] = b;
        local += b;
    }
    scan[t] = local;
    __syncthreads();
    for (uint32_t off = 1; off < kPlanThreads; off <<= 1) {
        const uint64_t v = t >= off ? scan[t - off] : 0ull;
        __syncthreads();
        scan[t] += v;
        __syncthreads();
    }
    const uint64_t PG = scan[kPlanThreads - 1];
    // P_H for every candidate H <= hcap, then each thread takes H = t, t + 1024, ..
    uint64_t P = scan[t] - local;  // P_{g0}
    for (uint32_t g = g0; g <= g1 && g <= hcap; ++g) {
        prefix[g] = P;
        if (g < g1) P += plan_blocks(sorted_len, blocks, g);
    }
    __syncthreads();
    double bm = 1e300;
    uint32_t bh = 0, bf = 4;
    for (uint32_t H = t; H <= hcap; H += kPlanThreads) {
        for (uint32_t F = 4; F <= (H < G ? 8u : 4u); F += 4) {  // H = G: every group split
            const double m = makespan(sorted_len, blocks, G, cus, 0, H, F, prefix[H], PG);
            if (m < bm) { bm = m; bh = H; bf = F; }
        }
    }
    if (t == 0 && G > hcap) {  // H = G beyond the searched head sizes
        const double m = makespan(sorted_len, blocks, G, cus, 0, G, 4, PG, PG);
        if (m < bm) { bm = m; bh = G; bf = 4; }
    }
    best_m[t] = bm;
    best_h[t] = bh;
    best_f[t] = bf;
    __syncthreads();
    for (uint32_t s = kPlanThreads / 2; s > 0; s >>= 1) {
        if (t < s) {
            const double mo = best_m[t + s];
            const uint32_t ho = best_h[t + s];
            if (mo < best_m[t] || (mo == best_m[t] && ho < best_h[t])) {
                best_m[t] = mo;
                best_h[t] = ho;
                best_f[t] = best_f[t + s];
            }
        }
        __syncthreads();
    }
    const bool simulate = G <= kSimMaxG && cus % kSimXcds == 0 && cus / kSimXcds <= kSimCus;
    if (!simulate) {
        if (t == 0) {
            const bool split8 = makespan(sorted_len, blocks, G, cus, 1, 0, 0, 0, PG) < best_m[0];
            plan[0] = split8 ? 1u : 0u;
            plan[1] = split8 ? 0u : best_h[0];
            plan[2] = split8 ? 0u : best_f[0];
        }
        return;
    }
    // Candidates: the bounds' best plan, the 8-wave mode, all-split, split
    // heads around the bounds' best, and a grid of heads up to 2C (both F).
    constexpr uint32_t kMaxCand = kPlanThreads / kSimXcds;
    __shared__ uint32_t cmode[kMaxCand], chead[kMaxCand], cf[kMaxCand], ncand;
    __shared__ float cmk[kMaxCand];
    if (t == 0) {
        uint32_t k = 0;
        auto add = [&](uint32_t m, uint32_t h, uint32_t f) {
            cmode[k] = m;
            chead[k] = h;
            cf[k] = h == G ? 4u : f;
            ++k;
        };
        const uint32_t hb = best_h[0], fb = best_f[0];
        add(0, hb, fb);
        add(1, 0, 0);
        add(0, G, 4);
        // heads below the bounds' best; only H <= hcap (prefix[] holds P_H
        // there) -- when the best is all-split beyond hcap, hb - d would be
        // neither a searched head nor all-split
        for (uint32_t d = 1; d <= 64; d *= 2) {
            if (hb >= d && hb - d <= hcap) add(0, hb - d, fb);
            if (hb + d <= hcap) add(0, hb + d, fb);
        }
        const uint32_t top = min(hcap, 2u * cus);
        for (uint32_t i = 0; i < 32; ++i) {
            const uint32_t h = i * top / 31u;
            add(0, h, 4);
            if (h < G) add(0, h, 8);
        }
        ncand = k;
    }
    __syncthreads();
    // Pass 1 simulates the bounds' plan; pass 2 every other candidate whose
    // bounds are below that time (the rest cannot beat it; a 4096-group
    // all-split candidate alone is ~100 us of simulation).
    const uint32_t c = t / kSimXcds, x = t % kSimXcds;
    for (uint32_t pass = 0; pass < 2; ++pass) {
        bool run = pass == 0 ? c == 0 : (c >= 1 && c < ncand);
        if (run && pass == 1) {
            const uint32_t m = cmode[c], h = chead[c], f = cf[c];
            const double lb = m == 1 ? makespan(sorted_len, blocks, G, cus, 1, 0, 0, 0, PG)
                                     : makespan(sorted_len, blocks, G, cus, 0, h, f, h <= hcap ? prefix[h] : PG, PG);
            run = lb < (double)cmk[0];
        }
        float mk = __builtin_inff();
        if (run) mk = sim_xcd(blocks, G, cmode[c], chead[c], cf[c], x, cus / kSimXcds);
#pragma unroll
        for (uint32_t m = 1; m < kSimXcds; m *= 2) mk = fmaxf(mk, __shfl_xor(mk, m));
        if (x == 0 && (pass == 0 ? c == 0 : c >= 1)) cmk[c] = mk;
        __syncthreads();
    }
    if (t == 0) {
        uint32_t bi = 0;
        for (uint32_t i = 1; i < ncand; ++i)
            if (cmk[i] < cmk[bi]) bi = i;
        // All-split (candidate 2) within 0.5 % of the best is taken instead:
        // a chain-bound batch then runs with no fused waves heating the chip
        // (65536 chunks of the config-5 law: 12.14 ms all-split against 12.50
        // for a split head + fused tail simulated as equal).
        if (cmk[2] <= cmk[bi] * 1.005f) bi = 2;
        plan[0] = cmode[bi];
        plan[1] = cmode[bi] == 1 ? 0u : chead[bi];
        plan[2] = cmode[bi] == 1 ? 0u : cf[bi];
    }
}

// ------------------------------------------------------------ utilities ---
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// One workgroup per chunk: chunk c (global index first + blockIdx.x) of
// length len is written at dst + off.  dst + off must be 8-byte aligned.
__global__ __launch_bounds__(256) void synth_fill_kernel(uint8_t* dst, const uint64_t* off,
                                                         const uint32_t* lens, uint32_t ulen,
                                                         uint64_t first, uint64_t seed) {
    const uint64_t c = blockIdx.x;
    const uint32_t len = lens ? lens[c] : ulen;
    uint8_t* out = dst + (off ? off[c] : c * (uint64_t)ulen);
    const uint64_t key = seed ^ ((first + c) << 24);
    const uint32_t nw = len >> 3;
    uint64_t* o = reinterpret_cast<uint64_t*>(out);
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) o[w] = splitmix64(key ^ (uint64_t)w);
    const uint32_t rem = len & 7u;
    if (rem && threadIdx.x == 0) {
        const uint64_t v = splitmix64(key ^ (uint64_t)nw);
        for (uint32_t b = 0; b < rem; ++b) out[8ull * nw + b] = (uint8_t)(v >> (8 * b));
    }
}

__global__ __launch_bounds__(256) void compare_kernel(const uint8_t* dig, const uint8_t* exp,
                                                      uint32_t n, uint8_t* mismatch) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t diff = 0;
#pragma unroll
    for (int b = 0; b < 20; ++b) diff |= (uint32_t)(dig[20ull * i + b] ^ exp[20ull * i + b]);
    mismatch[i] = diff ? 1 : 0;
}

// ------------------------------------------------------------ launchers ---
hipError_t launch_lane(const BatchArgs& A, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t grid = (A.n + 255u) / 256u;
    hipLaunchKernelGGL(sha1_lane_kernel, dim3(grid), dim3(256), 0, st, A);
    return hipGetLastError();
}

hipError_t launch_fused(const BatchArgs& A, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
#ifdef SHA1CHUNK_AB_VARIANTS
    if (const char* e = getenv("SHA1CHUNK_FUSED_VARIANT")) {
        const int rv = atoi(e);
        if (rv == 1)
            hipLaunchKernelGGL(sha1_fused_kernel<1>, dim3((A.n + 255u) / 256u), dim3(256), 0, st, A);
        else if (rv == 2)
            hipLaunchKernelGGL(sha1_fused_kernel<2>, dim3((A.n + 255u) / 256u), dim3(256), 0, st, A);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    }
#endif
    hipLaunchKernelGGL(sha1_fused_kernel<0>, dim3((A.n + 255u) / 256u), dim3(256), 0, st, A);
    return hipGetLastError();
}

bool split_unit_built(int u) {
#ifdef SHA1CHUNK_AB_VARIANTS
    static const int built[] = {1,  2,  3,  4,  8,  9,  10, 11, 12, 20, 21, 22, 23, 24, 26, 27,
                                30, 31, 32, 33, 34, 36, 37, 42, 44, 45, 46, 504, 505, 506, 507,
                                569, 577, 578, 579, 580, 581, 13, 583, 584, 585, 86, 87, 590, 14, 15,
                                16, 17, 18, 19};
    for (int b : built)
        if (u == b) return true;
    return false;
#else
    return u == 1 || u == 4 || u == 11;
#endif
}

hipError_t launch_split(const BatchArgs& A, int unit_blocks, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t groups = (A.n + 63u) / 64u;
    switch (unit_blocks) {
    case 1: hipLaunchKernelGGL((sha1_split_kernel<1, 1>), dim3(groups), dim3(128), 0, st, A); break;
    case 4:  // two producers per consumer (kSplitNProd<4>), wave 2 empty: 256 threads
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, kSplitV<4>, kSplitNProd<4>>), dim3(groups),
                           dim3(64 * (1 + kSplitNProd<4>) + ((kSplitV<4> & kVSkipWave2) ? 64 : 0)), 0,
                           st, A);
        break;
    case 11:  // <= 2 groups per CU: 2 pairs x (consumer + 2 producers), 2-block
              // units, 8-wave layout, producer SIMDs crossed between the pairs.
              // Chunks back to back (the uniform layout): lane-per-chunk producer
              // loads -- no TLB thrash to avoid, and the shared loads' LDS
              // transpose adds to this shape's LDS contention (LDS-issue stall
              // 9.8 % of wave time against 1.9 % at one group per CU): 6.33
              // against 6.41 ms at 32768 chunks, steady clock
              // (profiles/shard_ab_r03.json).  Ragged (possibly scattered)
              // chunks keep the shared loads.
        if (A.off == nullptr && A.order == nullptr)
            hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V & ~kVCoop, 2>), dim3((groups + 1) / 2), dim3(512),
                               0, st, A);
        else
            hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V, 2>), dim3((groups + 1) / 2), dim3(512), 0,
                               st, A);
        break;
#ifdef SHA1CHUNK_AB_VARIANTS
    // The shapes and variants of the split-kernel study (profiles/sweep_r01.json,
    // split_variants_r01.json, split_2prod_sweep_r01.json), built only into
    // the A/B library (`make ab` -> build-ab/libsha1chunk.so, selected with
    // SHA1CHUNK_LIB).  The product library holds only what AUTO dispatches:
    // 1.8 instead of 3.3 MiB of code object (start-up measured the same
    // either way, profiles/startup_r02.json).
    case 2: hipLaunchKernelGGL((sha1_split_kernel<2, 1>), dim3(groups), dim3(128), 0, st, A); break;
    case 3: hipLaunchKernelGGL((sha1_split_kernel<3, 1>), dim3(groups), dim3(128), 0, st, A); break;
#define SPLIT_V(U, V)                                                                             \
    case 10 * U + V:                                                                              \
        hipLaunchKernelGGL((sha1_split_kernel<U, 1, V>), dim3(groups), dim3(128), 0, st, A);   \
        break;
    // A/B variants: unit 10*U + V (V = kVWK | kVRtSlot | kVUnmask bits)
    SPLIT_V(3, 0) SPLIT_V(3, 1) SPLIT_V(3, 2) SPLIT_V(3, 3) SPLIT_V(3, 4) SPLIT_V(3, 6)
    SPLIT_V(3, 7) SPLIT_V(2, 0) SPLIT_V(2, 1) SPLIT_V(2, 2) SPLIT_V(2, 3) SPLIT_V(2, 4) SPLIT_V(2, 6)
    SPLIT_V(2, 7) SPLIT_V(4, 2) SPLIT_V(4, 4) SPLIT_V(4, 5) SPLIT_V(4, 6)
#undef SPLIT_V
#define SPLIT_2P(V)                                                                               \
    case 500 + V:                                                                                 \
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, V, 2>), dim3(groups), dim3(192), 0, st, A);   \
        break;
    // two producer waves per consumer, 4-block units: unit 500 + V
    SPLIT_2P(4) SPLIT_2P(5) SPLIT_2P(6) SPLIT_2P(7)
#undef SPLIT_2P
    case 569:  // 500 + (kVWK | kVUnmask | kVSkipWave2): producers on waves 1 and 3
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, 69, 2>), dim3(groups), dim3(256), 0, st, A);
        break;
    case 578:  // 577 with wave 1 empty (producers on waves 2 and 3), A/B
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, 77 | kVSkipWave1, 2>), dim3(groups), dim3(256), 0, st, A);
        break;
    case 577:  // 569 + kVRead10
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, 77, 2>), dim3(groups), dim3(256), 0, st, A);
        break;
    case 579:  // 577 + consumer at s_setprio 3
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, 77 | kVPrio, 2>), dim3(groups), dim3(256), 0, st, A);
        break;
    case 580:  // 577 with all 20 reads in one burst
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, (77 & ~kVRead10) | kVRead20, 2>), dim3(groups),
                           dim3(256), 0, st, A);
        break;
    case 581:  // 580 + s_setprio 3
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, (77 & ~kVRead10) | kVRead20 | kVPrio, 2>),
                           dim3(groups), dim3(256), 0, st, A);
        break;

    case 583:  // the product's case 4 (77 | kVCoop) + consumer at s_setprio 3
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, 77 | kVCoop | kVPrio, 2>), dim3(groups), dim3(256), 0, st, A);
        break;
    case 584:  // the product's case 4 with all 20 schedule reads in one burst
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, (77 & ~kVRead10) | kVRead20 | kVCoop, 2>), dim3(groups),
                           dim3(256), 0, st, A);
        break;
    case 585:  // the product's case 4 with schedule reads in four bursts of 5
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, (77 & ~kVRead10) | kVCoop, 2>), dim3(groups), dim3(256), 0,
                           st, A);
        break;
    case 14:  // case 11 with the consumers at s_setprio 3 (round-3 A/B: LDS issue contention)
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V | kVPrio, 2>), dim3((groups + 1) / 2), dim3(512), 0,
                           st, A);
        break;
    case 15:  // case 13 with the consumers at s_setprio 3
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVPrio, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    case 13:  // case 11 with lane-per-chunk producer loads (round-2 A/B of kVCoop)
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V & ~kVCoop, 2>), dim3((groups + 1) / 2), dim3(512), 0,
                           st, A);
        break;

    // Round-3 A/B: one pair per workgroup with 2-block units and two producers
    // (one block each per unit; waves 0, 1, 3 as in case 4): the config-2
    // layout with case 11's unit size and 80 KiB of LDS.  Separates the cost
    // of barriers every 2 blocks from that of two pairs sharing a CU.
    case 16:
        hipLaunchKernelGGL((sha1_split_kernel<2, 1, kVWK | kVUnmask | kVSkipWave2 | kVRead10 | kVCoop, 2>),
                           dim3(groups), dim3(256), 0, st, A);
        break;
    case 17:  // case 16 with lane-per-chunk producer loads
        hipLaunchKernelGGL((sha1_split_kernel<2, 1, kVWK | kVUnmask | kVSkipWave2 | kVRead10, 2>), dim3(groups),
                           dim3(256), 0, st, A);
        break;

    // Round-3 A/B of the LDS store-path halves (kVHalves), lane-per-chunk
    // producer loads as in the product's uniform case 11 (= case 13)
    case 18:  // each consumer's producers on the other half
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~kVCoop) | kVHalves, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    case 19:  // each consumer's producers on its own half
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, (kSplit8V & ~(kVCoop | kVCross)) | kVHalves, 2>),
                           dim3((groups + 1) / 2), dim3(512), 0, st, A);
        break;

    case 8:  // 4 pairs per workgroup (512 threads), one consumer + producer per SIMD
        hipLaunchKernelGGL((sha1_split_kernel<1, 4>), dim3((groups + 3) / 4), dim3(512), 0, st, A);
        break;
    case 590: {  // the product's case 4 with the W+K ring in global memory (kVGlobalW)
        static uint8_t* wring = nullptr;
        static size_t wcap = 0;
        const size_t need = (size_t)groups * 2 * 4 * kWBlockBytes;
        if (need > 0x7fffffffu) return hipErrorInvalidValue;
        if (need > wcap) {
            if (wring) (void)hipFree(wring);
            wring = nullptr;
            wcap = 0;
            hipError_t e = hipMalloc(&wring, need);
            if (e != hipSuccess) return e;
            wcap = need;
        }
        hipLaunchKernelGGL((sha1_split_gw_kernel<kSplitV<4> | kVGlobalW>), dim3(groups), dim3(256), 0, st, A, wring);
        break;
    }
    case 86:  // case 8 with shared producer loads (4 groups per CU, A/B vs fused)
        hipLaunchKernelGGL((sha1_split_kernel<1, 4, kVWK | kVUnmask | kVCoop>), dim3((groups + 3) / 4), dim3(512),
                           0, st, A);
        break;
    case 87:  // case 86 with K added in the consumer (cheaper producer)
        hipLaunchKernelGGL((sha1_split_kernel<1, 4, kVUnmask | kVCoop>), dim3((groups + 3) / 4), dim3(512), 0,
                           st, A);
        break;
    case 10:  // 2 pairs x (consumer + 2 producers), 2-block units, 8-wave layout
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kVWK | kVUnmask | kVLayout8, 2>), dim3((groups + 1) / 2),
                           dim3(512), 0, st, A);
        break;
    case 12:  // case 10 with schedule reads in bursts of 10
        hipLaunchKernelGGL((sha1_split_kernel<2, 2, kVWK | kVUnmask | kVLayout8 | kVRead10, 2>),
                           dim3((groups + 1) / 2), dim3(512), 0, st, A);
        break;
    case 9:  // 2 pairs per workgroup, 2-block units
        hipLaunchKernelGGL((sha1_split_kernel<2, 2>), dim3((groups + 1) / 2), dim3(256), 0, st, A);
        break;
#endif
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

uint32_t mixed_grid(uint32_t groups, int cus, uint32_t* hcap) {
    *hcap = std::min<uint32_t>(std::min<uint32_t>(groups, 4u * (uint32_t)cus), kPlanMaxH);
    // the largest workgroup count of any plan: every group split (H = G)
    return groups;
}

hipError_t launch_mixed(const BatchArgs& A, const uint32_t* sorted_len, uint32_t* plan, int cus,
                        const int* forced, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t groups = (A.n + 63u) / 64u;
    uint32_t hcap;
    const uint32_t grid = mixed_grid(groups, cus, &hcap);
    hipLaunchKernelGGL(plan_mixed_kernel, dim3(1), dim3(kPlanThreads), 0, st, A, sorted_len,
                       (uint32_t)cus, hcap, forced ? 1 : 0, forced ? (uint32_t)forced[0] : 0u,
                       forced ? (uint32_t)forced[1] : 0u, forced ? (uint32_t)forced[2] : 0u, plan);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    BatchArgs B = A;
    B.plan = plan;
    // Default: the persistent work-queue variant (one workgroup per CU
    // pulling the plan's jobs).  SHA1CHUNK_MIXED_DISPATCH=hw launches one
    // workgroup per job instead (the hardware dispatcher's order).  The two
    // measure the same plan for plan: geometric mean 0.999, -2.8 .. +1.8 %
    // over 92 (plan, size, layout) points (profiles/mixed_dispatch_ab_r03.json).
    const char* disp = getenv("SHA1CHUNK_MIXED_DISPATCH");
    const bool persistent = !(disp && !strcmp(disp, "hw"));
    if (persistent)
        hipLaunchKernelGGL(sha1_mixed_persistent_kernel, dim3((uint32_t)cus), dim3(kMixedThreads), 0, st, B,
                           plan + 3);
    else
        hipLaunchKernelGGL(sha1_mixed_kernel, dim3(grid), dim3(kMixedThreads), 0, st, B);
    return hipGetLastError();
}

hipError_t launch_vq_drain(const VqDrainArgs& Q, uint32_t grid, hipStream_t st) {
    hipLaunchKernelGGL(sha1_vq_drain_kernel, dim3(grid), dim3(kMixedThreads), 0, st, Q);
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* dst, const uint64_t* off, const uint32_t* lens, uint32_t ulen,
                        uint64_t first, uint64_t count, uint64_t seed, hipStream_t st) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_fill_kernel, dim3((uint32_t)count), dim3(256), 0, st, dst, off, lens,
                       ulen, first, seed);
    return hipGetLastError();
}

hipError_t launch_compare(const uint8_t* dig, const uint8_t* exp, uint32_t n, uint8_t* mismatch,
                          hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(compare_kernel, dim3((n + 255u) / 256u), dim3(256), 0, st, dig, exp, n,
                       mismatch);
    return hipGetLastError();
}
