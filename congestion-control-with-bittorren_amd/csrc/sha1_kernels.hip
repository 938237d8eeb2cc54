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
//   sha1_fused_kernel  one wave per 64 chunks; the wave pulls 128 contiguous
//                      bytes of each chunk per stage with global_load_lds
//                      (16 B/lane, 8 lanes per chunk = whole 128-B lines)
//                      into an XOR-swizzled LDS ring, each lane reads its
//                      own row back conflict-free; schedule + rounds in VGPRs.
//   sha1_split_kernel  workgroup = producer wave + consumer wave on the same
//                      64 chunks.  The producer streams the blocks (same LDS
//                      ring), byte-swaps and expands the 80-word schedule into
//                      an LDS W-ring; the consumer runs only the 80 rounds.
//                      This halves the serial instruction stream per chunk
//                      when there are too few chunks to fill the SIMDs
//                      (BASELINE config 2: 4096 chunks = 64 waves).
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

// Blocks [k0, nfull) of one lane straight from global memory, then the
// padded tail (unless the batch is in update mode).
__device__ __forceinline__ void lane_blocks(const BatchArgs& A, const Entry& en, uint32_t k0,
                                            uint32_t (&h)[5]) {
    const uint32_t nfull = en.len >> 6;
    uint32_t cur[16], nxt[16];
    if (k0 < nfull) load_block_full(en.p + 64ull * k0, cur);
    for (uint32_t k = k0; k < nfull; ++k) {
        if (k + 1 < nfull) load_block_full(en.p + 64ull * (k + 1), nxt);
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap(cur[j]);
        compress(h, w);
#pragma unroll
        for (int j = 0; j < 16; ++j) cur[j] = nxt[j];
    }
    if (!A.out_state)
        finish_message(h, en.p + 64ull * nfull, en.len & 63u, A.prefix_bytes + en.len);
}

// ------------------------------------------------------------------------
// LDS raw-block ring shared by the fused kernel and the split producer.
// One stage = 2 blocks (128 B) of each of the wave's 64 chunks = 8 KiB,
// written by 8 global_load_lds_dwordx4: instruction i covers rows 8i..8i+7,
// lane l fetches row 8i+(l>>3), 16-B segment q = (l&7) ^ ((row>>1)&7) and
// lands at ring + i*1024 + l*16 = row*128 + (l&7)*16.  Lane r reads its row
// segment q at row*128 + (q ^ ((r>>1)&7))*16: every 16-lane group of a
// ds_read_b128 then hits 16 distinct 16-B bank slots (conflict-free).
// ------------------------------------------------------------------------
constexpr int kStageBytes = 8192;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

struct RawRing {
    const uint8_t* src[8];  // per-lane source for instruction i, stage 0
    uint32_t swz;           // this lane's read swizzle ((lane>>1)&7)

    __device__ __forceinline__ void setup(const uint8_t* my_p, int lane) {
        const uint64_t mine = reinterpret_cast<uint64_t>(my_p);
        const uint32_t lo = static_cast<uint32_t>(mine), hi = static_cast<uint32_t>(mine >> 32);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = 8 * i + (lane >> 3);
            const uint32_t rlo = __shfl(lo, row), rhi = __shfl(hi, row);
            const uint32_t q = (uint32_t)(lane & 7) ^ (uint32_t)((row >> 1) & 7);
            src[i] = reinterpret_cast<const uint8_t*>(((uint64_t)rhi << 32) | rlo) + 16u * q;
        }
        swz = (uint32_t)((lane >> 1) & 7);
    }

    // The 8 LDS-DMA loads of one stage.  Issued from inline asm so that hipcc
    // does not see them: otherwise it drains vmcnt(0) before every ds_read of
    // the ring and the prefetch never overlaps compute.  Completion is
    // tracked by hand with wait_stages().  M0 (the DMA's LDS base) is set
    // and restored inside the statement.
    __device__ __forceinline__ void issue(uint32_t ring_lds, int buf, uint32_t stage) const {
        const uint32_t dst = __builtin_amdgcn_readfirstlane(ring_lds + (uint32_t)buf * kStageBytes);
        const uint64_t step = 128ull * stage;
        const uint8_t* p0 = src[0] + step;
        const uint8_t* p1 = src[1] + step;
        const uint8_t* p2 = src[2] + step;
        const uint8_t* p3 = src[3] + step;
        const uint8_t* p4 = src[4] + step;
        const uint8_t* p5 = src[5] + step;
        const uint8_t* p6 = src[6] + step;
        const uint8_t* p7 = src[7] + step;
        uint32_t keep, m;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %10\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %2, off\n\t"
            "s_add_u32 %1, %10, 0x400\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %3, off\n\t"
            "s_add_u32 %1, %10, 0x800\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %4, off\n\t"
            "s_add_u32 %1, %10, 0xc00\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %5, off\n\t"
            "s_add_u32 %1, %10, 0x1000\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %6, off\n\t"
            "s_add_u32 %1, %10, 0x1400\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %7, off\n\t"
            "s_add_u32 %1, %10, 0x1800\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %8, off\n\t"
            "s_add_u32 %1, %10, 0x1c00\n\t"
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %9, off\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep), "=&s"(m)
            : "v"(p0), "v"(p1), "v"(p2), "v"(p3), "v"(p4), "v"(p5), "v"(p6), "v"(p7), "s"(dst)
            : "memory", "scc");
    }

    // Little-endian words of block `half` (0/1) of the stage in buffer buf.
    __device__ __forceinline__ void read(const uint8_t* ring, int buf, int half, int lane,
                                         uint32_t (&w)[16]) const {
        const uint8_t* row = ring + buf * kStageBytes + lane * 128;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t q = (uint32_t)(4 * half + j) ^ swz;
            const uint4 x = *reinterpret_cast<const uint4*>(row + 16u * q);
            w[4 * j + 0] = x.x;
            w[4 * j + 1] = x.y;
            w[4 * j + 2] = x.z;
            w[4 * j + 3] = x.w;
        }
    }
};

// Wait until at most `ahead` stages (8 LDS-DMA each) are still in flight.
__device__ __forceinline__ void wait_stages(int ahead) {
    if (ahead >= 2)
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

// Per-wave setup common to the fused kernel and the split producer/consumer.
struct WaveChunks {
    Entry en;
    bool valid;
    uint32_t bulk;  // wave-uniform number of LDS-staged stages (2 blocks each)
};

__device__ __forceinline__ WaveChunks wave_setup(const BatchArgs& A, uint32_t group, int lane) {
    WaveChunks c;
    const uint32_t e = group * 64u + (uint32_t)lane;
    c.valid = e < A.n;
    c.en = fetch_entry(A, c.valid ? e : group * 64u);
    if (!c.valid) c.en.len = 0;
    const bool aligned = (reinterpret_cast<uintptr_t>(c.en.p) & 15u) == 0;
    const uint32_t stages = c.valid ? (c.en.len >> 7) : 0xffffffffu;
    uint32_t bulk = wave_min(stages);
    const uint64_t misaligned = __ballot(c.valid && !aligned);
    if (misaligned) bulk = 0;
    c.bulk = __builtin_amdgcn_readfirstlane(bulk);
    return c;
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

// --------------------------------------------------------------- fused ----
template <int STAGES>
__global__ __launch_bounds__(64) void sha1_fused_kernel(BatchArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[STAGES * kStageBytes];
    const int lane = threadIdx.x;
    const WaveChunks c = wave_setup(A, blockIdx.x, lane);
    uint32_t h[5];
    init_state(h);

    const uint32_t S = c.bulk;
    if (S > 0) {
        RawRing rr;
        rr.setup(c.en.p, lane);
#pragma unroll
        for (int s = 0; s < STAGES - 1; ++s)
            if ((uint32_t)s < S) rr.issue(lds_addr(ring), s, s);
        int buf = 0;
        for (uint32_t s = 0; s < S; ++s) {
            const uint32_t pre = s + STAGES - 1;
            if (pre < S) {
                int pbuf = buf + STAGES - 1;
                if (pbuf >= STAGES) pbuf -= STAGES;
                rr.issue(lds_addr(ring), pbuf, pre);
            }
            const uint32_t left = S - 1 - s;
            wait_stages(left < (uint32_t)(STAGES - 1) ? (int)left : STAGES - 1);
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                uint32_t w[16];
                rr.read(ring, buf, half, lane, w);
#pragma unroll
                for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
                compress(h, w);
            }
            // The next issue overwrites this buffer: keep its reads ahead.
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (++buf == STAGES) buf = 0;
        }
    }
    if (c.valid) {
        lane_blocks(A, c.en, 2u * S, h);
        emit(A, c.en.id, h);
    }
}

// --------------------------------------------------------------- split ----
// LDS: raw ring (producer only) + 2-slot W ring.  W slot layout: group q of
// four schedule words (q = 0..19) of lane r at q*1024 + r*16, so both the
// producer's ds_write_b128 and the consumer's ds_read_b128 touch one
// contiguous KiB per instruction (conflict-free).
constexpr int kSplitRaw = 3;
constexpr int kWSlotBytes = 20 * 1024;

__device__ __forceinline__ void split_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Producer: fill the schedule of block k into W slot `slot`.
template <int T>
struct SchedWrite {
    __device__ __forceinline__ static void run(uint32_t (&w)[16], uint8_t* slot, int lane) {
        if constexpr (T >= 16) sched_step<T>(w);
        if constexpr ((T & 3) == 3) {
            constexpr int j = (T - 3) & 15;
            *reinterpret_cast<uint4*>(slot + (T >> 2) * 1024 + lane * 16) =
                make_uint4(w[j], w[j + 1], w[j + 2], w[j + 3]);
        }
        SchedWrite<T + 1>::run(w, slot, lane);
    }
};
template <>
struct SchedWrite<80> {
    __device__ __forceinline__ static void run(uint32_t (&)[16], uint8_t*, int) {}
};

__device__ __forceinline__ uint32_t total_blocks(uint32_t len) {
    // nfull data blocks + 1 padded block (+1 more when len % 64 >= 56)
    return (len >> 6) + (((len & 63u) < 56u) ? 1u : 2u);
}

__global__ __launch_bounds__(128) void sha1_split_kernel(BatchArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kSplitRaw * kStageBytes + 2 * kWSlotBytes];
    uint8_t* ring = lds;
    uint8_t* wring = lds + kSplitRaw * kStageBytes;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const WaveChunks c = wave_setup(A, blockIdx.x, lane);
    const uint32_t T = c.valid ? total_blocks(c.en.len) : 0u;
    const uint32_t Tmax = __builtin_amdgcn_readfirstlane(wave_max(T));
    const uint32_t S = c.bulk;

    if (wave == 1) {
        // ----------------------------- producer -------------------------
        RawRing rr;
        if (S > 0) {
            rr.setup(c.en.p, lane);
#pragma unroll
            for (int s = 0; s < kSplitRaw - 1; ++s)
                if ((uint32_t)s < S) rr.issue(lds_addr(ring), s, s);
        }
        const uint32_t nfull = c.en.len >> 6, rem = c.en.len & 63u;
        const uint64_t bits = (uint64_t)c.en.len * 8ull;
        int buf = 0;
        for (uint32_t k = 0; k < Tmax; ++k) {
            uint32_t w[16];
            if (k < 2u * S) {
                const uint32_t s = k >> 1;
                const int half = (int)(k & 1u);
                if (half == 0) {
                    const uint32_t pre = s + kSplitRaw - 1;
                    if (pre < S) {
                        int pbuf = buf + kSplitRaw - 1;
                        if (pbuf >= kSplitRaw) pbuf -= kSplitRaw;
                        rr.issue(lds_addr(ring), pbuf, pre);
                    }
                    const uint32_t left = S - 1 - s;
                    wait_stages(left < (uint32_t)(kSplitRaw - 1) ? (int)left : kSplitRaw - 1);
                }
                rr.read(ring, buf, half, lane, w);
#pragma unroll
                for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
                if (half == 1 && ++buf == kSplitRaw) buf = 0;
            } else if (k < nfull) {
                load_block_full(c.en.p + 64ull * k, w);
#pragma unroll
                for (int j = 0; j < 16; ++j) w[j] = bswap(w[j]);
            } else if (k == nfull) {
                if (rem) {
                    load_block_partial(c.en.p + 64ull * k, rem, w);
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
            SchedWrite<0>::run(w, wring + (k & 1u) * kWSlotBytes, lane);
            split_barrier();
        }
    } else {
        // ----------------------------- consumer -------------------------
        uint32_t h[5];
        init_state(h);
        for (uint32_t k = 0; k < Tmax; ++k) {
            split_barrier();
            const uint8_t* slot = wring + (k & 1u) * kWSlotBytes + lane * 16;
            uint32_t W[80];
#pragma unroll
            for (int q = 0; q < 20; ++q) {
                const uint4 x = *reinterpret_cast<const uint4*>(slot + q * 1024);
                W[4 * q + 0] = x.x;
                W[4 * q + 1] = x.y;
                W[4 * q + 2] = x.z;
                W[4 * q + 3] = x.w;
            }
            uint32_t v[5] = {h[0], h[1], h[2], h[3], h[4]};
            RoundsW<0>::run(v, W);
            const bool live = k < T;
#pragma unroll
            for (int i = 0; i < 5; ++i) h[i] = live ? h[i] + v[i] : h[i];
        }
        if (c.valid) emit(A, c.en.id, h);
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
    const uint32_t groups = (A.n + 63u) / 64u;
    hipLaunchKernelGGL(sha1_fused_kernel<2>, dim3(groups), dim3(64), 0, st, A);
    return hipGetLastError();
}

hipError_t launch_split(const BatchArgs& A, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t groups = (A.n + 63u) / 64u;
    hipLaunchKernelGGL(sha1_split_kernel, dim3(groups), dim3(128), 0, st, A);
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
