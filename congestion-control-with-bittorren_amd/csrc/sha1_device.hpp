// sha1_device.hpp -- SHA-1 compression for gfx950 (CDNA4), device side.
//
// What the reference computes (file:line in /root/reference):
//   SHA1Guts      sha.c:176-451  one compression of a 64-byte block
//     BE load     sha.c:186-189  W[0..15] = byte-swapped input words
//     schedule    sha.c:191-200  W[t] = ROTL1(W[t-3]^W[t-8]^W[t-14]^W[t-16])
//     rounds      sha.c:57-69    temp = ROTL5(a)+F(b,c,d)+e+W+K, c = ROTL30(b)
//     feed-fwd    sha.c:446-450  hash[i] += a..e
//   SHA1Final     sha.c:529-558  0x80 pad to 56 mod 64, 64-bit BE bit count
//
// How it maps to CDNA4 (one SHA-1 message per lane; 64 messages per wave):
//   rotate            -> v_alignbit_b32 (1 op)
//   Ch/Parity/Maj     -> v_bitop3_b32 (one op each)
//   5-term round sum  -> 2 x v_add3_u32 (split consumer: v_add + v_add3)
//   schedule xor4     -> v_bitop3_b32(xor3) + v_xor_b32, then v_alignbit_b32
//   byte swap         -> v_perm_b32
// = ~613 VALU per 64-byte block, no MFMA, no LDS inside the compression.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace s1 {

constexpr uint32_t K0 = 0x5a827999u, K1 = 0x6ed9eba1u, K2 = 0x8f1bbcdcu, K3 = 0xca62c1d6u;
constexpr uint32_t IV0 = 0x67452301u, IV1 = 0xefcdab89u, IV2 = 0x98badcfeu, IV3 = 0x10325476u,
                   IV4 = 0xc3d2e1f0u;

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t s) {
    return __builtin_amdgcn_alignbit(x, x, 32u - s);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
// Ch = b ? c : d.  Written as d ^ (b & (c ^ d)), which hipcc folds into one
// v_bitop3_b32 in every shipped kernel (profiles/isa_mix_r02.json: 80
// bitop3 per block in the consumer, no v_bfi).  Round 1 measured forcing the
// bitop3 through the builtin 3% slower in the consumer, because of where
// hipcc then scheduled it (profiles/ch_bitop3_ab_r01.json); this form lets
// the compiler place it.
__device__ __forceinline__ uint32_t chf(uint32_t b, uint32_t c, uint32_t d) {
    return d ^ (b & (c ^ d));
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
// The same byte swap (one v_perm_b32), its result forced into a register
// other than its source's.  For a prefetched stage that is swapped into the
// schedule window and then refilled by the next load: with bswap() hipcc
// swaps the stage's second half in place and keeps those registers as the
// window through the compression, so the refill lands elsewhere and is
// copied back once per trip (8 v_mov_b64 per block in the fused loop); here
// the stage registers die at the swap and the refill targets them directly
// (621.75 -> 613.75 VALU per block, profiles/fused_vmov_r04.json).
__device__ __forceinline__ uint32_t bswap_fresh(uint32_t x) {
    uint32_t r;
    asm("v_perm_b32 %0, %1, %1, %2" : "=&v"(r) : "v"(x), "s"(0x00010203u));
    return r;
}

// Round t (compile-time after unrolling) over the five-word state v[], kept
// in place: a = v[(0-t)%5] ... e = v[(4-t)%5]; the new a lands in e's slot
// and b is rotated in its own slot, so no register moves are emitted.
template <int T>
__device__ __forceinline__ constexpr uint32_t round_k() {
    return T < 20 ? K0 : T < 40 ? K1 : T < 60 ? K2 : K3;
}

// WK = true: wt already holds W[t] + K[t] (the split producer adds it), so
// e + W + K is a 2-operand v_add_u32 (VOP2, issues ~6% faster than VOP3).
// (The fused kernel keeps the two v_add3_u32: forms with every sum as a VOP2
// add were measured no faster, profiles/fused_roundsum_ab_r02.json; their
// code left the source in round 4.)
template <int T, bool WK = false>
__device__ __forceinline__ void round_step(uint32_t (&v)[5], uint32_t wt) {
    constexpr int ia = (5 - (T % 5)) % 5;
    constexpr int ib = (ia + 1) % 5, ic = (ia + 2) % 5, id = (ia + 3) % 5, ie = (ia + 4) % 5;
    uint32_t f;
    if constexpr (T < 20)
        f = chf(v[ib], v[ic], v[id]);
    else if constexpr (T < 40)
        f = xor3(v[ib], v[ic], v[id]);
    else if constexpr (T < 60)
        f = maj(v[ib], v[ic], v[id]);
    else
        f = xor3(v[ib], v[ic], v[id]);
    // temp = ROTL5(a) + F + e + K + W.  e + K + W does not depend on a, so it
    // is summed first, off the chain; the chain a -> {ROTL5(a), F} -> add3
    // is then 2 dependent VALU ops per round instead of 3.  The add3 is
    // pinned in asm because LLVM otherwise re-associates the 5-term sum as
    // (e + ROTL5(a) + F) + (W + K), putting both adds on the chain.
    uint32_t x;
    if constexpr (WK)
        x = v[ie] + wt;
    else
        x = v[ie] + wt + round_k<T>();
    uint32_t t;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(t) : "v"(rotl(v[ia], 5)), "v"(f), "v"(x));
    v[ie] = t;
    v[ib] = rotl(v[ib], 30);
}

// In-place 16-word window expansion for round T >= 16.
template <int T>
__device__ __forceinline__ uint32_t sched_step(uint32_t (&w)[16]) {
    uint32_t x = rotl(xor3(w[(T - 3) & 15], w[(T - 8) & 15], w[(T - 14) & 15]) ^ w[T & 15], 1);
    w[T & 15] = x;
    return x;
}

template <int T>
struct Rounds {
    __device__ __forceinline__ static void run(uint32_t (&v)[5], uint32_t (&w)[16]) {
        if constexpr (T < 80) {
            uint32_t wt;
            if constexpr (T < 16)
                wt = w[T];
            else
                wt = sched_step<T>(w);
            round_step<T, false>(v, wt);
            Rounds<T + 1>::run(v, w);
        }
    }
};

// One full compression: h[] <- h[] + F(h[], w[]); w[] holds the block as
// big-endian words and is consumed (overwritten by the schedule).
__device__ __forceinline__ void compress(uint32_t (&h)[5], uint32_t (&w)[16]) {
    uint32_t v[5] = {h[0], h[1], h[2], h[3], h[4]};
    Rounds<0>::run(v, w);
#pragma unroll
    for (int i = 0; i < 5; ++i) h[i] += v[i];
}

// Rounds only, with W[t] + K[t] supplied in registers (split kernel
// consumer: the producer wave computed the schedule and added K).
template <int T, int END = 80, bool WK = true>
struct RoundsW {
    __device__ __forceinline__ static void run(uint32_t (&v)[5], const uint32_t (&W)[80]) {
        if constexpr (T < END) {
            round_step<T, WK>(v, W[T]);
            RoundsW<T + 1, END, WK>::run(v, W);
        }
    }
};

// Padding of the final partial block (sha.c:536-543): word i of the block
// holds message bytes [4i, 4i+4) as a big-endian word; keep the first
// `rem` bytes of the block, put 0x80 right after them, zero the rest.
__device__ __forceinline__ uint32_t pad_word(uint32_t w, int i, int rem) {
    const int valid = rem - 4 * i;  // message bytes of this word still in the block
    if (valid >= 4) return w;
    if (valid < 0) return 0u;
    const uint32_t keep = valid == 0 ? 0u : (0xffffffffu << (32 - 8 * valid));
    return (w & keep) | (0x80000000u >> (8 * valid));
}

__device__ __forceinline__ void init_state(uint32_t (&h)[5]) {
    h[0] = IV0;
    h[1] = IV1;
    h[2] = IV2;
    h[3] = IV3;
    h[4] = IV4;
}

// ---------------------------------------------------------------------------
// Per-lane loads from global memory (any byte alignment).  `p` points at the
// first byte of the block, `avail` is how many message bytes remain from p
// (>= 64 for a full block).  Reads never touch a 4-byte word that holds no
// message byte, so they never cross into an unmapped page.  Output: the
// block's words as LITTLE-endian loads (byte-swap is done by the caller).
// ---------------------------------------------------------------------------
// A full block: 4 x global_load_dwordx4 of exactly its 64 bytes, no
// branches (so hipcc can count the loads with a partial vmcnt when they are
// prefetched), at any byte alignment: gfx950 under ROCm runs in unaligned
// access mode (hipcc emits global_load_dwordx4 for this align-1 type, and
// byte-unaligned loads read correctly on MI355X), so a chunk's bulk loads
// need not care where it starts.
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

__device__ __forceinline__ void load_block16(const uint8_t* p, uint32_t (&w)[16]) {
    const u32x4u* q = reinterpret_cast<const u32x4u*>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u32x4u x = q[j];
        w[4 * j + 0] = x.x;
        w[4 * j + 1] = x.y;
        w[4 * j + 2] = x.z;
        w[4 * j + 3] = x.w;
    }
}

// K dwords from any byte alignment, loaded raw now and shifted at use (so a
// prefetch does not wait for its loads): d holds the K + 1 dwords from
// p & ~3 (the last only when p is not 4-byte aligned; it then holds at
// least one byte of the span, so it never crosses into another page), and
// word j is alignbyte(d[j+1], d[j], p & 3).
template <int K>
struct RawSpan {
    uint32_t d[K + 1];
};

template <int K>
__device__ __forceinline__ void load_raw(const uint8_t* p, RawSpan<K>& r) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
#pragma unroll
    for (int j = 0; j < K; ++j) r.d[j] = q[j];
    r.d[K] = (a & 3u) ? q[K] : 0u;
}

template <int K, int J0 = 0, int N = K>
__device__ __forceinline__ void shift_raw(const RawSpan<K>& r, uint32_t sh, uint32_t (&w)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) w[j] = __builtin_amdgcn_alignbyte(r.d[J0 + j + 1], r.d[J0 + j], sh);
}

__device__ __forceinline__ void load_block_partial(const uint8_t* p, uint32_t avail,
                                                   uint32_t (&w)[16]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t sh = static_cast<uint32_t>(a & 3u);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t span = avail + sh;  // bytes from the aligned base to the message end
    uint32_t d[17];
#pragma unroll
    for (int j = 0; j < 17; ++j) d[j] = (uint32_t)(4 * j) < span ? q[j] : 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
}

// Final block(s) of a message whose last `rem` (< 64) bytes start at p.
// Compresses one or two padded blocks into h.  total_bytes is the whole
// message length (prefix + this call), used for the 64-bit bit count.
__device__ __forceinline__ void finish_message(uint32_t (&h)[5], const uint8_t* p, uint32_t rem,
                                               uint64_t total_bytes) {
    uint32_t w[16];
    if (rem) {
        load_block_partial(p, rem, w);
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = 0u;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = pad_word(bswap(w[j]), j, static_cast<int>(rem));
    const uint64_t bits = total_bytes * 8ull;
    const uint32_t hi = static_cast<uint32_t>(bits >> 32), lo = static_cast<uint32_t>(bits);
    if (rem < 56) {
        w[14] = hi;
        w[15] = lo;
        compress(h, w);
    } else {
        compress(h, w);
#pragma unroll
        for (int j = 0; j < 14; ++j) w[j] = 0u;
        w[14] = hi;
        w[15] = lo;
        compress(h, w);
    }
}

__device__ __forceinline__ void store_digest(uint8_t* out, const uint32_t (&h)[5]) {
    uint32_t* o = reinterpret_cast<uint32_t*>(out);  // 4-byte aligned (checked on host)
#pragma unroll
    for (int i = 0; i < 5; ++i) o[i] = bswap(h[i]);
}

}  // namespace s1
