/*
 * sha1_host.c -- the host-side SHA-1 compression behind the library's
 * single-message path (csrc/frontend.c routing).
 *
 * One chunk per call is the peer's synchronous receive verify
 * (packet_handler.c:472 -> job.c:217-228 verify_hash -> chunk.c:168-185
 * get_chunk_hash -> chunk.c:35-51 shahash).  On the GPU that is one lane's
 * serial chain of 8193 compressions, 6.0 ms for 512 KiB; the reference's
 * sha.c does it in ~0.7 ms on one core, this file in ~0.2 ms.  So by default
 * the reference's single-message calls (shahash and what is built on it,
 * the SHA1Update/SHA1Final trio) and make_chunks on a regular file of at
 * most 4 MiB are hashed here ("keep a CPU path",
 * "the streaming trio stays CPU"); SHA1CHUNK_HOST_SMALL=0 sends them to the
 * kernels, SHA1CHUNK_HOST_SMALL=<bytes> routes by size.  It is not a
 * fallback: the library still requires a gfx950 device for every call (no
 * device -> SHA1CHUNK_ENODEV), and every batch, device-resident,
 * verify-queue and larger-file call -- and every kernel parity test, smoke
 * and bench number of the GPU path -- runs on the kernels.
 *
 * Compression (FIPS 180-4 section 6.1.2, the function sha.c:176-451
 * implements): the x86 SHA extensions when the CPU has them (sha1rnds4 does
 * four rounds, sha1nexte folds e into the next four message words,
 * sha1msg1/sha1msg2 expand the schedule four words at a time), else a
 * portable loop.  SHA1HOST_PORTABLE=1 forces the portable loop (tests).
 * Padding follows sha.c:529-558: 0x80, zeros to 56 mod 64, 64-bit
 * big-endian bit count.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sha1_host.h"

static inline uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static inline uint32_t load_be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

static void compress_portable(uint32_t h[5], const uint8_t *blocks, size_t nblocks) {
    for (size_t b = 0; b < nblocks; ++b, blocks += 64) {
        uint32_t w[16];
        for (int t = 0; t < 16; ++t) w[t] = load_be32(blocks + 4 * t);
        uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4];
        for (int t = 0; t < 80; ++t) {
            uint32_t wt;
            if (t < 16) {
                wt = w[t];
            } else {  /* 16-word circular schedule */
                wt = rol32(w[(t + 13) & 15] ^ w[(t + 8) & 15] ^ w[(t + 2) & 15] ^ w[t & 15], 1);
                w[t & 15] = wt;
            }
            uint32_t f, k;
            if (t < 20) {
                f = d ^ (bb & (c ^ d));
                k = 0x5a827999u;
            } else if (t < 40) {
                f = bb ^ c ^ d;
                k = 0x6ed9eba1u;
            } else if (t < 60) {
                f = (bb & c) | (d & (bb | c));
                k = 0x8f1bbcdcu;
            } else {
                f = bb ^ c ^ d;
                k = 0xca62c1d6u;
            }
            const uint32_t x = rol32(a, 5) + f + e + k + wt;
            e = d;
            d = c;
            c = rol32(bb, 30);
            bb = a;
            a = x;
        }
        h[0] += a;
        h[1] += bb;
        h[2] += c;
        h[3] += d;
        h[4] += e;
    }
}

#if defined(__x86_64__)
#include <immintrin.h>

/* Four rounds 4I..4I+3 (function group G = 0..3) on message vector m[I&3]
 * (words 4I..4I+3 in lanes 3..0).  Their e is the block's e for step 0,
 * later rotl30 of the a that the previous step started from (sha1nexte of
 * that step's input ABCD, `eprev`), added to the first word. */
#define SHA1_STEP(I, G)                                                          \
    do {                                                                         \
        __m128i ein = (I) == 0 ? _mm_add_epi32(e, m[0]) : _mm_sha1nexte_epu32(eprev, m[(I)&3]); \
        eprev = abcd;                                                            \
        abcd = _mm_sha1rnds4_epu32(abcd, ein, G);                                \
    } while (0)
/* X_i = rotl1(X_{i-3} ^ X_{i-8} ^ X_{i-14} ^ X_{i-16}) four words at a time:
 * m[i&3] holds X_{i-4} on entry, m[(i+1)&3] .. m[(i+3)&3] X_{i-3} .. X_{i-1}. */
#define SHA1_NEXT_MSG(I)                                                         \
    m[(I)&3] = _mm_sha1msg2_epu32(                                               \
        _mm_xor_si128(_mm_sha1msg1_epu32(m[(I)&3], m[((I) + 1) & 3]), m[((I) + 2) & 3]), m[((I) + 3) & 3])

__attribute__((target("sha,sse4.1,ssse3"))) static void compress_shani(uint32_t h[5], const uint8_t *blocks,
                                                                        size_t nblocks) {
    const __m128i bswap_words = _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    /* lane 3 = a .. lane 0 = d; e in lane 3 of its own vector */
    __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *)h), 0x1B);
    __m128i e = _mm_set_epi32((int)h[4], 0, 0, 0);
    for (size_t b = 0; b < nblocks; ++b, blocks += 64) {
        const __m128i abcd0 = abcd, e0 = e;
        __m128i m[4], eprev = _mm_setzero_si128();
        for (int j = 0; j < 4; ++j)
            m[j] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(blocks + 16 * j)), bswap_words);
        SHA1_STEP(0, 0);
        SHA1_STEP(1, 0);
        SHA1_STEP(2, 0);
        SHA1_STEP(3, 0);
        SHA1_NEXT_MSG(4);  SHA1_STEP(4, 0);
        SHA1_NEXT_MSG(5);  SHA1_STEP(5, 1);
        SHA1_NEXT_MSG(6);  SHA1_STEP(6, 1);
        SHA1_NEXT_MSG(7);  SHA1_STEP(7, 1);
        SHA1_NEXT_MSG(8);  SHA1_STEP(8, 1);
        SHA1_NEXT_MSG(9);  SHA1_STEP(9, 1);
        SHA1_NEXT_MSG(10); SHA1_STEP(10, 2);
        SHA1_NEXT_MSG(11); SHA1_STEP(11, 2);
        SHA1_NEXT_MSG(12); SHA1_STEP(12, 2);
        SHA1_NEXT_MSG(13); SHA1_STEP(13, 2);
        SHA1_NEXT_MSG(14); SHA1_STEP(14, 2);
        SHA1_NEXT_MSG(15); SHA1_STEP(15, 3);
        SHA1_NEXT_MSG(16); SHA1_STEP(16, 3);
        SHA1_NEXT_MSG(17); SHA1_STEP(17, 3);
        SHA1_NEXT_MSG(18); SHA1_STEP(18, 3);
        SHA1_NEXT_MSG(19); SHA1_STEP(19, 3);
        e = _mm_sha1nexte_epu32(eprev, e0);  /* rotl30 of a four rounds back, + saved e */
        abcd = _mm_add_epi32(abcd, abcd0);
    }
    _mm_storeu_si128((__m128i *)h, _mm_shuffle_epi32(abcd, 0x1B));
    h[4] = (uint32_t)_mm_extract_epi32(e, 3);
}
#undef SHA1_STEP
#undef SHA1_NEXT_MSG
#endif

static int use_shani(void) {
#if defined(__x86_64__)
    static int cached = -1;  /* decided once; racing first callers store the same value */
    int v = __atomic_load_n(&cached, __ATOMIC_RELAXED);
    if (v < 0) {
        const char *p = getenv("SHA1HOST_PORTABLE");
        __builtin_cpu_init();
        v = !(p && atoi(p)) && __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
        __atomic_store_n(&cached, v, __ATOMIC_RELAXED);
    }
    return v;
#else
    return 0;
#endif
}

int sha1host_uses_shani(void) { return use_shani(); }

void sha1host_compress(uint32_t h[5], const void *blocks, size_t nblocks) {
#if defined(__x86_64__)
    if (use_shani()) {
        compress_shani(h, (const uint8_t *)blocks, nblocks);
        return;
    }
#endif
    compress_portable(h, (const uint8_t *)blocks, nblocks);
}

void sha1host_finish(const uint32_t state[5], uint64_t prefix_bytes, const void *tail, uint32_t tail_len,
                     uint8_t out[20]) {
    uint32_t h[5] = {state[0], state[1], state[2], state[3], state[4]};
    const uint8_t *t = (const uint8_t *)tail;
    const uint32_t whole = tail_len / 64u;
    if (whole) sha1host_compress(h, t, whole);
    const uint32_t rest = tail_len - 64u * whole;
    uint8_t pad[128];
    memset(pad, 0, sizeof pad);
    if (rest) memcpy(pad, t + 64u * whole, rest);
    pad[rest] = 0x80;
    const uint32_t padded = rest <= 55u ? 64u : 128u;
    const uint64_t bits = (prefix_bytes + tail_len) * 8u;
    for (int i = 0; i < 8; ++i) pad[padded - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha1host_compress(h, pad, padded / 64u);
    for (int i = 0; i < 5; ++i) {
        out[4 * i] = (uint8_t)(h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8);
        out[4 * i + 3] = (uint8_t)h[i];
    }
}

void sha1host_digest(const void *msg, uint64_t len, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
    const uint64_t whole = len / 64u;
    if (whole) sha1host_compress(h, msg, (size_t)whole);
    sha1host_finish(h, 64u * whole, (const uint8_t *)msg + 64u * whole, (uint32_t)(len - 64u * whole), out);
}
