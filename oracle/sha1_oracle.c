/*
 * sha1_oracle.c -- TEST INFRASTRUCTURE ONLY (see sha1_oracle.h).
 *
 * A clean-room FIPS 180-4 SHA-1, restated with the same observable
 * behaviour as the reference /root/reference/sha.c:
 *   - IV and zeroed counters ............................ sha.c:149-163
 *   - compression: big-endian word load, 80-word schedule
 *     W[t] = ROTL1(W[t-3]^W[t-8]^W[t-14]^W[t-16]), 80 rounds
 *     with Ch / Parity / Maj / Parity and K0..K3, feed-forward ... sha.c:176-451
 *   - Update stages every byte through the 64-byte block and
 *     compresses when it fills; the bit counter grows by 8*n ..... sha.c:453-527
 *   - Final pads 0x80 00.. to 56 mod 64 (120 - staged, minus 64
 *     when > 64) then the 64-bit big-endian bit count; the digest
 *     is the chaining value written most-significant byte first ... sha.c:529-558
 *   - shahash = Init, one Update(len), Final, wipe ............. chunk.c:35-51
 *   - lengths are uint32_t per Update call (sha.h:59) and int in
 *     shahash (chunk.c:35); both irrelevant below 2 GiB.
 */
#include "sha1_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static inline uint32_t rotl32(uint32_t x, unsigned s) { return (x << s) | (x >> (32u - s)); }

static inline uint32_t load_be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

/* One compression of a 64-byte block into h[5]. */
static void compress(uint32_t h[5], const uint8_t *block) {
    uint32_t sched[80];
    for (int t = 0; t < 16; ++t) sched[t] = load_be32(block + 4 * t);
    for (int t = 16; t < 80; ++t)
        sched[t] = rotl32(sched[t - 3] ^ sched[t - 8] ^ sched[t - 14] ^ sched[t - 16], 1);

    uint32_t v[5] = {h[0], h[1], h[2], h[3], h[4]}; /* a b c d e */
    for (int t = 0; t < 80; ++t) {
        uint32_t f, k;
        const uint32_t b = v[1], c = v[2], d = v[3];
        switch (t / 20) {
        case 0: f = (b & c) | (~b & d);          k = 0x5a827999u; break; /* Ch     */
        case 1: f = b ^ c ^ d;                   k = 0x6ed9eba1u; break; /* Parity */
        case 2: f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdcu; break; /* Maj    */
        default: f = b ^ c ^ d;                  k = 0xca62c1d6u; break; /* Parity */
        }
        const uint32_t tmp = rotl32(v[0], 5) + f + v[4] + k + sched[t];
        v[4] = d;
        v[3] = c;
        v[2] = rotl32(b, 30);
        v[1] = v[0];
        v[0] = tmp;
    }
    for (int i = 0; i < 5; ++i) h[i] += v[i];
}

void oracle_sha1_init(oracle_sha1_ctx *c) {
    static const uint32_t iv[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
    c->total_bits = 0;
    memcpy(c->h, iv, sizeof iv);
    c->staged = 0;
}

void oracle_sha1_update(oracle_sha1_ctx *c, const void *p, uint32_t n) {
    const uint8_t *src = (const uint8_t *)p;
    while (n > 0) {
        uint32_t room = 64u - c->staged;
        uint32_t take = n < room ? n : room;
        memcpy(c->blk.b + c->staged, src, take);
        c->staged += take;
        c->total_bits += (uint64_t)take * 8u;
        src += take;
        n -= take;
        if (c->staged == 64u) {
            compress(c->h, c->blk.b);
            c->staged = 0;
        }
    }
}

void oracle_sha1_final(oracle_sha1_ctx *c, uint8_t out[20]) {
    uint8_t pad[72];
    uint32_t npad = 120u - c->staged;
    if (npad > 64u) npad -= 64u;
    memset(pad, 0, sizeof pad);
    pad[0] = 0x80;
    const uint64_t bits = c->total_bits;
    uint8_t lenbe[8];
    for (int i = 0; i < 8; ++i) lenbe[i] = (uint8_t)(bits >> (56 - 8 * i));
    oracle_sha1_update(c, pad, npad);
    oracle_sha1_update(c, lenbe, 8);
    if (out) {
        for (int i = 0; i < 5; ++i) {
            out[4 * i + 0] = (uint8_t)(c->h[i] >> 24);
            out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
            out[4 * i + 2] = (uint8_t)(c->h[i] >> 8);
            out[4 * i + 3] = (uint8_t)(c->h[i]);
        }
    }
}

void oracle_shahash(const uint8_t *p, int len, uint8_t out[20]) {
    oracle_sha1_ctx c;
    oracle_sha1_init(&c);
    oracle_sha1_update(&c, p, (uint32_t)len);
    oracle_sha1_final(&c, out);
    memset(&c, 0, sizeof c);
}

/* ---------------------------------------------------------------- batch -- */

typedef struct {
    const uint8_t *base;
    const uint64_t *off;
    const uint32_t *len;
    size_t n;
    uint8_t *dig;
    int tid, nthr;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->nthr)
        oracle_shahash(j->base + j->off[i], (int)j->len[i], j->dig + 20 * i);
    return NULL;
}

void oracle_hash_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, size_t n,
                       uint8_t *digests, int threads) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > n && n > 0) threads = (int)n;
    batch_job *jobs = (batch_job *)calloc((size_t)threads, sizeof *jobs);
    pthread_t *tids = (pthread_t *)calloc((size_t)threads, sizeof *tids);
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (batch_job){base, off, len, n, digests, t, threads};
        if (t > 0) pthread_create(&tids[t], NULL, batch_worker, &jobs[t]);
    }
    batch_worker(&jobs[0]);
    for (int t = 1; t < threads; ++t) pthread_join(tids[t], NULL);
    free(jobs);
    free(tids);
}

/* ------------------------------------------------------------ synthetic -- */

uint64_t oracle_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_synth_chunk(uint8_t *dst, uint64_t chunk, uint32_t len, uint64_t seed) {
    const uint64_t key = seed ^ (chunk << 24);
    uint32_t nw = len / 8u;
    for (uint32_t w = 0; w < nw; ++w) {
        uint64_t v = oracle_splitmix64(key ^ (uint64_t)w);
        memcpy(dst + 8u * w, &v, 8); /* little-endian host */
    }
    uint32_t rem = len % 8u;
    if (rem) {
        uint64_t v = oracle_splitmix64(key ^ (uint64_t)nw);
        memcpy(dst + 8u * nw, &v, rem);
    }
}

void oracle_synth_fill(uint8_t *dst, uint64_t first, uint64_t count, uint32_t chunk_len,
                       uint64_t seed) {
    for (uint64_t i = 0; i < count; ++i)
        oracle_synth_chunk(dst + i * (uint64_t)chunk_len, first + i, chunk_len, seed);
}

uint32_t oracle_mixed_len(uint64_t i, uint64_t seed) {
    uint64_t r = oracle_splitmix64((seed + 1u) ^ i);
    uint32_t octave = (uint32_t)(r & 7u);              /* 0..7            */
    uint32_t mant = (uint32_t)((r >> 8) & 4095u);      /* 0..4095         */
    uint32_t len = (4096u + mant) << octave;           /* 4 KiB .. ~1 MiB */
    if (i % 7u == 6u) len += 1u + (uint32_t)(oracle_splitmix64((seed + 2u) ^ i) % 63u);
    return len;
}

double oracle_time_synth(uint64_t first, uint64_t count, uint32_t chunk_len, uint64_t seed,
                         int threads, uint8_t *agg20) {
    uint8_t *buf = (uint8_t *)malloc((size_t)count * chunk_len);
    uint64_t *off = (uint64_t *)malloc(count * sizeof *off);
    uint32_t *len = (uint32_t *)malloc(count * sizeof *len);
    uint8_t *dig = (uint8_t *)malloc(count * 20u);
    if (!buf || !off || !len || !dig) {
        free(buf); free(off); free(len); free(dig);
        return -1.0;
    }
    oracle_synth_fill(buf, first, count, chunk_len, seed);
    for (uint64_t i = 0; i < count; ++i) {
        off[i] = i * (uint64_t)chunk_len;
        len[i] = chunk_len;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    oracle_hash_batch(buf, off, len, count, dig, threads);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (agg20) oracle_shahash(dig, (int)(count * 20u), agg20);
    free(buf); free(off); free(len); free(dig);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Seconds for oracle_hash_batch over a batch already in memory (the CPU
 * baseline's restatement rows, bench.py). */
double oracle_time_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, size_t n,
                         uint8_t *dig, int threads) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    oracle_hash_batch(base, off, len, n, dig, threads);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
