/*
 * ref_driver.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin timing/batch driver compiled TOGETHER with the unmodified reference
 * /root/reference/sha.c into oracle/_ref/libsharef*.so (recipe:
 * oracle/Makefile).  It calls the reference's own SHA1Init / SHA1Update /
 * SHA1Final (sha.h:58-60) exactly the way shahash() does (chunk.c:35-51), so
 * the numbers it produces are the reference's, not the restatement's.
 * Nothing here is copied from the reference; only its public API is used.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "sha.h" /* resolved to /root/reference/sha.h by the Makefile */
#include "sha1_oracle.h"

void ref_shahash(const uint8_t *p, int len, uint8_t out[20]) {
    SHA1Context c;
    SHA1Init(&c);
    SHA1Update(&c, p, (uint32_t)len);
    SHA1Final(&c, out);
    memset(&c, 0, sizeof c);
}

typedef struct {
    const uint8_t *base;
    const uint64_t *off;
    const uint32_t *len;
    size_t n;
    uint8_t *dig;
    int tid, nthr;
} ref_job;

static void *ref_worker(void *arg) {
    ref_job *j = (ref_job *)arg;
    for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->nthr)
        ref_shahash(j->base + j->off[i], (int)j->len[i], j->dig + 20 * i);
    return NULL;
}

void ref_hash_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, size_t n,
                    uint8_t *dig, int threads) {
    if (threads < 1) threads = 1;
    ref_job *jobs = (ref_job *)calloc((size_t)threads, sizeof *jobs);
    pthread_t *tids = (pthread_t *)calloc((size_t)threads, sizeof *tids);
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (ref_job){base, off, len, n, dig, t, threads};
        if (t > 0) pthread_create(&tids[t], NULL, ref_worker, &jobs[t]);
    }
    ref_worker(&jobs[0]);
    for (int t = 1; t < threads; ++t) pthread_join(tids[t], NULL);
    free(jobs);
    free(tids);
}

/* Same contract as oracle_time_synth, hashing with the reference sha.c. */
double ref_time_synth(uint64_t first, uint64_t count, uint32_t chunk_len, uint64_t seed,
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
    ref_hash_batch(buf, off, len, count, dig, threads);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (agg20) ref_shahash(dig, (int)(count * 20u), agg20);
    free(buf); free(off); free(len); free(dig);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Seconds to hash n chunks already in memory with the reference sha.c on
 * `threads` pthreads (chunk-strided), digests into dig: the CPU-baseline
 * rows of bench.py time the same bytes on every build and thread count. */
double ref_time_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, size_t n,
                      uint8_t *dig, int threads) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    ref_hash_batch(base, off, len, n, dig, threads);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
