/* copy_probe.c -- host copy rates behind the verify queue's submit(): a
 * 512 KiB chunk that the calling thread has just written (hot in its own
 * caches) copied into a 1 GiB ring (DRAM), the ring walked in order, as
 * submit() copies a session buffer into the queue's pinned ring.
 *
 *   cc -O2 -mavx512f -pthread -o tools/copy_probe tools/copy_probe.c
 *   tools/copy_probe [threads]       one JSON line per (method, threads)
 *
 * Methods: glibc memcpy; rep movsb; 64-byte non-temporal stores
 * (_mm512_stream_si512, no read-for-ownership of the ring's lines).  Each
 * thread has its own source buffer and its own share of the ring (first
 * touched by it), and runs on its own L3 domain of the CPUs it may use, in
 * CPU order (one thread per L3 domain, as vq_zc_bench --pin l3).
 */
#define _GNU_SOURCE
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define CHUNK (512u << 10)
#define RING (1ull << 30)
#define PASSES 4

static int method, nthreads;
static uint8_t *ring;
static pthread_barrier_t bar;
static cpu_set_t dom[64];
static int ndom;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void copy_nt(uint8_t *dst, const uint8_t *src, size_t n) {
    for (size_t o = 0; o < n; o += 256) {
        __m512i a = _mm512_loadu_si512((const void *)(src + o));
        __m512i b = _mm512_loadu_si512((const void *)(src + o + 64));
        __m512i c = _mm512_loadu_si512((const void *)(src + o + 128));
        __m512i d = _mm512_loadu_si512((const void *)(src + o + 192));
        _mm512_stream_si512((void *)(dst + o), a);
        _mm512_stream_si512((void *)(dst + o + 64), b);
        _mm512_stream_si512((void *)(dst + o + 128), c);
        _mm512_stream_si512((void *)(dst + o + 192), d);
    }
    _mm_sfence();
}

static void copy_movsb(uint8_t *dst, const uint8_t *src, size_t n) {
    __asm__ volatile("rep movsb" : "+D"(dst), "+S"(src), "+c"(n) : : "memory");
}

static void *worker(void *arg) {
    const int t = (int)(intptr_t)arg;
    if (ndom) (void)sched_setaffinity(0, sizeof dom[0], &dom[t % ndom]);
    uint8_t *src = aligned_alloc(4096, CHUNK);
    memset(src, t + 1, CHUNK);
    const size_t part = RING / (size_t)nthreads / CHUNK * CHUNK;
    uint8_t *mine = ring + part * (size_t)t;
    memset(mine, 0, part); /* first touch by this thread */
    pthread_barrier_wait(&bar);
    pthread_barrier_wait(&bar);
    for (int p = 0; p < PASSES; ++p)
        for (size_t o = 0; o < part; o += CHUNK) {
            src[o / CHUNK % CHUNK] ^= 1; /* the chunk was just written */
            if (method == 0) memcpy(mine + o, src, CHUNK);
            else if (method == 1) copy_movsb(mine + o, src, CHUNK);
            else copy_nt(mine + o, src, CHUNK);
        }
    pthread_barrier_wait(&bar);
    free(src);
    return NULL;
}

/* L3 domains of the allowed CPUs, in CPU order */
static int l3_domains(void) {
    cpu_set_t allowed, seen;
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return 0;
    CPU_ZERO(&seen);
    int nd = 0;
    for (int c = 0; c < CPU_SETSIZE && nd < 64; ++c) {
        if (!CPU_ISSET(c, &allowed) || CPU_ISSET(c, &seen)) continue;
        char path[128], buf[1024];
        snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", c);
        FILE *f = fopen(path, "r");
        if (!f) return 0;
        if (!fgets(buf, sizeof buf, f)) buf[0] = 0;
        fclose(f);
        CPU_ZERO(&dom[nd]);
        for (char *tok = strtok(buf, ",\n"); tok; tok = strtok(NULL, ",\n")) {
            int a, b;
            const int k = sscanf(tok, "%d-%d", &a, &b);
            if (k < 1) continue;
            if (k == 1) b = a;
            for (int x = a; x <= b && x < CPU_SETSIZE; ++x)
                if (CPU_ISSET(x, &allowed)) {
                    CPU_SET(x, &dom[nd]);
                    CPU_SET(x, &seen);
                }
        }
        CPU_SET(c, &seen);
        if (CPU_COUNT(&dom[nd])) ++nd;
    }
    return nd;
}

int main(int argc, char **argv) {
    const int maxt = argc > 1 ? atoi(argv[1]) : 4;
    ndom = l3_domains();
    ring = aligned_alloc(1 << 21, RING);
    const char *names[3] = {"memcpy", "rep_movsb", "nt_avx512"};
    for (int threads = 1; threads <= maxt; threads *= 2)
        for (method = 0; method < 3; ++method) {
            nthreads = threads;
            pthread_barrier_init(&bar, NULL, (unsigned)threads + 1);
            pthread_t th[64];
            for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, (void *)(intptr_t)t);
            pthread_barrier_wait(&bar);
            const double t0 = now();
            pthread_barrier_wait(&bar);
            pthread_barrier_wait(&bar);
            const double dt = now() - t0;
            for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
            pthread_barrier_destroy(&bar);
            const double bytes = (double)(RING / (size_t)threads / CHUNK * CHUNK) * threads * PASSES;
            printf("{\"method\": \"%s\", \"threads\": %d, \"l3_domains\": %d, \"GiBps\": %.2f}\n", names[method],
                   threads, ndom, bytes / dt / (1 << 30));
            fflush(stdout);
        }
    free(ring);
    return 0;
}
