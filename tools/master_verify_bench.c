/*
 * master_verify_bench.c -- per-GET cost of the sender-side verify
 * (packet_handler.c:434 -> chunk.c:204-217
 * verify_chunk_hash, which re-reads and re-hashes 512 KiB of the master data
 * file per request).  Not part of the library.
 *
 *   master_verify_bench <master file> <requests file> <json out>
 *
 * <requests file>: one "idx hex40" line per GET, in request order.  Each
 * request is one verify_chunk_hash(fp, hex, idx) on one FILE* kept open (as
 * a send session does, reliable_udp.c:180), timed on its own.  The JSON
 * holds the first call, the second (with the product library the master
 * index is built there: SHA1CHUNK_MASTER_INDEX), and the median / mean /
 * p99 of the rest.  verify_chunk_hash exits the process (-1) on a mismatch,
 * so a run that writes its JSON verified every request.
 *
 * Built twice: against libsha1chunk.so (tools/master_verify_bench,
 * `make -C congestion-control-with-bittorren_amd tools`) and against the
 * reference's own chunk.c + sha.c (oracle/_ref/master_verify_ref, `make -C
 * oracle ref`: the CPU baseline).  stdout (the two lines get_chunk_hash
 * prints per call, chunk.c:179,182) goes to /dev/null.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

void verify_chunk_hash(FILE *f, char *requested_chunk_hash, size_t chunk_idx);

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int cmp_d(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s <master file> <requests file> <json out>\n", argv[0]);
        return 2;
    }
    FILE *rq = fopen(argv[2], "r");
    if (!rq) {
        perror(argv[2]);
        return 2;
    }
    size_t cap = 1024, n = 0;
    size_t *idx = malloc(cap * sizeof *idx);
    char (*hex)[41] = malloc(cap * sizeof *hex);
    unsigned long long i0;
    char h[64];
    while (fscanf(rq, "%llu %63s", &i0, h) == 2) {
        if (n == cap) {
            cap *= 2;
            idx = realloc(idx, cap * sizeof *idx);
            hex = realloc(hex, cap * sizeof *hex);
        }
        idx[n] = (size_t)i0;
        snprintf(hex[n], 41, "%.40s", h);
        ++n;
    }
    fclose(rq);
    if (n < 3) {
        fprintf(stderr, "need at least 3 requests\n");
        return 2;
    }
    FILE *fp = fopen(argv[1], "rb");
    if (!fp) {
        perror(argv[1]);
        return 2;
    }
    if (!freopen("/dev/null", "w", stdout)) return 2;
    double *t = malloc(n * sizeof *t);
    const double all0 = now_s();
    for (size_t k = 0; k < n; ++k) {
        const double a = now_s();
        verify_chunk_hash(fp, hex[k], idx[k]);
        t[k] = now_s() - a;
    }
    const double all = now_s() - all0;
    const size_t m = n - 2;
    double *rest = malloc(m * sizeof *rest), sum = 0;
    for (size_t k = 0; k < m; ++k) sum += (rest[k] = t[k + 2]);
    qsort(rest, m, sizeof *rest, cmp_d);
    FILE *o = fopen(argv[3], "w");
    if (!o) return 2;
    fprintf(o,
            "{\"requests\": %zu, \"first_call_ms\": %.4f, \"second_call_ms\": %.4f, \"rest_median_ms\": %.5f, "
            "\"rest_mean_ms\": %.5f, \"rest_p99_ms\": %.5f, \"rest_max_ms\": %.5f, \"all_seconds\": %.4f, "
            "\"verified\": %zu}\n",
            n, t[0] * 1e3, t[1] * 1e3, rest[m / 2] * 1e3, sum / (double)m * 1e3, rest[(m * 99) / 100] * 1e3,
            rest[m - 1] * 1e3, all, n);
    fclose(o);
    fclose(fp);
    return 0;
}
