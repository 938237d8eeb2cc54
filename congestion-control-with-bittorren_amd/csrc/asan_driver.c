/* asan_driver.c -- test program, not part of the library: drives every
 * host-side path of libsha1chunk (built with host AddressSanitizer +
 * UndefinedBehaviorSanitizer, `make asan`) on a real device, so the runtime's
 * host code -- pipelines, pinned staging, part pools, the verify queue, the
 * streaming trio, the chunk-file C layer -- runs under the sanitizers.  GPU
 * code is not instrumented (no GPU ASan on this pool).  Cross-checks the
 * paths against each other and the NIST "abc" vector (sha.c:32-38); prints
 * "asan-driver ok" and exits 0 when everything agrees.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/chunk_hash.h"
#include "../../include/sha.h"
#include "../../include/sha1chunk.h"

#define L512 524288u

/* the few HIP runtime calls the device-batch section needs (C linkage in
 * libamdhip64; hipMemcpyKind 1 = host to device, 2 = device to host) */
extern int hipMalloc(void **p, size_t bytes);
extern int hipFree(void *p);
extern int hipMemcpy(void *dst, const void *src, size_t bytes, int kind);
extern int hipDeviceSynchronize(void);

static int fails = 0;
#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);               \
            fprintf(stderr, "\n");                      \
            ++fails;                                    \
        }                                               \
    } while (0)

static uint64_t rng = 88172645463325252ull;
static uint8_t next_byte(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint8_t)rng;
}

int main(void) {
    CHECK(sha1chunk_device_count() > 0, "no device: %s", sha1chunk_last_error());
    /* receive-thread placement: the L3 domains of the GPU's node, round robin */
    {
        unsigned char m0[128], m[256];
        unsigned nd = 0, nd2 = 0;
        const int c0 = sha1chunk_receive_cpus(0, 0, m0, sizeof m0, &nd);
        CHECK(c0 > 0 && nd > 0, "receive_cpus: %d %s", c0, sha1chunk_last_error());
        for (unsigned s = 1; s <= 2 * nd && c0 > 0 && nd > 0; ++s) {
            const int c = sha1chunk_receive_cpus(0, s, m, sizeof m, &nd2);  /* a longer mask: zero-filled */
            CHECK(c > 0 && nd2 == nd, "receive_cpus slot %u", s);
            for (size_t i = 128; i < sizeof m; ++i) CHECK(m[i] == 0, "receive_cpus tail byte %zu", i);
            CHECK((s % nd == 0) == !memcmp(m, m0, sizeof m0), "receive_cpus round robin %u", s);
        }
        CHECK(sha1chunk_receive_cpus(0, 0, m, 64, NULL) == SHA1CHUNK_EINVAL, "receive_cpus short mask");
    }
    /* NIST "abc" (sha.c:32-38) through shahash and the streaming trio */
    static const uint8_t abc_want[20] = {0xa9, 0x99, 0x3e, 0x36, 0x47, 0x06, 0x81, 0x6a, 0xba, 0x3e,
                                         0x25, 0x71, 0x78, 0x50, 0xc2, 0x6c, 0x9c, 0xd0, 0xd8, 0x9d};
    uint8_t d[20], d2[20];
    shahash((uint8_t *)"abc", 3, d);
    CHECK(!memcmp(d, abc_want, 20), "shahash abc");
    SHA1Context c;
    SHA1Init(&c);
    SHA1Update(&c, "a", 1);
    SHA1Update(&c, "bc", 2);
    SHA1Final(&c, d2);
    CHECK(!memcmp(d2, abc_want, 20), "streaming abc");

    /* ragged host batch: digests vs one shahash per chunk and vs streaming */
    const size_t n = 300;
    uint64_t *off = malloc(n * sizeof *off);
    uint32_t *len = malloc(n * sizeof *len);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        len[i] = (i % 7 == 0) ? L512 : (uint32_t)((i * 7919u) % 70000u);
        off[i] = total + (i % 3);
        total = off[i] + len[i];
    }
    uint8_t *buf = malloc(total + 1);
    for (size_t i = 0; i < total; ++i) buf[i] = next_byte();
    uint8_t *dig = malloc(n * 20), *mis = malloc(n);
    CHECK(sha1chunk_hash_batch(buf, off, len, n, dig, SHA1CHUNK_HOST) == 0, "hash_batch: %s",
          sha1chunk_last_error());
    for (size_t i = 0; i < n; i += 37) {
        shahash(buf + off[i], (int)len[i], d);
        CHECK(!memcmp(d, dig + 20 * i, 20), "batch vs shahash %zu", i);
        SHA1Init(&c);
        for (uint32_t p = 0; p < len[i];) {
            uint32_t s = 1 + (p * 31u) % 5000u;
            if (s > len[i] - p) s = len[i] - p;
            SHA1Update(&c, buf + off[i] + p, s);
            p += s;
        }
        SHA1Final(&c, d2);
        CHECK(!memcmp(d2, dig + 20 * i, 20), "batch vs streaming %zu", i);
    }
    /* verify_batch with two corrupted expectations */
    uint8_t *exp = malloc(n * 20);
    memcpy(exp, dig, n * 20);
    exp[20 * 5] ^= 1;
    exp[20 * 200 + 19] ^= 0x80;
    CHECK(sha1chunk_verify_batch(buf, off, len, n, exp, mis, SHA1CHUNK_HOST) == 0, "verify_batch");
    for (size_t i = 0; i < n; ++i) CHECK(mis[i] == (i == 5 || i == 200), "verify_batch flag %zu", i);

    /* verify queue, both implementations (batch launches; the persistent
     * drain reading a small pinned host ring, with a 1 ms idle exit so it
     * leaves and is relaunched): growth, polling, flush; every tag once with
     * the right flag.  The third pass is a batch-1 queue: the host path when
     * SHA1CHUNK_HOST_SMALL covers L512, else the drain with one-chunk groups */
    static const char *modes[3] = {"batch", "persistent", "persistent"};
    static const size_t vq_batch[3] = {16, 16, 1};
    for (int mo = 0; mo < 3; ++mo) {
    setenv("SHA1CHUNK_VQ_MODE", modes[mo], 1);
    setenv("SHA1CHUNK_VQ_IDLE_MS", "1", 1);
    setenv("SHA1CHUNK_VQ_RING_MIB", "8", 1);
    sha1chunk_vq *q = sha1chunk_vq_create(vq_batch[mo], L512);
    CHECK(q != NULL, "vq_create: %s", sha1chunk_last_error());
    size_t seen = 0;
    uint8_t *got = calloc(n, 1);
    uint64_t tags[64];
    uint8_t bad[64];
    for (size_t i = 0; i < n; ++i) {
        CHECK(sha1chunk_vq_submit(q, buf + off[i], len[i], exp + 20 * i, i) == 0, "vq_submit");
        long k = sha1chunk_vq_poll(q, tags, bad, 64, 0);
        for (long j = 0; j < k; ++j) {
            CHECK(tags[j] < n && !got[tags[j]], "vq tag");
            got[tags[j]] = 1;
            CHECK(bad[j] == (tags[j] == 5 || tags[j] == 200), "vq flag %llu", (unsigned long long)tags[j]);
            ++seen;
        }
    }
    for (;;) {
        long k = sha1chunk_vq_poll(q, tags, bad, 64, 1);
        if (k <= 0) break;
        for (long j = 0; j < k; ++j) {
            CHECK(tags[j] < n && !got[tags[j]], "vq tag");
            got[tags[j]] = 1;
            CHECK(bad[j] == (tags[j] == 5 || tags[j] == 200), "vq flag");
            ++seen;
        }
    }
    CHECK(seen == n && sha1chunk_vq_pending(q) == 0, "vq drained %zu of %zu", seen, n);
    /* zero-copy receive: reserve a buffer in the ring, fill it in place as
     * DATA packets would (1484-byte pieces, reliable_udp.c:339), commit it,
     * and release it once its result is back (after the job-buffer copy,
     * reliable_udp.c:696-709) -- up to 8 buffers outstanding, every 7th
     * reservation dropped without a commit; the chunk is checked in place
     * after its result, before the release */
    {
        void **bufp = calloc(n, sizeof *bufp);
        memset(got, 0, n);
        seen = 0;
        size_t held = 0;
        for (size_t i = 0; i < n; ++i) {
            if (i % 7 == 3) { /* an aborted session */
                void *b = sha1chunk_vq_reserve(q, L512);
                CHECK(b != NULL, "vq_reserve (abort): %s", sha1chunk_last_error());
                CHECK(sha1chunk_vq_release(q, b) == 0, "vq_release (abort)");
            }
            uint8_t *b = sha1chunk_vq_reserve(q, len[i] ? len[i] : 1);
            CHECK(b != NULL, "vq_reserve: %s", sha1chunk_last_error());
            for (uint32_t o = 0; o < len[i]; o += 1484)
                memcpy(b + o, buf + off[i] + o, len[i] - o < 1484 ? len[i] - o : 1484);
            bufp[i] = b;
            CHECK(sha1chunk_vq_commit(q, b, len[i], exp + 20 * i, i) == 0, "vq_commit: %s", sha1chunk_last_error());
            ++held;
            for (;;) {
                long k = sha1chunk_vq_poll(q, tags, bad, 64, held >= 8);
                CHECK(k >= 0, "vq_poll: %s", sha1chunk_last_error());
                for (long j = 0; j < k; ++j) {
                    const uint64_t t = tags[j];
                    CHECK(t < n && !got[t], "vq tag");
                    got[t] = 1;
                    CHECK(bad[j] == (t == 5 || t == 200), "vq flag %llu", (unsigned long long)t);
                    CHECK(memcmp(bufp[t], buf + off[t], len[t]) == 0, "reserved buffer changed");
                    CHECK(sha1chunk_vq_release(q, bufp[t]) == 0, "vq_release");
                    CHECK(sha1chunk_vq_release(q, bufp[t]) != 0, "double release accepted");
                    --held;
                    ++seen;
                }
                if (held < 8) break;
            }
        }
        for (;;) {
            long k = sha1chunk_vq_poll(q, tags, bad, 64, 1);
            if (k <= 0) break;
            for (long j = 0; j < k; ++j) {
                const uint64_t t = tags[j];
                CHECK(t < n && !got[t], "vq tag");
                got[t] = 1;
                CHECK(bad[j] == (t == 5 || t == 200), "vq flag");
                CHECK(sha1chunk_vq_release(q, bufp[t]) == 0, "vq_release");
                ++seen;
            }
        }
        CHECK(seen == n && sha1chunk_vq_pending(q) == 0, "vq zero-copy drained %zu of %zu", seen, n);
        CHECK(sha1chunk_vq_commit(q, buf, 3, exp, 1) != 0, "commit of a foreign buffer accepted");
        if (mo == 1) {
            /* the persistent ring (its floor: 2 groups of 64 max-length
             * chunks, 64 MiB here): reservations never released fill it, and
             * reserve fails instead of waiting forever */
            void *hold[256];
            size_t k = 0;
            while (k < 256 && (hold[k] = sha1chunk_vq_reserve(q, L512)) != NULL) ++k;
            CHECK(k >= 126 && k <= 128, "ring of 64 MiB took %zu reservations of 512 KiB", k);
            for (size_t j = 0; j < k; ++j) CHECK(sha1chunk_vq_release(q, hold[j]) == 0, "vq_release (hold)");
            void *b = sha1chunk_vq_reserve(q, L512);
            CHECK(b != NULL && sha1chunk_vq_release(q, b) == 0, "reserve after releasing the ring");
        }
        free(bufp);
    }
    sha1chunk_vq_destroy(q);
    free(got);
    }
    unsetenv("SHA1CHUNK_VQ_MODE");
    unsetenv("SHA1CHUNK_VQ_IDLE_MS");
    unsetenv("SHA1CHUNK_VQ_RING_MIB");

    /* device ragged batch above one group per CU: the length sort, the
     * mixed kernel's planner and its forced plans (env parsing included),
     * against the host batch path; a malformed plan must fail */
    {
        const size_t nd = 64 * 320 + 17; /* > 256 CUs' worth of groups */
        uint64_t *doff = malloc(nd * sizeof *doff);
        uint32_t *dlen = malloc(nd * sizeof *dlen);
        size_t dtot = 0;
        for (size_t i = 0; i < nd; ++i) {
            dlen[i] = (i % 97 == 0) ? 20000u + (uint32_t)(i % 300u) : (uint32_t)((i * 2654435761u) % 1500u);
            doff[i] = dtot;
            dtot += (dlen[i] + 127u) / 128u * 128u;
        }
        uint8_t *hb = malloc(dtot + 64);
        for (size_t i = 0; i < dtot + 64; ++i) hb[i] = next_byte();
        uint8_t *want = malloc(nd * 20), *gotd = malloc(nd * 20);
        CHECK(sha1chunk_hash_batch(hb, doff, dlen, nd, want, SHA1CHUNK_HOST) == 0, "host ragged: %s",
              sha1chunk_last_error());
        void *dbase = NULL, *doffp = NULL, *dlenp = NULL, *ddig = NULL;
        CHECK(!hipMalloc(&dbase, dtot + 64) && !hipMalloc(&doffp, nd * 8) && !hipMalloc(&dlenp, nd * 4) &&
                  !hipMalloc(&ddig, nd * 20),
              "hipMalloc");
        CHECK(!hipMemcpy(dbase, hb, dtot + 64, 1) && !hipMemcpy(doffp, doff, nd * 8, 1) &&
                  !hipMemcpy(dlenp, dlen, nd * 4, 1),
              "hipMemcpy H2D");
        static const char *plans[] = {NULL, "0,0,4", "0,0,8", "0,7,4", "0,321,4", "1,0,0"};
        for (size_t k = 0; k < sizeof plans / sizeof plans[0]; ++k) {
            if (plans[k]) setenv("SHA1CHUNK_MIXED_PLAN", plans[k], 1);
            else unsetenv("SHA1CHUNK_MIXED_PLAN");
            setenv("SHA1CHUNK_MIXED_DEBUG", k == 0 ? "1" : "0", 1);
            memset(gotd, 0, nd * 20);
            CHECK(sha1chunk_hash_device_async(dbase, doffp, dlenp, nd, ddig, NULL, SHA1CHUNK_KERNEL_AUTO) == 0,
                  "device ragged plan %s: %s", plans[k] ? plans[k] : "device", sha1chunk_last_error());
            CHECK(!hipDeviceSynchronize() && !hipMemcpy(gotd, ddig, nd * 20, 2), "device sync");
            CHECK(!memcmp(gotd, want, nd * 20), "device ragged plan %s differs", plans[k] ? plans[k] : "device");
        }
        setenv("SHA1CHUNK_MIXED_PLAN", "0,99999,4", 1);
        CHECK(sha1chunk_hash_device_async(dbase, doffp, dlenp, nd, ddig, NULL, SHA1CHUNK_KERNEL_AUTO) ==
                  SHA1CHUNK_EINVAL,
              "bad plan accepted");
        unsetenv("SHA1CHUNK_MIXED_PLAN");
        unsetenv("SHA1CHUNK_MIXED_DEBUG");
        hipDeviceSynchronize();
        hipFree(dbase), hipFree(doffp), hipFree(dlenp), hipFree(ddig);
        free(doff), free(dlen), free(hb), free(want), free(gotd);
    }

    /* file pipeline: make_chunks(FILE*) and the fd path over a temp file, on
     * one device and split over every device (SHA1CHUNK_FILE_DEVICES; the
     * test runs the driver with SHA1CHUNK_VIRTUAL_DEVICES=2) */
    char path[] = "/tmp/asan_driver_XXXXXX";
    int fd = mkstemp(path);
    const size_t fbytes = 9 * (size_t)L512 + 12345;
    CHECK(fd >= 0 && write(fd, buf, fbytes) == (ssize_t)fbytes, "temp file");
    close(fd);
    for (int fdv = 0; fdv < 2; ++fdv) {
        if (fdv) setenv("SHA1CHUNK_FILE_DEVICES", "all", 1);
        FILE *f = fopen(path, "r");
        uint8_t *hs[10];
        for (int i = 0; i < 10; ++i) hs[i] = malloc(20);
        int m = make_chunks(f, hs);
        fclose(f);
        CHECK(m == 10, "make_chunks count %d (file devices: %d)", m, fdv);
        for (int i = 0; i < 10; ++i) {
            shahash(buf + (size_t)i * L512, i < 9 ? (int)L512 : 12345, d);
            CHECK(i >= m || !memcmp(d, hs[i], 20), "make_chunks chunk %d (file devices: %d)", i, fdv);
            free(hs[i]);
        }
    }
    unsetenv("SHA1CHUNK_FILE_DEVICES");
    char *hex = get_chunk_hash((char *)buf, L512);
    char want_hex[41];
    shahash(buf, L512, d);
    binary2hex(d, 20, want_hex);
    CHECK(!strcmp(hex, want_hex), "get_chunk_hash");
    CHECK(verify_hash(hex, (char *)buf) == 0, "verify_hash match");
    free(hex);
    unlink(path);

    free(off), free(len), free(buf), free(dig), free(mis), free(exp);
    /* _exit: skip the HIP/HSA runtime's own teardown, which trips the ROCm
     * ASan runtime's device-allocator check after main (not this code) */
    if (fails) {
        fprintf(stderr, "asan-driver: %d failures\n", fails);
        fflush(NULL);
        _exit(1);
    }
    printf("asan-driver ok\n");
    fflush(NULL);
    _exit(0);
}
