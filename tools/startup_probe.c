/* startup_probe.c -- diagnostic only: where a short-lived caller of the
 * library (the make-chunks CLI on a small file, one verify_hash) spends its
 * fixed start-up time.  Prints milliseconds since main() at each step.
 *   gcc -O1 -I include tools/startup_probe.c -o tools/startup_probe \
 *       -L congestion-control-with-bittorren_amd -lsha1chunk \
 *       -Wl,-rpath,$PWD/congestion-control-with-bittorren_amd
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include "chunk_hash.h"
#include "sha1chunk.h"

static double t0;
static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}
static void mark(const char *what) { printf("{\"step\": \"%s\", \"ms\": %.2f}\n", what, now_ms() - t0); }

int main(void) {
    static uint8_t buf[524288];
    uint8_t out[20];
    t0 = now_ms();
    mark("main");
    int n = sha1chunk_device_count();
    mark(n > 0 ? "device_count (HIP runtime init + device probe)" : "device_count FAILED");
    shahash(buf, 64, out);
    mark("first shahash 64 B (streams, first kernel: code object load)");
    shahash(buf, 64, out);
    mark("second shahash 64 B");
    shahash(buf, (int)sizeof buf, out);
    mark("shahash 512 KiB (one chunk, one lane)");
    uint64_t off = 0;
    uint32_t len = sizeof buf;
    sha1chunk_hash_batch(buf, &off, &len, 1, out, SHA1CHUNK_HOST);
    mark("hash_batch 1 x 512 KiB");
    return 0;
}
