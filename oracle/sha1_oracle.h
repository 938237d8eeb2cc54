/*
 * sha1_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference SHA-1 path (Allan Saddi's sha.c as used by
 * chunk.c / make_chunks.c in /root/reference), written from FIPS 180-4.  It is
 * the parity CHECKER for the HIP engine: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product library
 * (libsha1chunk.so) never links or calls anything in this directory.
 *
 * Parity pinning: checked against the NIST vectors quoted at sha.c:32-38, the
 * chunk.c:235-255 "dash" self test, the tmp/{A,B,C}.chunks fixtures and the
 * compiled reference sha.c itself (oracle/_ref, built by oracle/Makefile).
 */
#ifndef SHA1_ORACLE_H
#define SHA1_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same 96-byte layout as SHA1Context (sha.h:39-52): total bit count @0,
 * chaining value @8, staged byte count @28, 64-byte staging block @32. */
typedef struct oracle_sha1_ctx {
    uint64_t total_bits;
    uint32_t h[5];
    uint32_t staged;
    union {
        uint32_t w[16];
        uint8_t b[64];
    } blk;
} oracle_sha1_ctx;

void oracle_sha1_init(oracle_sha1_ctx *c);                             /* sha.c:149-163 */
void oracle_sha1_update(oracle_sha1_ctx *c, const void *p, uint32_t n); /* sha.c:453-527 */
void oracle_sha1_final(oracle_sha1_ctx *c, uint8_t out[20]);           /* sha.c:529-558 */

/* One-shot wrapper with the semantics of shahash() (chunk.c:35-51). */
void oracle_shahash(const uint8_t *p, int len, uint8_t out[20]);

/* Batch of independent messages: digest[i] = SHA1(base[off[i] .. off[i]+len[i])).
 * Chunk-strided over `threads` pthreads (threads <= 1 -> calling thread). */
void oracle_hash_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len,
                       size_t n, uint8_t *digests, int threads);
/* oracle_hash_batch timed (seconds, CLOCK_MONOTONIC). */
double oracle_time_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, size_t n,
                         uint8_t *dig, int threads);

/* Synthetic corpus: 64-bit little-endian word w of chunk c is
 * splitmix64(seed ^ (c << 24) ^ w); a trailing partial word keeps its low
 * bytes.  Writes chunk c = first .. first+count-1, each `chunk_len` bytes,
 * back to back into dst. */
void oracle_synth_fill(uint8_t *dst, uint64_t first, uint64_t count, uint32_t chunk_len,
                       uint64_t seed);
/* Fill one chunk of arbitrary length (same formula). */
void oracle_synth_chunk(uint8_t *dst, uint64_t chunk, uint32_t len, uint64_t seed);

/* Integer-only log-spaced length generator for the mixed verify batch
 * (BASELINE config 5): 4 KiB .. ~1 MiB, every 7th length gets +1..63. */
uint32_t oracle_mixed_len(uint64_t i, uint64_t seed);

uint64_t oracle_splitmix64(uint64_t x);

/* Timed CPU throughput leg: hashes `count` synthetic chunks of chunk_len
 * bytes (generated first, untimed) on `threads` threads; returns seconds of
 * hashing and writes the digest of all digests to agg20 (may be NULL). */
double oracle_time_synth(uint64_t first, uint64_t count, uint32_t chunk_len, uint64_t seed,
                         int threads, uint8_t *agg20);

#ifdef __cplusplus
}
#endif
#endif
