/*
 * sha.h -- drop-in replacement header for the reference's sha.h.
 *
 * Replaces: /root/reference/sha.h:39-64 (SHA1Context, SHA1Init/Update/Final).
 * The context keeps the reference's 96-byte layout (offsetof-checked in
 * tests/test_boundary.py) so code that embeds or memsets it is unaffected:
 *   totalLength @0 (bits), hash[5] @8, bufferLength @28, buffer @32.
 * The implementation lives in libsha1chunk.so (chunk_api.c).  Routing
 * (include/sha1chunk.h, csrc/frontend.c): a SHA1Update/SHA1Final stream is
 * one message, one serial chain of compressions, so by default its whole
 * 64-byte blocks are compressed on the host (csrc/sha1_host.c: the x86 SHA
 * extensions, ~2.5 GB/s a core, against ~85 MB/s for one GPU lane); a gfx950
 * device is still required.  SHA1CHUNK_HOST_SMALL=0 sends them to the gfx950
 * kernels (sha1chunk_compress_blocks); "<bytes>" hashes calls up to that
 * size on the host and larger ones on the kernels.
 */
#ifndef SHA1CHUNK_SHA_H
#define SHA1CHUNK_SHA_H

#include <inttypes.h>

#define SHA1_HASH_SIZE 20
#define SHA1_HASH_WORDS 5

struct _SHA1Context {
    uint64_t totalLength;          /* message length so far, in bits     */
    uint32_t hash[SHA1_HASH_WORDS]; /* chaining value                     */
    uint32_t bufferLength;         /* bytes staged in buffer (0..63)     */
    union {
        uint32_t words[16];
        uint8_t bytes[64];
    } buffer;                      /* partial block awaiting compression */
};
typedef struct _SHA1Context SHA1Context;

#ifdef __cplusplus
extern "C" {
#endif

/* sha.h:58 -- IV, zero counters. */
void SHA1Init(SHA1Context *sc);
/* sha.h:59 -- append len bytes; complete blocks are compressed as routed above. */
void SHA1Update(SHA1Context *sc, const void *data, uint32_t len);
/* sha.h:60 -- pad, append the 64-bit length, emit the big-endian digest
 * (hash may be NULL, as in the reference). */
void SHA1Final(SHA1Context *sc, uint8_t hash[SHA1_HASH_SIZE]);

#ifdef __cplusplus
}
#endif

#endif
