/* sha1_host.h -- host-side SHA-1 for the single-message path (the default
 * routing of shahash / the SHA1Update trio / small files, csrc/frontend.c;
 * SHA1CHUNK_HOST_SMALL; sha1_host.c).  Internal to libsha1chunk.so (hidden
 * symbols); tests/test_host_small.py builds sha1_host.c on its own to check
 * it on the CPU. */
#ifndef SHA1_HOST_H
#define SHA1_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef SHA1HOST_API
#define SHA1HOST_API __attribute__((visibility("hidden")))
#endif

/* compress nblocks whole 64-byte blocks into the chaining value h */
SHA1HOST_API void sha1host_compress(uint32_t h[5], const void *blocks, size_t nblocks);
/* digest of (prefix_bytes already compressed into state) + tail: pads as
 * sha.c:529-558 and writes the 20-byte big-endian digest */
SHA1HOST_API void sha1host_finish(const uint32_t state[5], uint64_t prefix_bytes, const void *tail,
                                  uint32_t tail_len, uint8_t out[20]);
/* one whole message (shahash, chunk.c:35-51) */
SHA1HOST_API void sha1host_digest(const void *msg, uint64_t len, uint8_t out[20]);
/* 1 when the x86 SHA extensions are in use, 0 for the portable loop */
SHA1HOST_API int sha1host_uses_shani(void);

#ifdef __cplusplus
}
#endif
#endif
