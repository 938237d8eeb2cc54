/* frontend.h -- calls between the reference-named C layer (chunk_api.c) and
 * the front end (frontend.c) of libsha1chunk.so.  Hidden symbols: not part
 * of the library's ABI (include/ holds that). */
#ifndef SHA1CHUNK_FRONTEND_H
#define SHA1CHUNK_FRONTEND_H

#include <stdint.h>

/* 1 when make_chunks on a regular file of `bytes` bytes hashes on the host. */
__attribute__((visibility("hidden"))) int fe_file_on_host(uint64_t bytes);

#endif
