/*
 * chunk_hash.h -- the hashing half of the reference's chunk.h, plus the
 * receiver-side verify_hash() of job.h, exported by libsha1chunk.so with the
 * reference's exact C signatures.
 *
 * Replaces (file:line in /root/reference):
 *   make_chunks        chunk.h:35  (chunk.c:15-27)   file -> per-512KiB digests
 *   shahash            chunk.h:38  (chunk.c:35-51)   one-shot SHA-1
 *   binary2hex         chunk.h:41  (chunk.c:57-63)   20 B -> 40 lowercase hex
 *   hex2binary         chunk.h:44  (chunk.c:78-85)   hex -> bytes
 *   verify_chunk_hash  chunk.h:50  (chunk.c:204-217) sender-side check, exit(-1) on mismatch
 *   get_chunk_hash     chunk.h:51  (chunk.c:168-185) malloc'd hex digest, caller frees
 *   verify_hash        job.h:65    (job.c:217-228)   0 = match, 1 = mismatch
 * The non-hash helpers of chunk.h (read_chunk, find_chunk_idx_from_hash,
 * seek_to_*) stay in the peer's chunk.c; see INTEGRATION.md.
 */
#ifndef SHA1CHUNK_CHUNK_HASH_H
#define SHA1CHUNK_CHUNK_HASH_H

#include <inttypes.h>
#include <stddef.h>
#include <stdio.h>

#define BT_CHUNK_SIZE (512 * 1024) /* chunk.h:17 */

#define ascii2hex(ascii, len, buf) hex2binary((ascii), (len), (buf)) /* chunk.h:19 */
#define hex2ascii(buf, len, ascii) binary2hex((buf), (len), (ascii)) /* chunk.h:20 */

#ifdef __cplusplus
extern "C" {
#endif

/* Hashes every 512 KiB chunk of fp (last one at its true length) into the
 * caller-allocated chunk_hashes[i] (20 bytes each); returns the count. The
 * file is streamed through pinned host buffers and hashed in device batches. */
int make_chunks(FILE *fp, uint8_t **chunk_hashes);

void shahash(uint8_t *chr, int len, uint8_t *target);
void binary2hex(uint8_t *buf, int len, char *ascii);
void hex2binary(char *hex, int len, uint8_t *buf);
void verify_chunk_hash(FILE *f, char *requested_chunk_hash, size_t chunk_idx);
char *get_chunk_hash(char *chunk, size_t size);
int verify_hash(char *chunk_hash, char *data);

#ifdef __cplusplus
}
#endif

#endif
