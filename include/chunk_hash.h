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
 * and the non-hash rest of chunk.h, so the peer links without chunk.o
 * (csrc/chunk_file.c):
 *   read_chunk                chunk.h:46  (chunk.c:93-115)   hash column -> peer's vector
 *   find_chunk_idx_from_hash  chunk.h:47  (chunk.c:123-160)  (size_t)-1 when absent
 *   seek_to_chunk_pos         chunk.h:48  (chunk.c:192-196)
 *   seek_to_packet_pos        chunk.h:49  (chunk.c:226-233)
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
 * caller-allocated chunk_hashes[i] (20 bytes each); returns the count.  A
 * regular file of more than 4 MiB (8 chunks) -- and any stream or pipe -- is
 * read into pinned host buffers and hashed in device batches on the gfx950
 * kernels; a regular file of at most 4 MiB (BASELINE config 1's tmp/C.tar is
 * 2 MiB) is hashed on the host by default, where its few serial chains take
 * ~0.2 ms each instead of a kernel launch plus ~6 ms per chain
 * (SHA1CHUNK_HOST_SMALL changes this: include/sha1chunk.h).
 *
 * shahash, get_chunk_hash, verify_hash and verify_chunk_hash hash ONE message
 * per call; by default on the host (a gfx950 device is still required),
 * SHA1CHUNK_HOST_SMALL=0 puts them on the kernels.  verify_chunk_hash serves
 * a master file from a digest table built in one device pass from its second
 * call on (SHA1CHUNK_MASTER_INDEX=0: per call). */
int make_chunks(FILE *fp, uint8_t **chunk_hashes);

void shahash(uint8_t *chr, int len, uint8_t *target);
void binary2hex(uint8_t *buf, int len, char *ascii);
void hex2binary(char *hex, int len, uint8_t *buf);
void verify_chunk_hash(FILE *f, char *requested_chunk_hash, size_t chunk_idx);
char *get_chunk_hash(char *chunk, size_t size);
int verify_hash(char *chunk_hash, char *data);

/* The peer's vector (utility.h:16-21); read_chunk appends through the
 * peer's own vec_add (utility.c:22-34), resolved from the executable. */
struct vector;
void read_chunk(char *filename, struct vector *v);
size_t find_chunk_idx_from_hash(char *chunk_hash, char *hash_chunk_file);
void seek_to_chunk_pos(FILE *f, size_t chunk_idx);
void seek_to_packet_pos(FILE *f, size_t chunk_idx, size_t last_sent_packet);

#ifdef __cplusplus
}
#endif

#endif
