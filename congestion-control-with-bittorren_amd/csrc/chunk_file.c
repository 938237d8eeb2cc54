/*
 * chunk_file.c -- the non-hash half of the reference's chunk.h, so that the
 * peer's Makefile can drop chunk.o together with sha.o and link
 * libsha1chunk.so instead.  No hashing happens
 * here; these are the chunk-file readers and file-position helpers the peer
 * calls around the hash path:
 *
 *   read_chunk                chunk.h:46  chunk.c:93-115   hash column of a chunk file
 *   find_chunk_idx_from_hash  chunk.h:47  chunk.c:123-160  index of a hash in a
 *                                                          chunk / master-chunk file
 *   seek_to_chunk_pos         chunk.h:48  chunk.c:192-196
 *   seek_to_packet_pos        chunk.h:49  chunk.c:226-233
 *
 * Same names, signatures, stdout/stderr lines and exit(-1) on an unopenable
 * file (utility.c:261-268 Fopen) as the reference.  Deviations, each one a
 * place where the reference reads uninitialised memory:
 *   - read_chunk hands vec_add a zero-filled copy of the hash token, so the
 *     bytes past its NUL (which vec_add copies, ele_size = CHUNK_HASH_SIZE,
 *     and vec_diff/vec_common memcmp, utility.c:117) are zeros instead of
 *     whatever followed the line in getline's buffer.  A digit line without
 *     a second token is skipped as a comment line instead of crashing.
 *   - find_chunk_idx_from_hash reads chunk 0's index on the master file's
 *     header line ("File: <path> Chunks:0 <hex>", tmp/C.masterchunks:1) as
 *     the number after "Chunks:" instead of the first four bytes of that
 *     token reinterpreted as an int (chunk.c:138); a hash that is not in the
 *     file returns (size_t)-1 instead of an uninitialised value; the getline
 *     buffer starts NULL (chunk.c:125 passes an uninitialised pointer).
 *   - seek_to_chunk_pos seeks with a 64-bit offset (chunk.c:193 truncates
 *     it to uint32_t).
 * Same rules as congestion-control-with-bittorren_amd/chunkfile.py.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include "../../include/chunk_hash.h"

#define CHUNK_LEN 524288         /* constants.h:14 */
#define UDP_MAX_PACK_SIZE 1500   /* constants.h:11 */
#define PACK_HEADER_BASE_LEN 16  /* constants.h:16 */

/* The peer's vector (utility.h:16-21).  The library only reads ele_size to
 * size the copy it hands to the peer's own vec_add (utility.c:22-34), which
 * resolves from the peer executable at load time. */
struct vector_head {
    int ele_size;
    int len;
    int size;
    void *val;
};
extern void vec_add(struct vector *vec, void *ele) __attribute__((weak));

static FILE *open_or_exit(const char *filename) {
    FILE *f = fopen(filename, "r");
    if (!f) { /* utility.c:263-266 */
        fprintf(stderr, "Failed to open file %s \n", filename);
        exit(-1);
    }
    return f;
}

void read_chunk(char *filename, struct vector *v) {
    if (!vec_add) {
        fprintf(stderr, "sha1chunk: read_chunk needs the peer's vec_add (utility.c)\n");
        exit(-1);
    }
    FILE *f = open_or_exit(filename);
    const int ele_size = ((const struct vector_head *)v)->ele_size;
    char *line = NULL;
    size_t cap = 0;
    while (getline(&line, &cap, f) != -1) {
        char *save = NULL;
        char *token = strtok_r(line, " ", &save);
        char *hash = (token && isdigit((unsigned char)token[0])) ? strtok_r(NULL, " ", &save) : NULL;
        if (!hash) {
            fprintf(stdout, "Comment line in chunk file\n");
            continue;
        }
        size_t n = strlen(hash);
        if (n && hash[n - 1] == '\n') hash[--n] = '\0';
        const size_t sz = (size_t)(ele_size > 0 ? ele_size : 0) > n + 1 ? (size_t)ele_size : n + 1;
        char *ele = (char *)calloc(1, sz);
        if (!ele) {
            fprintf(stderr, "Failed to allocate memory\n");
            exit(-1);
        }
        memcpy(ele, hash, n);
        vec_add(v, ele);
        free(ele);
    }
    free(line);
    fclose(f);
}

/* chunk.c:140,149: strcmp(t, hash) == 0 || strstr(t, hash) != NULL */
static int hex_matches(const char *token, const char *chunk_hash) {
    return strcmp(token, chunk_hash) == 0 || strstr(token, chunk_hash) != NULL;
}

size_t find_chunk_idx_from_hash(char *chunk_hash, char *hash_chunk_file) {
    FILE *f = open_or_exit(hash_chunk_file);
    char *line = NULL;
    size_t cap = 0;
    size_t found = (size_t)-1;
    while (found == (size_t)-1 && getline(&line, &cap, f) != -1) {
        char *tok[4] = {NULL, NULL, NULL, NULL};
        char *save = NULL;
        int nt = 0;
        for (char *t = strtok_r(line, " ", &save); t && nt < 4; t = strtok_r(NULL, " ", &save))
            tok[nt++] = t;
        if (nt == 0) continue;
        if (!isdigit((unsigned char)tok[0][0])) {
            /* header line: File: <path> Chunks:<idx> <hex> */
            if (nt >= 4 && strncmp(tok[2], "Chunks:", 7) == 0 && hex_matches(tok[3], chunk_hash))
                found = (size_t)strtoull(tok[2] + 7, NULL, 10);
        } else if (nt >= 2 && hex_matches(tok[1], chunk_hash)) {
            found = (size_t)strtoull(tok[0], NULL, 10);
        }
    }
    free(line);
    fclose(f);
    return found;
}

void seek_to_chunk_pos(FILE *f, size_t chunk_idx) {
    fseeko(f, (off_t)chunk_idx * CHUNK_LEN, SEEK_SET);
}

void seek_to_packet_pos(FILE *f, size_t chunk_idx, size_t last_sent_packet) {
    const off_t off = (off_t)chunk_idx * CHUNK_LEN +
                      (off_t)(UDP_MAX_PACK_SIZE - PACK_HEADER_BASE_LEN) * (off_t)last_sent_packet;
    fseeko(f, off, SEEK_SET);
}
