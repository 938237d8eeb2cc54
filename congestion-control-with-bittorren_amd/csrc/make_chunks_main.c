/*
 * make_chunks_main.c -- the `make-chunks <file>` tool (BASELINE config 1)
 * linked against libsha1chunk.so instead of the reference's sha.o/chunk.o.
 *
 * Behaviour of /root/reference/make_chunks.c:14-76: chunk count from the
 * file size, rounded up to whole 512 KiB chunks; one 20-byte buffer per
 * chunk; make_chunks(); then one "%d %s\n" line per chunk with the lowercase
 * hex digest (chunk.c:57-63).  Usage errors and unreadable files print to
 * stderr and exit(-1), as the reference does.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "../../include/chunk_hash.h"
#include "../../include/sha.h"

int main(int argc, char *argv[]) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <input-file>", argv[0]);
        exit(-1);
    }
    const char *path = argv[1];
    struct stat st;
    FILE *fp = fopen(path, "rb");
    if (fp == NULL || stat(path, &st) != 0) {
        fprintf(stderr, "Can't stat the file %s: %s\n", path, strerror(errno));
        exit(-1);
    }
    const long long nchunks = ((long long)st.st_size + BT_CHUNK_SIZE - 1) / BT_CHUNK_SIZE;
    /* A one-shot process pins its pipeline ring once and never reuses it
     * (~0.1-0.2 s per GiB pinned, profiles/init_cost_r02.jsonl), so smaller
     * slots start sooner, while 512 MiB slots stream ~8 % faster per GiB.
     * Measured through this CLI on page-cached files (tools/file_bench.py
     * --cli-slot-ab, profiles/cli_slot_r02.json): 128 MiB slots are ahead by
     * a constant ~0.3 s at 8, 16 and 24 GiB (0.67 / 0.83 / 1.05 s against
     * 0.99 / 1.14 / 1.33 s, medians of 3), and the per-GiB slopes (0.0234 vs
     * 0.0218 s/GiB) put the crossover near 190 GiB.  An explicit
     * SHA1CHUNK_STREAM_SLOT_MIB wins. */
    setenv("SHA1CHUNK_STREAM_SLOT_MIB", st.st_size < (192LL << 30) ? "128" : "512", 0);
    uint8_t **hashes = (uint8_t **)malloc((size_t)(nchunks > 0 ? nchunks : 1) * sizeof *hashes);
    uint8_t *store = (uint8_t *)malloc((size_t)(nchunks > 0 ? nchunks : 1) * SHA1_HASH_SIZE);
    if (hashes == NULL || store == NULL) {
        fprintf(stderr, "Out of memory!!!");
        exit(-1);
    }
    for (long long i = 0; i < nchunks; ++i) hashes[i] = store + i * SHA1_HASH_SIZE;

    const int made = make_chunks(fp, hashes);
    char ascii[SHA1_HASH_SIZE * 2 + 1];
    for (int i = 0; i < made; ++i) {
        hex2ascii(hashes[i], SHA1_HASH_SIZE, ascii);
        printf("%d %s\n", i, ascii);
    }
    free(store);
    free(hashes);
    fclose(fp);
    return 0;
}
