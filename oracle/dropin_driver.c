/*
 * dropin_driver.c -- TEST INFRASTRUCTURE ONLY (oracle/Makefile `dropin`).
 *
 * Drives the reference peer's own receive-side code, compiled unmodified
 * from /root/reference and linked without chunk.o and sha.o against
 * libsha1chunk.so.  Nothing here hashes; every
 * digest comes from the library through the reference's call sites:
 *
 *   job.c:56-62     job_init: read_chunk of the GET chunk file and of the
 *                   has-chunk file, vec_common (utility.c) of the two
 *   job.c:80-99     populate_chunks_to_download -> find_chunk_idx_from_hash
 *                   on the master chunk file
 *   job.c:217-228   verify_hash -> get_chunk_hash -> shahash (the check
 *                   packet_handler.c:472 runs on every reassembled chunk)
 *
 * usage: dropin_driver <data file> <GET chunk file> <master chunk file> <has-chunk file>
 * prints  COMMON <n>
 *         TODO <hash40> <chunk_id> <own>        (one per GET chunk)
 *         VERIFY <i> <intact rc> <corrupted rc> (verify_hash on chunk i of the
 *                                                data file, zero-padded to
 *                                                CHUNK_LEN, then with one bit
 *                                                flipped)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "chunk.h"
#include "job.h"
#include "utility.h"

int main(int argc, char **argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s <data> <get chunks> <master chunks> <has chunks>\n", argv[0]);
        return 2;
    }
    vector want, has;
    init_vector(&want, CHUNK_HASH_SIZE);
    init_vector(&has, CHUNK_HASH_SIZE);
    read_chunk(argv[2], &want);
    read_chunk(argv[4], &has);
    vector *common = vec_common(&want, &has);
    printf("COMMON %d\n", common->len);

    job_t job;
    memset(&job, 0, sizeof job);
    strncpy(job.master_chunk_file, argv[3], BT_FILENAME_LEN - 1);
    vector todo;
    init_vector(&todo, sizeof(chunk_to_download));
    populate_chunks_to_download(&todo, &want, common, &job);
    for (int i = 0; i < todo.len; ++i) {
        chunk_to_download *c = (chunk_to_download *)vec_get(&todo, i);
        printf("TODO %.40s %zu %d\n", c->chunk_hash, c->chunk_id, c->own);
    }

    FILE *f = fopen(argv[1], "rb");
    if (!f) {
        perror(argv[1]);
        return 2;
    }
    char *buf = (char *)malloc(CHUNK_LEN);
    for (int i = 0; i < want.len; ++i) {
        memset(buf, 0, CHUNK_LEN);
        if (fread(buf, 1, CHUNK_LEN, f) == 0) break;
        char *hash = (char *)vec_get(&want, i);
        const int intact = verify_hash(hash, buf);
        buf[(i * 7919) % CHUNK_LEN] ^= 0x10;
        const int corrupted = verify_hash(hash, buf);
        printf("VERIFY %d %d %d\n", i, intact, corrupted);
    }
    free(buf);
    fclose(f);
    vec_free(common);
    free(common);
    return 0;
}
