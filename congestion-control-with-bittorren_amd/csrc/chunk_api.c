/*
 * chunk_api.c -- the reference's C hashing API, re-implemented on top of the
 * gfx950 batch engine (sha1_runtime.hip).  Same names, signatures, return
 * conventions and stdout side effects as /root/reference:
 *
 *   SHA1Init / SHA1Update / SHA1Final   sha.h:58-60, sha.c:149-558
 *   make_chunks                         chunk.c:15-27
 *   shahash                             chunk.c:35-51
 *   binary2hex / hex2binary             chunk.c:57-85
 *   get_chunk_hash                      chunk.c:168-185
 *   verify_chunk_hash                   chunk.c:204-217
 *   verify_hash                         job.c:217-228
 *
 * Routing (frontend.c, SHA1CHUNK_HOST_SMALL): the single-message calls --
 * shahash and what is built on it (get_chunk_hash, verify_hash, the per-call
 * verify_chunk_hash), the SHA1Update/SHA1Final trio -- and make_chunks on a
 * regular file of at most 4 MiB hash on the host by default (sha1_host.c;
 * SURVEY.md 7.1 step 2, 8(b)), since one message is one serial chain that a
 * GPU lane runs ~30x slower than a CPU core; make_chunks on larger files and
 * streams, and the master-file index, run on the gfx950 kernels
 * (sha1_runtime.hip), as everything does under SHA1CHUNK_HOST_SMALL=0.  A
 * device is required either way.  The reference
 * reports failures by printing and exit(-1) (chunk.c:171-178); these void
 * functions do the same when the engine fails (no device, HIP error), so a
 * missing GPU is loud, never a silent CPU fallback.
 */
#include <ctype.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "../../include/chunk_hash.h"
#include "../../include/sha.h"
#include "../../include/sha1chunk.h"
#include "frontend.h"

#define CHUNK_LEN 524288 /* constants.h:14 */

static void die(const char *what, int rc) {
    fprintf(stderr, "sha1chunk: %s failed (%d): %s\n", what, rc, sha1chunk_last_error());
    exit(-1);
}

static void check(const char *what, int rc) {
    if (rc < 0) die(what, rc);
}

/* ------------------------------------------------------- sha.h streaming -- */

void SHA1Init(SHA1Context *sc) {
    sc->totalLength = 0;
    sc->hash[0] = 0x67452301u;
    sc->hash[1] = 0xefcdab89u;
    sc->hash[2] = 0x98badcfeu;
    sc->hash[3] = 0x10325476u;
    sc->hash[4] = 0xc3d2e1f0u;
    sc->bufferLength = 0;
}

/* Whole blocks per device call when streaming a large update. */
#define STREAM_BLOCKS (1u << 20) /* 64 MiB */

void SHA1Update(SHA1Context *sc, const void *vdata, uint32_t len) {
    const uint8_t *data = (const uint8_t *)vdata;
    sc->totalLength += (uint64_t)len * 8u;
    if (sc->bufferLength) {
        uint32_t take = 64u - sc->bufferLength;
        if (take > len) take = len;
        memcpy(sc->buffer.bytes + sc->bufferLength, data, take);
        sc->bufferLength += take;
        data += take;
        len -= take;
        if (sc->bufferLength < 64u) return;
        check("SHA1Update", sha1chunk_compress_blocks(sc->hash, sc->buffer.bytes, 1));
        sc->bufferLength = 0;
    }
    uint32_t nblocks = len / 64u;
    while (nblocks) {
        uint32_t nb = nblocks < STREAM_BLOCKS ? nblocks : STREAM_BLOCKS;
        check("SHA1Update", sha1chunk_compress_blocks(sc->hash, data, nb));
        data += (size_t)nb * 64u;
        len -= nb * 64u;
        nblocks -= nb;
    }
    if (len) {
        memcpy(sc->buffer.bytes, data, len);
        sc->bufferLength = len;
    }
}

void SHA1Final(SHA1Context *sc, uint8_t hash[SHA1_HASH_SIZE]) {
    uint8_t digest[SHA1_HASH_SIZE];
    const uint64_t bytes = sc->totalLength / 8u;
    check("SHA1Final", sha1chunk_finish(sc->hash, bytes - sc->bufferLength, sc->buffer.bytes,
                                        sc->bufferLength, digest));
    /* Leave the context as the reference does after its padding updates:
     * chaining value = digest words, nothing staged, length padded. */
    for (int i = 0; i < SHA1_HASH_WORDS; ++i)
        sc->hash[i] = ((uint32_t)digest[4 * i] << 24) | ((uint32_t)digest[4 * i + 1] << 16) |
                      ((uint32_t)digest[4 * i + 2] << 8) | (uint32_t)digest[4 * i + 3];
    sc->totalLength = ((bytes + 9u + 63u) / 64u) * 512u;
    sc->bufferLength = 0;
    if (hash) memcpy(hash, digest, SHA1_HASH_SIZE);
}

/* --------------------------------------------------------- chunk.h API -- */

void shahash(uint8_t *str, int len, uint8_t *hash) {
    if (len < 0) {
        fprintf(stderr, "sha1chunk: shahash: negative length %d\n", len);
        exit(-1);
    }
    check("shahash", sha1chunk_digest(str, (uint64_t)len, hash));
}

void binary2hex(uint8_t *buf, int len, char *hex) {
    static const char digits[] = "0123456789abcdef";
    for (int i = 0; i < len; ++i) {
        hex[2 * i] = digits[buf[i] >> 4];
        hex[2 * i + 1] = digits[buf[i] & 15];
    }
    hex[2 * (len > 0 ? len : 0)] = 0;
}

static uint8_t nibble(char c) {
    /* chunk.c:68-72: toupper, digits map to c-'0', letters to c-'A'+10
     * (no validation, same as the reference). */
    c = (char)toupper((unsigned char)c);
    return (uint8_t)(c <= '9' ? c - '0' : c - ('A' - 10));
}

void hex2binary(char *hex, int len, uint8_t *buf) {
    for (int i = 0; i < len; i += 2) buf[i / 2] = (uint8_t)((nibble(hex[i]) << 4) | nibble(hex[i + 1]));
}

/* fread-driven reader for the device pipeline (chunk.c:22 reads the FILE*
 * from its current position to EOF in 512 KiB pieces). */
static size_t file_reader(void *ctx, void *dst, size_t n) {
    FILE *fp = (FILE *)ctx;
    size_t got = fread(dst, 1, n, fp);
    if (got == 0 && ferror(fp)) return (size_t)-1;
    return got;
}

/* Digests land in the caller's chunk_hashes[i] (20 bytes each, allocated by
 * the caller from the file size as make_chunks.c:32-45 does). */
static void hashes_sink(void *ctx, size_t first, const uint8_t *dig, size_t count) {
    uint8_t **out = (uint8_t **)ctx;
    for (size_t j = 0; j < count; ++j) memcpy(out[first + j], dig + 20 * j, 20);
}

int make_chunks(FILE *fp, uint8_t **chunk_hashes) {
    /* Regular file: hash from the stream position to EOF through
     * sha1chunk_hash_fd (multi-threaded pread into the pinned slots). */
    struct stat st;
    const int fd = fileno(fp);
    const off_t pos = ftello(fp);
    if (fd >= 0 && pos >= 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
        const size_t cap = st.st_size > pos ? (size_t)((st.st_size - pos + CHUNK_LEN - 1) / CHUNK_LEN) : 0;
        uint8_t *tmp = (uint8_t *)malloc(20 * (cap ? cap : 1));
        if (!tmp) {
            fprintf(stderr, "Failed to allocate memory\n");
            exit(-1);
        }
        /* stdio may have read ahead of `pos` (and a seek inside its buffer
         * does not move the fd), so set the fd offset explicitly */
        if (lseek(fd, pos, SEEK_SET) != pos) {
            fprintf(stderr, "sha1chunk: make_chunks: lseek failed\n");
            exit(-1);
        }
        size_t total = 0;
        long n = sha1chunk_hash_fd(fd, tmp, cap, &total);
        if (n < 0) die("make_chunks", (int)n);
        for (long i = 0; i < n; ++i) memcpy(chunk_hashes[i], tmp + 20 * i, 20);
        free(tmp);
        fseeko(fp, 0, SEEK_END); /* where the reference's fread loop leaves it */
        return (int)n;
    }
    long n = sha1chunk_hash_stream(file_reader, fp, hashes_sink, chunk_hashes);
    if (n < 0) die("make_chunks", (int)n);
    return (int)n;
}

char *get_chunk_hash(char *chunk, size_t size) {
    uint8_t hash[SHA1_HASH_SIZE];
    char *chunk_hash = (char *)malloc(SHA1_HASH_SIZE * 2 + 1);
    if (!chunk_hash) {
        fprintf(stderr, "Failed to allocate memory\n");
        exit(-1);
    }
    /* chunk.c:179 and :182 print these two lines around the hash. */
    fprintf(stdout, "calculating chunk hash for a chunk of size %d\n", (int)size);
    shahash((uint8_t *)chunk, (int)size, hash);
    hex2ascii(hash, SHA1_HASH_SIZE, chunk_hash);
    fprintf(stdout, "the ascii of calculated hash is %s\n", chunk_hash);
    return chunk_hash;
}

/* Master-file digest index.  The sender verifies every
 * GET'd chunk against the master data file (packet_handler.c:434 ->
 * chunk.c:204-217), re-reading and re-hashing 512 KiB per request, while
 * every send session opens the same file afresh (reliable_udp.c:180).  From
 * the second verify against one file on, a single streamed device pass
 * digests all of its chunks -- each zero-padded to CHUNK_LEN, exactly what
 * this verify hashes -- and later requests are a table lookup.  The table is
 * keyed on (st_dev, st_ino, st_size, st_mtim, st_ctim) and rebuilt when any
 * of them changes.  st_ctim moves on every write and on every utime(), so an
 * in-place rewrite that keeps the size and restores the mtime is caught.  A
 * write landing in the same timestamp tick as the keyed one would not be, so
 * a file whose ctime is less than SHA1CHUNK_MASTER_SETTLE_MS (default 2000)
 * old is never served from the table: it is re-read and re-hashed per call,
 * as the reference does (chunk.c:204-217).  Non-regular files and
 * SHA1CHUNK_MASTER_INDEX=0 keep the per-call path. */
typedef struct {
    dev_t dev;
    ino_t ino;
    off_t size;
    struct timespec mtime;
    struct timespec ctime;
} file_key;

static struct {
    pthread_mutex_t mu;
    file_key key;
    int seen;        /* verifies against `key` so far */
    uint8_t *digest; /* nchunks x 20 B once built */
    size_t nchunks;
} master = {.mu = PTHREAD_MUTEX_INITIALIZER};

typedef struct {
    int fd;
    off_t pos, size, padded;
} padded_reader;

/* Reads the file from offset 0 and then zeros up to the next CHUNK_LEN
 * boundary, so the last chunk is hashed at full length like chunk.c:206-208. */
static size_t padded_read(void *ctx, void *dst, size_t n) {
    padded_reader *r = (padded_reader *)ctx;
    size_t done = 0;
    while (done < n && r->pos < r->padded) {
        size_t want = n - done;
        if (r->pos < r->size) {
            if ((off_t)want > r->size - r->pos) want = (size_t)(r->size - r->pos);
            ssize_t got = pread(r->fd, (char *)dst + done, want, r->pos);
            if (got < 0) return (size_t)-1;
            if (got == 0) { /* file shrank under us: pad the rest */
                r->size = r->pos;
                continue;
            }
            want = (size_t)got;
        } else {
            if ((off_t)want > r->padded - r->pos) want = (size_t)(r->padded - r->pos);
            memset((char *)dst + done, 0, want);
        }
        done += want;
        r->pos += (off_t)want;
    }
    return done;
}

static int same_key(const file_key *a, const file_key *b) {
    return a->dev == b->dev && a->ino == b->ino && a->size == b->size &&
           a->mtime.tv_sec == b->mtime.tv_sec && a->mtime.tv_nsec == b->mtime.tv_nsec &&
           a->ctime.tv_sec == b->ctime.tv_sec && a->ctime.tv_nsec == b->ctime.tv_nsec;
}

/* 1 when the file's last change (ctime) is older than the settle time. */
static int settled(const struct stat *st) {
    const char *env = getenv("SHA1CHUNK_MASTER_SETTLE_MS");
    const long long settle_ms = env ? atoll(env) : 2000;
    struct timespec now;
    if (settle_ms <= 0) return 1;
    if (clock_gettime(CLOCK_REALTIME, &now)) return 0;
    const long long age_ms = (long long)(now.tv_sec - st->st_ctim.tv_sec) * 1000 +
                             (now.tv_nsec - st->st_ctim.tv_nsec) / 1000000;
    return age_ms >= settle_ms;
}

/* The master file's digest table: every chunk through sha1chunk_hash_fd
 * (parallel pread into the pinned ring, the device pipeline make_chunks
 * uses: 8 GiB in ~0.17 s against ~0.9 s for one reader thread,
 * profiles/bench_r06*.log `master_verify`), the fd's offset put back after
 * (the caller's FILE* keeps its position); a short last chunk is then
 * rehashed zero-padded to CHUNK_LEN, which is what verify_chunk_hash hashes
 * (padded_read).  1 when the table covers exactly the n chunks keyed. */
static int build_index(int fd, const struct stat *st, size_t n, uint8_t *tab) {
    const off_t save = lseek(fd, 0, SEEK_CUR);
    if (save < 0 || lseek(fd, 0, SEEK_SET) != 0) return 0;
    size_t total = 0;
    const long got = sha1chunk_hash_fd(fd, tab, n, &total);
    const int back = lseek(fd, save, SEEK_SET) == save;
    if (got < 0) die("verify_chunk_hash index", (int)got);
    if (!back || (size_t)got != n || total != n) return 0;
    const off_t tail = st->st_size - (off_t)(n - 1) * CHUNK_LEN;
    if (tail < CHUNK_LEN) {
        padded_reader r = {fd, (off_t)(n - 1) * CHUNK_LEN, st->st_size, (off_t)n * CHUNK_LEN};
        uint8_t *buf = (uint8_t *)malloc(CHUNK_LEN);
        if (!buf) return 0;
        const size_t have = padded_read(&r, buf, CHUNK_LEN);
        int rc = have == CHUNK_LEN && r.size == st->st_size ? sha1chunk_digest(buf, CHUNK_LEN, tab + 20 * (n - 1)) : 1;
        free(buf);
        if (rc < 0) die("verify_chunk_hash index", rc);
        if (rc) return 0;
    }
    return 1;
}

/* Copies chunk `idx`'s digest from the index into out20 and the file size
 * into *size; 0 if unavailable. */
static int master_lookup(FILE *f, size_t idx, uint8_t out20[20], off_t *size) {
    const char *env = getenv("SHA1CHUNK_MASTER_INDEX");
    if (env && env[0] == '0') return 0;
    struct stat st;
    int fd = fileno(f);
    if (fd < 0 || fstat(fd, &st) || !S_ISREG(st.st_mode) || st.st_size <= 0) return 0;
    if (fe_file_on_host((uint64_t)st.st_size)) return 0; /* small file: per-call host hash */
    if (!settled(&st)) return 0; /* changed just now: re-read and re-hash */
    file_key k = {st.st_dev, st.st_ino, st.st_size, st.st_mtim, st.st_ctim};
    int hit = 0;
    pthread_mutex_lock(&master.mu);
    if (!same_key(&k, &master.key)) {
        free(master.digest);
        master.digest = NULL;
        master.nchunks = 0;
        master.key = k;
        master.seen = 0;
    }
    if (++master.seen >= 2 && !master.digest) {
        const size_t n = (size_t)((st.st_size + CHUNK_LEN - 1) / CHUNK_LEN);
        uint8_t *tab = (uint8_t *)malloc(20 * n);
        if (tab && build_index(fd, &st, n, tab)) {
            master.digest = tab;
            master.nchunks = n;
        } else {
            free(tab);
        }
    }
    if (master.digest && idx < master.nchunks) {
        memcpy(out20, master.digest + 20 * idx, 20);
        *size = st.st_size;
        hit = 1;
    }
    pthread_mutex_unlock(&master.mu);
    return hit;
}

void verify_chunk_hash(FILE *f, char *requested_chunk_hash, size_t chunk_idx) {
    /* chunk.c:204-217.  Deviation: the reference hashes a full CHUNK_LEN
     * buffer even past EOF (uninitialised tail); here the unread tail is
     * zero so the result is deterministic.  Offsets are 64-bit. */
    char *calculated;
    uint8_t hash[SHA1_HASH_SIZE];
    off_t size = 0;
    if (master_lookup(f, chunk_idx, hash, &size)) {
        /* same observable behaviour as the per-call path: the two lines
         * get_chunk_hash prints, and the stream left after the chunk */
        calculated = (char *)malloc(SHA1_HASH_SIZE * 2 + 1);
        if (!calculated) {
            fprintf(stderr, "Failed to allocate memory\n");
            exit(-1);
        }
        fprintf(stdout, "calculating chunk hash for a chunk of size %d\n", CHUNK_LEN);
        hex2ascii(hash, SHA1_HASH_SIZE, calculated);
        fprintf(stdout, "the ascii of calculated hash is %s\n", calculated);
        const off_t after = (off_t)(chunk_idx + 1) * CHUNK_LEN; /* idx < nchunks: starts before EOF */
        fseeko(f, after < size ? after : size, SEEK_SET);
    } else {
        fseeko(f, (off_t)chunk_idx * CHUNK_LEN, SEEK_SET);
        char *buffer = (char *)calloc(1, CHUNK_LEN);
        if (!buffer) {
            fprintf(stderr, "Failed to allocate memory\n");
            exit(-1);
        }
        if (fread(buffer, 1, CHUNK_LEN, f) == 0 && ferror(f)) {
            fprintf(stderr, "sha1chunk: verify_chunk_hash: read error\n");
            exit(-1);
        }
        calculated = get_chunk_hash(buffer, CHUNK_LEN);
        free(buffer);
    }
    if (strncmp(calculated, requested_chunk_hash, strlen(calculated))) {
        fprintf(stderr, "Unmatched chunk hashes, requested hash %s, calculated hash %s\n",
                requested_chunk_hash, calculated);
        exit(-1);
    }
    free(calculated);
}

int verify_hash(char *chunk_hash, char *data) {
    char *calculated = get_chunk_hash(data, CHUNK_LEN);
    fprintf(stdout, "calculated hash is %s\n", calculated);
    fprintf(stdout, "correct hash is %s\n", chunk_hash);
    const int mismatch = strncmp(chunk_hash, calculated, strlen(calculated)) != 0;
    free(calculated);
    return mismatch;
}
