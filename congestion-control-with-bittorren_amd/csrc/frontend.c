/*
 * frontend.c -- the thin C front end of libsha1chunk.so.
 *
 * libsha1chunk.so is what the peer and make-chunks link (INTEGRATION.md
 * section 2): the reference's hashing symbols (chunk_api.c, chunk_file.c)
 * and the sha1chunk_* batch API of include/sha1chunk.h.  It depends on libc
 * alone.  Every call that reaches the GPU is forwarded to the HIP backend,
 * libsha1chunk_hip.so (sha1_runtime.hip + the gfx950 kernels), which this
 * file dlopen()s from its own directory on the first such call -- so a
 * process that only makes single-message host calls (below) never loads the
 * HIP runtime: loading libamdhip64 costs ~11 ms and starting it 50-250 ms
 * (profiles/startup_r03.json), against the 6.5 ms the reference's whole
 * make-chunks takes on tmp/C.tar (BASELINE config 1).
 *
 * What the front end does itself:
 *   - the host path (sha1_host.c, x86 SHA extensions) for the reference's
 *     single-message calls by default -- shahash and its callers, the
 *     streaming trio, make_chunks on a regular file of at most 4 MiB -- and,
 *     under SHA1CHUNK_HOST_SMALL=<bytes>, for host batches and the batch-1
 *     verify queue of at most that many bytes (routing rules below);
 *   - the device check of those paths, without starting HIP: the kernel
 *     driver's KFD topology must list an accessible gfx950 agent
 *     (light_count);
 *   - the calling thread's device index and last error, which it hands to
 *     the backend (s1be_set_device) before forwarding.
 * Everything else is a forward.  There is no CPU fallback: without a device
 * every call fails with SHA1CHUNK_ENODEV, host paths included, and a missing
 * backend library fails the same way with the loader's message.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/sha1chunk.h"
#include "frontend.h"
#include "sha1_host.h"

#define FE_API __attribute__((visibility("default")))
#define FE_HIDDEN __attribute__((visibility("hidden")))

static __thread char t_err[512];
static __thread int t_dev = 0;       /* this thread's device (sha1chunk_set_device) */
static __thread int t_be_dev = -1;   /* the device last handed to the backend by this thread */

static int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t_err, sizeof t_err, fmt, ap);
    va_end(ap);
    return code;
}

/* ---------------------------------------------------------- the backend -- */
/* Every backend entry point: (return type, name, parameter list). */
#define BACKEND_FUNCS(X)                                                                          \
    X(int, hash_batch, (const void *, const uint64_t *, const uint32_t *, size_t, uint8_t *,       \
                        unsigned))                                                                \
    X(int, verify_batch, (const void *, const uint64_t *, const uint32_t *, size_t,               \
                          const uint8_t *, uint8_t *, unsigned))                                  \
    X(int, hash_device_async, (const void *, const uint64_t *, const uint32_t *, size_t,          \
                               uint8_t *, void *, int))                                           \
    X(int, hash_uniform_async, (const void *, uint32_t, size_t, uint8_t *, void *, int))          \
    X(int, compare_device_async, (const uint8_t *, const uint8_t *, size_t, uint8_t *, void *))   \
    X(long, hash_stream_sized, (sha1chunk_reader_fn, void *, sha1chunk_sink_fn, void *, uint64_t)) \
    X(long, hash_fd, (int, uint8_t *, size_t, size_t *))                                          \
    X(int, compress_blocks, (uint32_t *, const void *, size_t))                                   \
    X(int, finish, (const uint32_t *, uint64_t, const void *, uint32_t, uint8_t *))               \
    X(int, synth_fill_async, (void *, uint64_t, uint64_t, uint32_t, uint64_t, void *))            \
    X(int, synth_fill_ragged_async, (void *, const uint64_t *, const uint32_t *, uint64_t,        \
                                     uint64_t, uint64_t, void *))                                 \
    X(void *, vq_create, (size_t, uint32_t))                                                      \
    X(int, vq_submit, (void *, const void *, uint32_t, const uint8_t *, uint64_t))                \
    X(void *, vq_reserve, (void *, uint32_t))                                                     \
    X(int, vq_commit, (void *, void *, uint32_t, const uint8_t *, uint64_t))                      \
    X(int, vq_release, (void *, void *))                                                          \
    X(int, vq_flush, (void *))                                                                    \
    X(long, vq_poll, (void *, uint64_t *, uint8_t *, size_t, int))                                \
    X(size_t, vq_pending, (const void *))                                                         \
    X(void, vq_destroy, (void *))                                                                 \
    X(int, device_count, (void))                                                                  \
    X(int, set_device, (int))                                                                     \
    X(int, device_pci_bus_id, (int, char *, size_t))                                              \
    X(int, receive_cpus, (int, unsigned, void *, size_t, unsigned *))                             \
    X(const char *, last_error, (void))

#define BE_FIELD(ret, name, args) ret(*name) args;
static struct {
    BACKEND_FUNCS(BE_FIELD)
} BE;
static int be_ok = 0;
static char be_err[512];
static pthread_once_t be_once = PTHREAD_ONCE_INIT;

static void be_load(void) {
    Dl_info info;
    char path[4096];
    const char *env = getenv("SHA1CHUNK_BACKEND"); /* another build of the backend (tests) */
    if (env && *env) {
        snprintf(path, sizeof path, "%s", env);
    } else if (dladdr((void *)&be_load, &info) && info.dli_fname) {
        snprintf(path, sizeof path, "%s", info.dli_fname);
        char *slash = strrchr(path, '/');
        const size_t dir = slash ? (size_t)(slash - path) + 1 : 0;
        snprintf(path + dir, sizeof path - dir, "libsha1chunk_hip.so");
    } else {
        snprintf(path, sizeof path, "libsha1chunk_hip.so");
    }
    void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        snprintf(be_err, sizeof be_err, "HIP backend not loaded (%s)", dlerror());
        return;
    }
#define BE_SYM(ret, name, args)                                                                   \
    BE.name = (ret(*) args)dlsym(h, "s1be_" #name);                                               \
    if (!BE.name) {                                                                               \
        snprintf(be_err, sizeof be_err, "HIP backend %.400s lacks s1be_" #name, path);                \
        memset(&BE, 0, sizeof BE);                                                                \
        dlclose(h);                                                                               \
        return;                                                                                   \
    }
    BACKEND_FUNCS(BE_SYM)
    __atomic_store_n(&be_ok, 1, __ATOMIC_RELEASE); /* read without the once by set_device */
}

/* The backend, loaded; 0 or a negative error. */
static int backend(void) {
    pthread_once(&be_once, be_load);
    return be_ok ? SHA1CHUNK_OK : fail(SHA1CHUNK_ENODEV, "%s", be_err);
}

/* The backend with this thread's device selected in it. */
static int backend_dev(void) {
    int rc = backend();
    if (rc) return rc;
    if (t_be_dev != t_dev) {
        if ((rc = BE.set_device(t_dev)) < 0) return fail(rc, "%s", BE.last_error());
        t_be_dev = t_dev;
    }
    return SHA1CHUNK_OK;
}

/* Forward a call returning a negative code on failure, copying the
 * backend's message into this thread's error. */
#define FORWARD(type, call)                                                                       \
    do {                                                                                          \
        int rc_ = backend_dev();                                                                  \
        if (rc_) return rc_;                                                                      \
        type r_ = BE.call;                                                                        \
        if (r_ < 0) fail((int)r_, "%s", BE.last_error());                                         \
        return r_;                                                                                \
    } while (0)

/* --------------------------------------------------- host small-call path -- */
/* SHA1CHUNK_HOST_SMALL, read once per process, routes the calls that hash on
 * the host (sha1_host.c; a device is required either way, require_device):
 *
 *   unset      the default ("shahash() /
 *              verify_hash() keep a CPU path", "the streaming trio stays
 *              CPU"): the reference's synchronous single-message calls --
 *              shahash, get_chunk_hash, verify_hash, verify_chunk_hash's
 *              per-call path, and the SHA1Update / SHA1Final trio
 *              (sha1chunk_compress_blocks / sha1chunk_finish) -- are hashed
 *              on the host at any length, and make_chunks /
 *              sha1chunk_hash_fd on a regular file of at most REF_FILE_BYTES.
 *              One message is one serial chain: a lane of the GPU hashes it
 *              at ~85 MB/s, a CPU core at ~2.5 GB/s.  Every batch, device and
 *              verify-queue call runs on the kernels.
 *   "0"        every call on the kernels (the GPU tests pin this).
 *   "<bytes>"  the opt-in of rounds 3-4: every host call of at most that
 *              many bytes on the host -- batches, the trio, a regular file,
 *              a verify queue of batch 1 whose max length fits -- and larger
 *              ones on the kernels. */
#define REF_FILE_BYTES (4ull << 20) /* make-chunks on tmp/C.tar (2 MiB), BASELINE config 1 */
static uint64_t g_small;
static int g_small_set;
static pthread_once_t small_once = PTHREAD_ONCE_INIT;
static void small_init(void) {
    const char *e = getenv("SHA1CHUNK_HOST_SMALL");
    g_small_set = e != NULL && *e != 0;
    g_small = g_small_set ? strtoull(e, NULL, 10) : 0ull;
}
/* The explicit knob's byte count (0 when unset or "0"): batches and queues. */
static uint64_t host_small_bytes(void) {
    pthread_once(&small_once, small_init);
    return g_small;
}
/* 1 when a single-message reference call of `bytes` bytes hashes on the host. */
static int ref_on_host(uint64_t bytes) {
    pthread_once(&small_once, small_init);
    return g_small_set ? g_small != 0 && bytes <= g_small : 1;
}
/* 1 when make_chunks on a regular file of `bytes` bytes hashes on the host. */
static int file_on_host(uint64_t bytes) {
    pthread_once(&small_once, small_init);
    return g_small_set ? g_small != 0 && bytes <= g_small : bytes <= REF_FILE_BYTES;
}

/* Presence check of the host small-call paths without starting HIP: the KFD
 * topology lists gfx950 agents (gfx_target_version 90500) whose properties
 * and render node this process can open, next to an accessible /dev/kfd, and
 * no such GPU agent of another kind (the backend's rule that every device be
 * gfx950).  Agents this process cannot read (a container exposing one GPU
 * of a node) are not its devices.  Visibility masks are applied in the
 * order the runtime applies them (ROCR_VISIBLE_DEVICES to the agents, then
 * HIP/CUDA_VISIBLE_DEVICES and GPU_DEVICE_ORDINAL to what is left); a mask
 * this check cannot judge -- empty, an entry that is not a plain index
 * (UUIDs, "-1"), an index out of range or repeated -- leaves the answer to
 * the HIP probe.  Returns the device count, 0 for none, -1 to let HIP
 * decide. */
static int g_light = -1;
static char g_light_err[256];
static pthread_once_t light_once = PTHREAD_ONCE_INIT;

/* Number of devices a mask leaves of `visible`, or -1 when unsure. */
static int apply_mask(const char *m, int visible) {
    int count = 0;
    char seen[1024] = {0};
    if (!*m) return -1;
    for (const char *c = m;;) {
        const char *e = strchr(c, ',');
        const size_t len = e ? (size_t)(e - c) : strlen(c);
        if (len == 0 || len > 4) return -1;
        int idx = 0;
        for (size_t i = 0; i < len; ++i) {
            if (c[i] < '0' || c[i] > '9') return -1;
            idx = idx * 10 + (c[i] - '0');
        }
        if (idx >= visible || idx >= (int)sizeof seen || seen[idx]) return -1;
        seen[idx] = 1;
        ++count;
        if (!e) break;
        c = e + 1;
    }
    return count;
}

static void light_init(void) {
    if (access("/dev/kfd", R_OK | W_OK) != 0) {
        g_light = 0;
        snprintf(g_light_err, sizeof g_light_err, "no HIP device visible (/dev/kfd not accessible)");
        return;
    }
    const char *dir = "/sys/class/kfd/kfd/topology/nodes";
    int n = 0, readable = 0;
    for (int node = 0; node < 4096; ++node) {
        char path[128];
        snprintf(path, sizeof path, "%s/%d", dir, node);
        if (access(path, F_OK) != 0) break;
        snprintf(path, sizeof path, "%s/%d/properties", dir, node);
        FILE *f = fopen(path, "r");
        if (!f) continue; /* not this process's agent */
        ++readable;
        char key[64];
        unsigned long long val, target = 0, minor = 0;
        while (fscanf(f, "%63s %llu", key, &val) == 2) {
            if (!strcmp(key, "gfx_target_version")) target = val;
            if (!strcmp(key, "drm_render_minor")) minor = val;
        }
        fclose(f);
        if (target == 0) continue; /* a CPU agent */
        snprintf(path, sizeof path, "/dev/dri/renderD%llu", minor);
        if (access(path, R_OK | W_OK) != 0) continue;
        if (target != 90500) {
            g_light = 0;
            snprintf(g_light_err, sizeof g_light_err,
                     "a GPU agent is gfx_target_version %llu, this build targets gfx950 only", target);
            return;
        }
        ++n;
    }
    if (readable == 0) return; /* no readable topology: HIP decides */
    int visible = n;
    static const char *masks[] = {"ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                                  "GPU_DEVICE_ORDINAL"};
    for (size_t i = 0; i < sizeof masks / sizeof *masks; ++i) {
        const char *m = getenv(masks[i]);
        if (!m) continue;
        visible = apply_mask(m, visible);
        if (visible < 0) return;
    }
    g_light = visible;
    if (visible == 0) snprintf(g_light_err, sizeof g_light_err, "no HIP device visible (no accessible gfx950 agent)");
}

static int light_count(void) {
    pthread_once(&light_once, light_init);
    return g_light;
}

/* Logical devices over n physical ones (SHA1CHUNK_VIRTUAL_DEVICES, tests). */
static int logical_count(int n) {
    const char *e = getenv("SHA1CHUNK_VIRTUAL_DEVICES");
    if (!e) return n;
    const int k = atoi(e);
    return k < 1 ? 1 : (k > 64 ? 64 : k);
}

/* The library's contract for every call, the host paths included: a gfx950
 * device is present and the thread's device index is valid. */
static int require_device(void) {
    const int lc = light_count();
    if (lc < 0) {
        int rc = backend();
        if (rc) return rc;
        const int n = BE.device_count();
        if (n <= 0) return fail(SHA1CHUNK_ENODEV, "%s", BE.last_error());
        if (t_dev < 0 || t_dev >= n) return fail(SHA1CHUNK_EINVAL, "bad device %d", t_dev);
        return SHA1CHUNK_OK;
    }
    if (lc == 0) return fail(SHA1CHUNK_ENODEV, "%s", g_light_err);
    if (t_dev < 0 || t_dev >= logical_count(lc)) return fail(SHA1CHUNK_EINVAL, "bad device %d", t_dev);
    return SHA1CHUNK_OK;
}

/* Total bytes of a host batch, stopping once past `cap`. */
static uint64_t batch_bytes(const uint32_t *lengths, size_t n, uint64_t cap) {
    uint64_t total = 0;
    for (size_t i = 0; i < n && total <= cap; ++i) total += lengths[i];
    return total;
}

/* ================================================================ C ABI == */

FE_API int sha1chunk_device_count(void) {
    int rc = backend();
    if (rc) return rc;
    const int n = BE.device_count();
    if (n <= 0) fail(SHA1CHUNK_ENODEV, "%s", BE.last_error());
    return n;
}

FE_API int sha1chunk_set_device(int device) {
    /* With the backend loaded it validates against the HIP probe; before
     * that, against the KFD check (a host-only process stays HIP-free), and
     * the backend validates again at the first forwarded call. */
    const int lc = __atomic_load_n(&be_ok, __ATOMIC_ACQUIRE) ? -1 : light_count();
    if (lc < 0) {
        int rc = backend();
        if (rc) return rc;
        if ((rc = BE.set_device(device)) < 0) return fail(rc, "%s", BE.last_error());
        t_dev = t_be_dev = device;
        return SHA1CHUNK_OK;
    }
    if (lc == 0) return fail(SHA1CHUNK_ENODEV, "%s", g_light_err);
    if (device < 0 || device >= logical_count(lc))
        return fail(SHA1CHUNK_EINVAL, "device %d of %d", device, logical_count(lc));
    t_dev = device;
    return SHA1CHUNK_OK;
}

FE_API int sha1chunk_get_device(void) { return t_dev; }

FE_API const char *sha1chunk_last_error(void) { return t_err; }

FE_API const char *sha1chunk_version(void) { return "sha1chunk gfx950: lane,fused,split,mixed"; }

FE_API int sha1chunk_device_pci_bus_id(int device, char *buf, size_t len) {
    if (!buf || len == 0) return fail(SHA1CHUNK_EINVAL, "null buffer");
    int rc = backend();
    if (rc) return rc;
    if ((rc = BE.device_pci_bus_id(device, buf, len)) < 0) fail(rc, "%s", BE.last_error());
    return rc;
}

FE_API int sha1chunk_receive_cpus(int device, unsigned slot, void *mask, size_t len, unsigned *domains) {
    if (!mask) return fail(SHA1CHUNK_EINVAL, "null mask");
    if (len < sizeof(cpu_set_t)) return fail(SHA1CHUNK_EINVAL, "mask of %zu bytes, a cpu_set_t needs %zu", len,
                                             sizeof(cpu_set_t));
    int rc = backend();
    if (rc) return rc;
    if ((rc = BE.receive_cpus(device, slot, mask, len, domains)) < 0) fail(rc, "%s", BE.last_error());
    return rc;
}

FE_API int sha1chunk_hash_batch(const void *base, const uint64_t *offsets, const uint32_t *lengths,
                                size_t n, uint8_t *digests, unsigned flags) {
    if (n == 0) return SHA1CHUNK_OK;
    if (!base || !offsets || !lengths || !digests) return fail(SHA1CHUNK_EINVAL, "null pointer");
    if (n > 0xffffffffu) return fail(SHA1CHUNK_EINVAL, "n too large");
    const uint64_t small = host_small_bytes();
    if (!(flags & SHA1CHUNK_DEVICE) && small && batch_bytes(lengths, n, small) <= small) {
        int rc = require_device();
        if (rc) return rc;
        const uint8_t *b = (const uint8_t *)base;
        for (size_t i = 0; i < n; ++i) sha1host_digest(b + offsets[i], lengths[i], digests + 20 * i);
        return SHA1CHUNK_OK;
    }
    FORWARD(int, hash_batch(base, offsets, lengths, n, digests, flags));
}

FE_API int sha1chunk_verify_batch(const void *base, const uint64_t *offsets, const uint32_t *lengths,
                                  size_t n, const uint8_t *expected, uint8_t *mismatch, unsigned flags) {
    if (n == 0) return SHA1CHUNK_OK;
    if (!expected || !mismatch) return fail(SHA1CHUNK_EINVAL, "null pointer");
    const uint64_t small = host_small_bytes();
    if (!(flags & SHA1CHUNK_DEVICE) && small && lengths && batch_bytes(lengths, n, small) <= small) {
        if (!base || !offsets) return fail(SHA1CHUNK_EINVAL, "null pointer");
        int rc = require_device();
        if (rc) return rc;
        const uint8_t *b = (const uint8_t *)base;
        for (size_t i = 0; i < n; ++i) {
            uint8_t d[20];
            sha1host_digest(b + offsets[i], lengths[i], d);
            mismatch[i] = memcmp(d, expected + 20 * i, 20) != 0;
        }
        return SHA1CHUNK_OK;
    }
    FORWARD(int, verify_batch(base, offsets, lengths, n, expected, mismatch, flags));
}

/* One message (shahash, chunk.c:35-51, and the calls built on it), routed
 * like the other single-message reference calls (ref_on_host). */
FE_API int sha1chunk_digest(const void *msg, uint64_t len, uint8_t digest[20]) {
    if ((len && !msg) || !digest) return fail(SHA1CHUNK_EINVAL, "null pointer");
    if (ref_on_host(len)) {
        int rc = require_device();
        if (rc) return rc;
        sha1host_digest(msg, len, digest);
        return SHA1CHUNK_OK;
    }
    if (len > 0xffffffffull) return fail(SHA1CHUNK_EINVAL, "a message above 4 GiB - 1 on the kernels");
    const uint64_t off = 0;
    const uint32_t n = (uint32_t)len;
    FORWARD(int, hash_batch(len ? msg : digest, &off, &n, 1, digest, SHA1CHUNK_HOST));
}

/* make_chunks's master-file index (chunk_api.c): a device pass over the
 * whole file pays off only where make_chunks itself would use the device. */
FE_HIDDEN int fe_file_on_host(uint64_t bytes) { return file_on_host(bytes); }

FE_API int sha1chunk_hash_device_async(const void *d_base, const uint64_t *d_offsets,
                                       const uint32_t *d_lengths, size_t n, uint8_t *d_digests,
                                       void *stream, int kernel) {
    FORWARD(int, hash_device_async(d_base, d_offsets, d_lengths, n, d_digests, stream, kernel));
}

FE_API int sha1chunk_hash_uniform_async(const void *d_base, uint32_t chunk_len, size_t n,
                                        uint8_t *d_digests, void *stream, int kernel) {
    FORWARD(int, hash_uniform_async(d_base, chunk_len, n, d_digests, stream, kernel));
}

FE_API int sha1chunk_compare_device_async(const uint8_t *d_digests, const uint8_t *d_expected,
                                          size_t n, uint8_t *d_mismatch, void *stream) {
    FORWARD(int, compare_device_async(d_digests, d_expected, n, d_mismatch, stream));
}

FE_API long sha1chunk_hash_stream(sha1chunk_reader_fn reader, void *reader_ctx, sha1chunk_sink_fn sink,
                                  void *sink_ctx) {
    FORWARD(long, hash_stream_sized(reader, reader_ctx, sink, sink_ctx, 0));
}

FE_API long sha1chunk_hash_stream_sized(sha1chunk_reader_fn reader, void *reader_ctx,
                                        sha1chunk_sink_fn sink, void *sink_ctx, uint64_t size_hint) {
    FORWARD(long, hash_stream_sized(reader, reader_ctx, sink, sink_ctx, size_hint));
}

/* A regular file of at most SHA1CHUNK_HOST_SMALL bytes (make-chunks on a
 * small file, BASELINE config 1's tmp/C.tar): read and hashed here chunk by
 * chunk, as the reference's fread + shahash loop does (chunk.c:15-27).  The
 * fd is left at the end of what was read. */
static long hash_file_host(int fd, off_t pos, off_t end, uint8_t *digests, size_t max_chunks) {
    uint8_t *buf = (uint8_t *)malloc(SHA1CHUNK_CHUNK_LEN);
    if (!buf) return fail(SHA1CHUNK_ENOMEM, "file buffer");
    long n = 0;
    while (pos < end) {
        const size_t want = (size_t)(end - pos < SHA1CHUNK_CHUNK_LEN ? end - pos : SHA1CHUNK_CHUNK_LEN);
        size_t got = 0;
        while (got < want) {
            const ssize_t r = pread(fd, buf + got, want - got, pos + (off_t)got);
            if (r < 0) {
                if (errno == EINTR) continue;
                free(buf);
                return fail(SHA1CHUNK_EIO, "file read error");
            }
            if (r == 0) break; /* the file shrank under us */
            got += (size_t)r;
        }
        if (got == 0) break;
        uint8_t dig[20];
        sha1host_digest(buf, got, dig);
        if ((size_t)n < max_chunks && digests) memcpy(digests + 20 * (size_t)n, dig, 20);
        ++n;
        pos += (off_t)got;
        if (got < want) break;
    }
    free(buf);
    (void)lseek(fd, pos, SEEK_SET);
    return n;
}

FE_API long sha1chunk_hash_fd(int fd, uint8_t *digests, size_t max_chunks, size_t *total_chunks) {
    struct stat st;
    const off_t pos = lseek(fd, 0, SEEK_CUR);
    if (pos >= 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode) &&
        file_on_host((uint64_t)(st.st_size > pos ? st.st_size - pos : 0))) {
        int rc = require_device();
        if (rc) return rc;
        const long n = hash_file_host(fd, pos, st.st_size > pos ? st.st_size : pos, digests, max_chunks);
        if (n < 0) return n;
        if (total_chunks) *total_chunks = (size_t)n;
        return (size_t)n < max_chunks ? n : (long)max_chunks;
    }
    FORWARD(long, hash_fd(fd, digests, max_chunks, total_chunks));
}

FE_API int sha1chunk_compress_blocks(uint32_t state[5], const void *blocks, size_t nblocks) {
    if (!state || (nblocks && !blocks)) return fail(SHA1CHUNK_EINVAL, "null pointer");
    if (nblocks == 0) return SHA1CHUNK_OK;
    if (nblocks * 64 > 0xffffffffull) return fail(SHA1CHUNK_EINVAL, "too many blocks");
    if (ref_on_host(nblocks * 64)) {
        int rc = require_device();
        if (rc) return rc;
        sha1host_compress(state, blocks, nblocks);
        return SHA1CHUNK_OK;
    }
    FORWARD(int, compress_blocks(state, blocks, nblocks));
}

FE_API int sha1chunk_finish(const uint32_t state[5], uint64_t prefix_bytes, const void *tail,
                            uint32_t tail_len, uint8_t digest[20]) {
    if (!state || !digest || (tail_len && !tail) || tail_len >= 64)
        return fail(SHA1CHUNK_EINVAL, "bad argument");
    if (ref_on_host(tail_len)) {
        int rc = require_device();
        if (rc) return rc;
        sha1host_finish(state, prefix_bytes, tail, tail_len, digest);
        return SHA1CHUNK_OK;
    }
    FORWARD(int, finish(state, prefix_bytes, tail, tail_len, digest));
}

FE_API int sha1chunk_synth_fill_async(void *d_dst, uint64_t first, uint64_t count, uint32_t chunk_len,
                                      uint64_t seed, void *stream) {
    FORWARD(int, synth_fill_async(d_dst, first, count, chunk_len, seed, stream));
}

FE_API int sha1chunk_synth_fill_ragged_async(void *d_base, const uint64_t *d_offsets,
                                             const uint32_t *d_lengths, uint64_t first, uint64_t count,
                                             uint64_t seed, void *stream) {
    FORWARD(int, synth_fill_ragged_async(d_base, d_offsets, d_lengths, first, count, seed, stream));
}

/* ------------------------------------------------------------ verify queue -- */
/* A queue is either a backend queue (the persistent drain or batch
 * launches) or, with batch 1 and SHA1CHUNK_HOST_SMALL >= max_chunk_len, the
 * batch-size-1 host queue: each submit hashes and compares its chunk here
 * before returning; results wait in a FIFO for poll(). */
struct sha1chunk_vq {
    void *be; /* backend queue, or NULL: the host batch-1 queue */
    uint32_t maxlen;
    pthread_mutex_t mu; /* the host queue's lock (the backend locks its own) */
    uint64_t *tags;     /* host queue results: a ring of cap entries */
    uint8_t *mis;
    size_t head, count, cap;
    void **held; /* host queue reservations (malloc'd), not yet released */
    size_t nheld, capheld;
};

/* Index of reservation `buf` in the host queue, or -1. */
static long host_held(sha1chunk_vq *q, const void *buf) {
    for (size_t i = 0; i < q->nheld; ++i)
        if (q->held[i] == buf) return (long)i;
    return -1;
}

static int host_push(sha1chunk_vq *q, uint64_t tag, uint8_t mismatch) {
    if (q->count == q->cap) {
        const size_t cap = q->cap ? 2 * q->cap : 64;
        uint64_t *t = (uint64_t *)malloc(cap * sizeof *t);
        uint8_t *m = (uint8_t *)malloc(cap);
        if (!t || !m) {
            free(t);
            free(m);
            return fail(SHA1CHUNK_ENOMEM, "vq: result ring");
        }
        for (size_t i = 0; i < q->count; ++i) {
            t[i] = q->tags[(q->head + i) % q->cap];
            m[i] = q->mis[(q->head + i) % q->cap];
        }
        free(q->tags);
        free(q->mis);
        q->tags = t;
        q->mis = m;
        q->head = 0;
        q->cap = cap;
    }
    const size_t at = (q->head + q->count) % q->cap;
    q->tags[at] = tag;
    q->mis[at] = mismatch;
    ++q->count;
    return SHA1CHUNK_OK;
}

FE_API sha1chunk_vq *sha1chunk_vq_create(size_t batch, uint32_t max_chunk_len) {
    if (batch == 0 || batch > (1u << 20) || max_chunk_len == 0) {
        fail(SHA1CHUNK_EINVAL, "vq: batch 1..2^20 and max_chunk_len > 0 required");
        return NULL;
    }
    sha1chunk_vq *q = (sha1chunk_vq *)calloc(1, sizeof *q);
    if (!q) {
        fail(SHA1CHUNK_ENOMEM, "vq: allocation failed");
        return NULL;
    }
    q->maxlen = max_chunk_len;
    pthread_mutex_init(&q->mu, NULL);
    /* The batch-size-1 host path ("keep the CPU path for
     * batch size 1"): a peer verifying one chunk at a time, as
     * packet_handler.c:472 -> job.c:217 does, would otherwise wait for one
     * lane's serial chain (~6 ms per 512 KiB) per chunk.  Opt-in through the
     * same knob as the other small calls; a device is still required. */
    if (batch == 1 && max_chunk_len <= host_small_bytes()) {
        if (require_device()) {
            free(q);
            return NULL;
        }
        return q;
    }
    if (backend_dev() || !(q->be = BE.vq_create(batch, max_chunk_len))) {
        if (be_ok) fail(SHA1CHUNK_ENOMEM, "%s", BE.last_error());
        free(q);
        return NULL;
    }
    return q;
}

FE_API int sha1chunk_vq_submit(sha1chunk_vq *q, const void *chunk, uint32_t len, const uint8_t expected[20],
                               uint64_t tag) {
    if (!q || (len && !chunk) || !expected) return fail(SHA1CHUNK_EINVAL, "vq: null argument");
    if (q->be) FORWARD(int, vq_submit(q->be, chunk, len, expected, tag));
    if (len > q->maxlen) return fail(SHA1CHUNK_EINVAL, "vq: chunk of %u bytes > max %u", len, q->maxlen);
    uint8_t dig[20];
    sha1host_digest(chunk, len, dig);
    pthread_mutex_lock(&q->mu);
    const int rc = host_push(q, tag, memcmp(dig, expected, 20) != 0 ? 1 : 0);
    pthread_mutex_unlock(&q->mu);
    return rc;
}

FE_API void *sha1chunk_vq_reserve(sha1chunk_vq *q, uint32_t len) {
    if (!q) {
        fail(SHA1CHUNK_EINVAL, "vq: null queue");
        return NULL;
    }
    if (q->be) {
        if (backend_dev()) return NULL;
        void *p = BE.vq_reserve(q->be, len);
        if (!p) fail(SHA1CHUNK_ENOMEM, "%s", BE.last_error());
        return p;
    }
    /* the host queue hashes in place at commit: a plain host buffer */
    if (len > q->maxlen) {
        fail(SHA1CHUNK_EINVAL, "vq: reservation of %u bytes > max %u", len, q->maxlen);
        return NULL;
    }
    void *p = malloc(len ? len : 1);
    if (!p) {
        fail(SHA1CHUNK_ENOMEM, "vq: reservation of %u bytes", len);
        return NULL;
    }
    pthread_mutex_lock(&q->mu);
    if (q->nheld == q->capheld) {
        const size_t cap = q->capheld ? 2 * q->capheld : 16;
        void **h = (void **)realloc(q->held, cap * sizeof *h);
        if (!h) {
            pthread_mutex_unlock(&q->mu);
            free(p);
            fail(SHA1CHUNK_ENOMEM, "vq: reservation table");
            return NULL;
        }
        q->held = h;
        q->capheld = cap;
    }
    q->held[q->nheld++] = p;
    pthread_mutex_unlock(&q->mu);
    return p;
}

FE_API int sha1chunk_vq_commit(sha1chunk_vq *q, void *buf, uint32_t len, const uint8_t expected[20],
                               uint64_t tag) {
    if (!q || !buf || !expected) return fail(SHA1CHUNK_EINVAL, "vq: null argument");
    if (q->be) FORWARD(int, vq_commit(q->be, buf, len, expected, tag));
    if (len > q->maxlen) return fail(SHA1CHUNK_EINVAL, "vq: chunk of %u bytes > max %u", len, q->maxlen);
    pthread_mutex_lock(&q->mu);
    const long at = host_held(q, buf);
    pthread_mutex_unlock(&q->mu);
    if (at < 0) return fail(SHA1CHUNK_EINVAL, "vq: %p is not a reserved buffer", buf);
    uint8_t dig[20];
    sha1host_digest(buf, len, dig);
    pthread_mutex_lock(&q->mu);
    const int rc = host_push(q, tag, memcmp(dig, expected, 20) != 0 ? 1 : 0);
    pthread_mutex_unlock(&q->mu);
    return rc;
}

FE_API int sha1chunk_vq_release(sha1chunk_vq *q, void *buf) {
    if (!q || !buf) return fail(SHA1CHUNK_EINVAL, "vq: null argument");
    if (q->be) FORWARD(int, vq_release(q->be, buf));
    pthread_mutex_lock(&q->mu);
    const long at = host_held(q, buf);
    if (at >= 0) q->held[at] = q->held[--q->nheld];
    pthread_mutex_unlock(&q->mu);
    if (at < 0) return fail(SHA1CHUNK_EINVAL, "vq: %p is not a reserved buffer", buf);
    free(buf);
    return SHA1CHUNK_OK;
}

FE_API int sha1chunk_vq_flush(sha1chunk_vq *q) {
    if (!q) return fail(SHA1CHUNK_EINVAL, "vq: null queue");
    if (q->be) FORWARD(int, vq_flush(q->be));
    return SHA1CHUNK_OK;
}

FE_API long sha1chunk_vq_poll(sha1chunk_vq *q, uint64_t *tags, uint8_t *mismatch, size_t max, int wait) {
    if (!q || (max && (!tags || !mismatch))) return fail(SHA1CHUNK_EINVAL, "vq: null argument");
    if (q->be) FORWARD(long, vq_poll(q->be, tags, mismatch, max, wait));
    size_t n = 0;
    pthread_mutex_lock(&q->mu);
    while (n < max && q->count) {
        tags[n] = q->tags[q->head];
        mismatch[n] = q->mis[q->head];
        q->head = (q->head + 1) % q->cap;
        --q->count;
        ++n;
    }
    pthread_mutex_unlock(&q->mu);
    return (long)n;
}

FE_API size_t sha1chunk_vq_pending(const sha1chunk_vq *q) {
    if (!q) return 0;
    if (q->be) return BE.vq_pending(q->be);
    pthread_mutex_lock((pthread_mutex_t *)&q->mu);
    const size_t n = q->count;
    pthread_mutex_unlock((pthread_mutex_t *)&q->mu);
    return n;
}

FE_API void sha1chunk_vq_destroy(sha1chunk_vq *q) {
    if (!q) return;
    if (q->be) BE.vq_destroy(q->be);
    for (size_t i = 0; i < q->nheld; ++i) free(q->held[i]);
    free(q->held);
    free(q->tags);
    free(q->mis);
    pthread_mutex_destroy(&q->mu);
    free(q);
}
