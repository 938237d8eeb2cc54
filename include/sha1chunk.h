/*
 * sha1chunk.h -- the batch entry points of the MI355X SHA-1 chunk engine
 * (libsha1chunk.so).  Plain C ABI: pointers, sizes, a `void *` HIP stream.
 *
 * These are the one new interface SURVEY.md 7.1 step 2 asks for.  The
 * reference has no batch API: every digest in /root/reference is produced by
 * a serial shahash() call (chunk.c:23 from make_chunks, chunk.c:180 from
 * get_chunk_hash <- job.c:218 verify_hash and chunk.c:208 verify_chunk_hash).
 * sha1chunk_hash_batch() replaces a loop of those calls; the reference-
 * signature functions in chunk_hash.h / sha.h are implemented on top of it.
 *
 * The library is two files: libsha1chunk.so (what callers link: these
 * symbols, a thin C front end on libc alone) and libsha1chunk_hip.so (the
 * HIP runtime and gfx950 kernels), which the front end loads from its own
 * directory on the first call that needs the GPU -- so a process whose
 * calls all take the host small-call path below never starts HIP.
 *
 * Error convention: 0 on success, a negative SHA1CHUNK_E* code otherwise
 * (never exit()); sha1chunk_last_error() returns a thread-local message.
 * There is no CPU fallback: without a usable gfx950 device every call
 * fails with SHA1CHUNK_ENODEV, the host-routed calls below included.
 *
 * Routing.  One message is one serial chain of
 * compressions: a GPU lane runs it at ~85 MB/s, a CPU core with the x86 SHA
 * extensions at ~2.5 GB/s.  So by default the reference's single-message
 * calls hash on the host: sha1chunk_compress_blocks / sha1chunk_finish (the
 * SHA1Update / SHA1Final trio), shahash and what is built on it
 * (get_chunk_hash, verify_hash, verify_chunk_hash's per-call path), and
 * sha1chunk_hash_fd (make_chunks) on a regular file of at most 4 MiB --
 * one 512 KiB chunk in ~0.2 ms instead of one lane's ~6 ms.  Every batch,
 * device and verify-queue entry point, and make_chunks on larger files and
 * streams, runs on the gfx950 kernels.  SHA1CHUNK_HOST_SMALL in the
 * environment (read once per process) changes this: "0" puts every call on
 * the kernels; "<bytes>" hashes every host call of at most that many bytes
 * on the host (batches, the trio, a regular file, a verify queue of batch 1
 * whose max length fits) and larger ones on the kernels.
 */
#ifndef SHA1CHUNK_H
#define SHA1CHUNK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHA1CHUNK_DIGEST_LEN 20
#define SHA1CHUNK_CHUNK_LEN 524288 /* constants.h:14 CHUNK_LEN */

enum {
    SHA1CHUNK_OK = 0,
    SHA1CHUNK_EINVAL = -1, /* bad argument                                   */
    SHA1CHUNK_ENODEV = -2, /* no HIP device / runtime                        */
    SHA1CHUNK_ENOMEM = -3, /* device or pinned allocation failed             */
    SHA1CHUNK_EHIP = -4,   /* HIP runtime error (see sha1chunk_last_error)   */
    SHA1CHUNK_EALIGN = -5, /* digest (4 B) / synthetic (8 B) buffer misaligned */
    SHA1CHUNK_EIO = -6     /* read error on a file descriptor                */
};

/* Where the buffers of sha1chunk_hash_batch / sha1chunk_verify_batch live. */
#define SHA1CHUNK_HOST 0u        /* host memory: staged through pinned buffers  */
#define SHA1CHUNK_DEVICE 1u      /* device memory of the current device         */
#define SHA1CHUNK_ALL_DEVICES 2u /* HOST only: shard the chunk list over every
                                    visible device, one host thread per device */

/* Kernel choice for the device entry points (AUTO picks by batch shape:
 * the split kernel up to two groups of 64 chunks per CU, the fused kernel
 * beyond; a ragged batch is hashed longest-first, and with more groups than
 * CUs through the mixed kernel, whose device-side plan splits the groups
 * between the one-group split shape and the fused kernel). */
enum {
    SHA1CHUNK_KERNEL_AUTO = 0,
    SHA1CHUNK_KERNEL_LANE = 1,  /* one lane per chunk, per-lane loads; any alignment   */
    SHA1CHUNK_KERNEL_FUSED = 2, /* one lane per chunk, schedule + rounds in registers,
                                   two 128-byte stages of per-lane loads ahead       */
    SHA1CHUNK_KERNEL_SPLIT = 3  /* schedule-producer + round-consumer wave pairs        */
};

/* digests[i*20 .. i*20+19] = SHA-1(base[offsets[i] .. offsets[i]+lengths[i])).
 * Synchronous.  Host mode accepts any alignment and overlapping chunks. */
int sha1chunk_hash_batch(const void *base, const uint64_t *offsets, const uint32_t *lengths,
                         size_t n, uint8_t *digests, unsigned flags);

/* One message's digest, routed as the reference's single-message calls are
 * (shahash, chunk.c:35-51, is this call): on the host by default, on the
 * kernels under SHA1CHUNK_HOST_SMALL=0 or above an explicit threshold
 * (routing above).  len <= 2^32 - 1 on the kernels. */
int sha1chunk_digest(const void *msg, uint64_t len, uint8_t digest[20]);

/* mismatch[i] = 0 if the digest of chunk i equals expected[i*20..], else 1
 * (the verify_hash() convention of job.c:217-228). */
int sha1chunk_verify_batch(const void *base, const uint64_t *offsets, const uint32_t *lengths,
                           size_t n, const uint8_t *expected, uint8_t *mismatch, unsigned flags);

/* Device-resident, asynchronous on `stream` (a hipStream_t, NULL = default).
 * All pointers are device pointers.  Returns after enqueueing.  Chunks may
 * start at any byte and lie anywhere in the buffer.  With KERNEL_AUTO (the
 * split shapes and the mixed kernel, whose loads are shared across the
 * wave) placement costs nothing and 16-byte aligned starts are ~10 % faster
 * in the fused shapes.  A forced KERNEL_FUSED or KERNEL_LANE loads one chunk
 * per lane and is layout-sensitive: chunks scattered far apart thrash the
 * address-translation cache (~2.8x slower measured). */
int sha1chunk_hash_device_async(const void *d_base, const uint64_t *d_offsets,
                                const uint32_t *d_lengths, size_t n, uint8_t *d_digests,
                                void *stream, int kernel);

/* Same for n equal chunks of chunk_len bytes laid back to back at d_base
 * (the make_chunks layout): no offset/length arrays needed. */
int sha1chunk_hash_uniform_async(const void *d_base, uint32_t chunk_len, size_t n,
                                 uint8_t *d_digests, void *stream, int kernel);

/* Device compare of computed vs expected digests -> mismatch bytes. */
int sha1chunk_compare_device_async(const uint8_t *d_digests, const uint8_t *d_expected,
                                   size_t n, uint8_t *d_mismatch, void *stream);

/* Hash a byte stream in 512 KiB chunks (the last one at its true length,
 * as make_chunks does, chunk.c:22-23) through a ring of pinned slots:
 * read -> H2D -> hash -> D2H, slots overlapping.  `reader` fills up to n bytes of dst
 * (pinned memory) and returns the count, 0 at end of stream, or (size_t)-1
 * on error; `sink` receives each completed run of digests in order.
 * Returns the number of chunks (>= 0) or a negative error. */
typedef size_t (*sha1chunk_reader_fn)(void *ctx, void *dst, size_t n);
typedef void (*sha1chunk_sink_fn)(void *ctx, size_t first_chunk, const uint8_t *digests,
                                  size_t count);
long sha1chunk_hash_stream(sha1chunk_reader_fn reader, void *reader_ctx, sha1chunk_sink_fn sink,
                           void *sink_ctx);
/* Same, when the caller knows how many bytes the reader will deliver
 * (size_hint > 0): slots are sized to the input (a small file does not
 * allocate 512 MiB pinned slots; a mid-size one is spread over all slots). */
long sha1chunk_hash_stream_sized(sha1chunk_reader_fn reader, void *reader_ctx,
                                 sha1chunk_sink_fn sink, void *sink_ctx, uint64_t size_hint);
/* File-descriptor convenience: up to max_chunks digests into `digests`;
 * *total_chunks (optional) gets the file's chunk count.  Hashes from the
 * fd's current offset and leaves it at the end of what was read.  A regular
 * file is read with parallel pread; with SHA1CHUNK_FILE_DEVICES=all (or a
 * count) in the environment it is split into contiguous chunk-aligned ranges
 * over that many devices, one pipeline each (make_chunks and the
 * make-chunks CLI go through here). */
long sha1chunk_hash_fd(int fd, uint8_t *digests, size_t max_chunks, size_t *total_chunks);

/* Streaming support for SHA1Update/SHA1Final: compress nblocks whole 64-byte
 * blocks (host memory) into the chaining value state[5]. */
int sha1chunk_compress_blocks(uint32_t state[5], const void *blocks, size_t nblocks);
/* Finish a stream: state[5] after prefix_bytes hashed bytes, then tail_len
 * (< 64) buffered bytes -> padded final block(s) -> 20-byte digest. */
int sha1chunk_finish(const uint32_t state[5], uint64_t prefix_bytes, const void *tail,
                     uint32_t tail_len, uint8_t digest[20]);

/* Synthetic corpus generated on the device: chunk c, 64-bit
 * LE word w = splitmix64(seed ^ (c << 24) ^ w), chunks first..first+count-1
 * written back to back, chunk_len bytes each. */
int sha1chunk_synth_fill_async(void *d_dst, uint64_t first, uint64_t count, uint32_t chunk_len,
                               uint64_t seed, void *stream);
/* Ragged variant: chunk first+i of d_lengths[i] bytes at d_base + d_offsets[i]
 * (device arrays; every d_base + d_offsets[i] 8-byte aligned). */
int sha1chunk_synth_fill_ragged_async(void *d_base, const uint64_t *d_offsets,
                                      const uint32_t *d_lengths, uint64_t first, uint64_t count,
                                      uint64_t seed, void *stream);

/* ---- Asynchronous verify queue (the peer's receive path) --
 * The reference verifies each reassembled chunk synchronously inside its
 * select() loop (packet_handler.c:469-472 -> job.c:217 verify_hash).  A queue
 * verifies them asynchronously instead: submit() copies the chunk into pinned
 * memory (the caller may reuse its buffer at once) with its expected digest
 * and a tag, and poll() returns finished (tag, mismatch) pairs, mismatch
 * following verify_hash: 0 = match, 1 = mismatch -> re-GET.
 *
 * Default: a persistent drain kernel.  The chunks go into a ring in pinned
 * host memory (SHA1CHUNK_VQ_RING_MIB, default 1024) and are published in
 * groups of up to min(batch, 64); while fewer groups are in flight than the
 * drain has workgroups, each chunk goes out at once.  The copy engine
 * stages each group into a mirror of the ring in device memory
 * (SHA1CHUNK_VQ_DMA=0: the drain reads the pinned ring over PCIe instead).
 * The drain, one workgroup on each of SHA1CHUNK_VQ_CUS CUs (default 64;
 * all queues on a device share at most SHA1CHUNK_VQ_CU_BUDGET CUs, default
 * half, and queues beyond it launch per batch), hashes and compares the
 * groups and writes the results back to host memory; a workgroup exits
 * after SHA1CHUNK_VQ_IDLE_MS (default 20) without a claim or after
 * SHA1CHUNK_VQ_LIFE_MS (default 4) of work, and the next call starts it
 * again.  A lone chunk comes back after its own serial chain, with no
 * batch to fill and no flush.
 *
 * SHA1CHUNK_VQ_MODE=batch: batches are launched as kernels.  Once `batch`
 * submissions are pending (or on flush) the batch is hashed and
 * compared on the device asynchronously -- while two earlier batches are
 * still on the device a batch keeps growing by whole batches (up to 4 x
 * batch, at most 512; SHA1CHUNK_VQ_GROW=0 disables) and goes at the first
 * whole batch after one finishes (a submit or a poll notices); whole batches
 * therefore always come back through poll() without a flush.  Three batch
 * sets are in flight at once.
 *
 * batch == 1 with SHA1CHUNK_HOST_SMALL >= max_chunk_len (explicit opt-in): the
 * batch-size-1 host path.  Each submit hashes and compares its chunk on the
 * host before returning (0.2 ms per 512 KiB instead of a 6 ms device chain);
 * poll() returns the results in submission order.  A device is still
 * required.
 *
 * A queue's own streams (its drains' launch slots and its copy stream) are
 * created at a stream priority of their own (SHA1CHUNK_VQ_PRIO, default
 * "low"), so HIP maps them to other hardware queues than the caller's
 * default-priority streams: a persistent drain never sits in front of the
 * caller's own kernels.  Measured: a config-2 batch (4096 x 512 KiB)
 * launched on a fresh stream while four queues are continuously fed took
 * 6.25-6.47 ms against 6.02 solo (12-26 ms with the queues' streams at the
 * default priority); tests/test_gpu_vq_zero_copy.py::
 * test_wait_behind_busy_drains_is_bounded checks that the median stays
 * within 1.5x of solo.
 *
 * Every queue call takes the queue's lock, so several threads (receive
 * sessions) may share one queue; a call that waits (for ring space, or
 * poll(wait)) and submit()'s copy release the lock meanwhile, so the other
 * threads' calls go on.  destroy() must not overlap any other call on the
 * queue.  Persistent drains of all queues on one device hold at most
 * SHA1CHUNK_VQ_CU_BUDGET CUs (default half the device); a queue created
 * when that budget is spent uses batch launches.  The copy of submit() runs
 * on the calling thread, which has just filled the chunk and holds it in its
 * caches (SHA1CHUNK_VQ_THREADS=N > 1 splits it over N threads, the caller
 * and N - 1 helper threads per queue that spin briefly between submissions,
 * when no other submit is using them: measured slower, 1 / 4 receive threads
 * 7.7 / 26.8 GiB/s at N = 4 against 18.5 / 46.7 at the default 1);
 * reserve/commit has no copy.  Helper threads run on the CPUs of the GPU's
 * NUMA node (SHA1CHUNK_NUMA=off: anywhere); HIP's pinned allocation puts the
 * ring's pages on that node already (measured, every page).
 * Measured on 16384 x 512 KiB host chunks from 4 receive threads on the
 * GPU's node, one per L3 domain, pieces copied from a cache-resident
 * source: 45-48 GiB/s reserve/commit and submit alike, pass to pass, 0.88x
 * the PCIe copy rate; the same from a DRAM-resident source (DESIGN.md
 * section 6, profiles/vq_l3b.jsonl, bench_r06k*.log). */
typedef struct sha1chunk_vq sha1chunk_vq;
/* NULL on failure (sha1chunk_last_error() says why). */
sha1chunk_vq *sha1chunk_vq_create(size_t batch, uint32_t max_chunk_len);
int sha1chunk_vq_submit(sha1chunk_vq *q, const void *chunk, uint32_t len,
                        const uint8_t expected[20], uint64_t tag);
/* Zero-copy receive.  reserve() hands out a buffer of len (<= max_chunk_len)
 * bytes inside the queue's pinned ring -- the peer's per-session receive
 * buffer (reliable_udp.c:121 recv_session->data), filled in place as DATA
 * packets arrive (reliable_udp.c:339) -- and commit() verifies it where it
 * lies, with no copy (the call at packet_handler.c:472).  The buffer must
 * not change between commit() and its result; it stays valid after the
 * result is polled, until release() (after the caller copied the verified
 * chunk into its job buffer, reliable_udp.c:696-709, or dropped it).  A
 * reservation may also be released without a commit.  Unreleased buffers
 * hold ring space.  reserve() and submit() wait (bounded, SHA1CHUNK_VQ_WAIT_S,
 * default 120 s) for room while in-flight chunks or other threads'
 * reservations still filling hold it; they fail (NULL, resp.
 * SHA1CHUNK_ENOMEM) rather than wait when the ring's oldest region is the
 * calling thread's own reservation, not committed or not released -- room
 * only that thread could free -- or, after a 2 ms grace, any thread's
 * verified buffer whose result nobody has polled and released yet (room only
 * a poll() and release() free: when every receive thread waits in reserve()
 * nobody polls).  On NULL, poll, release and retry.  In batch mode and
 * on the batch-1 host path the buffer is ordinary host memory (commit
 * copies it, resp. hashes it in place). */
void *sha1chunk_vq_reserve(sha1chunk_vq *q, uint32_t len);
int sha1chunk_vq_commit(sha1chunk_vq *q, void *buf, uint32_t len, const uint8_t expected[20],
                        uint64_t tag);
int sha1chunk_vq_release(sha1chunk_vq *q, void *buf);
int sha1chunk_vq_flush(sha1chunk_vq *q);
/* Up to max finished results; wait != 0 blocks until everything submitted
 * before the call has finished (later submissions from other threads are not
 * waited for).  Returns the number written (>= 0) or a negative error. */
long sha1chunk_vq_poll(sha1chunk_vq *q, uint64_t *tags, uint8_t *mismatch, size_t max, int wait);
/* Submitted but not yet returned by poll(). */
size_t sha1chunk_vq_pending(const sha1chunk_vq *q);
void sha1chunk_vq_destroy(sha1chunk_vq *q);

/* Device management. */
int sha1chunk_device_count(void);
int sha1chunk_set_device(int device);
int sha1chunk_get_device(void);
/* PCI address ("dddd:bb:dd.f") of logical device `device`'s physical GPU:
 * tells apart the devices SHA1CHUNK_ALL_DEVICES / SHA1CHUNK_FILE_DEVICES
 * shard over (several logical devices map to one GPU only under
 * SHA1CHUNK_VIRTUAL_DEVICES, a test knob). */
int sha1chunk_device_pci_bus_id(int device, char *buf, size_t len);
/* Where a receive thread feeding a verify queue on `device` should run:
 * writes into `mask` (a Linux cpu_set_t, len >= sizeof(cpu_set_t); the rest
 * of len is zeroed) the CPUs of one L3 domain (one CCD on the MI355X boxes'
 * EPYC hosts) of the device's NUMA node, within the caller's affinity mask;
 * receive thread `slot` gets domain slot mod their count, so threads 0..k-1
 * land on k different domains.  *domains (if not NULL) receives that count.
 * With SHA1CHUNK_NUMA=off, or the node unknown, the domains of every allowed
 * CPU.  Returns the number of CPUs in the mask, or a negative error.  Use:
 *   cpu_set_t cs;
 *   if (sha1chunk_receive_cpus(sha1chunk_get_device(), i, &cs, sizeof cs, NULL) > 0)
 *       pthread_setaffinity_np(thread_i, sizeof cs, &cs);
 * Measured (16384 x 512 KiB, 4 receive threads): one
 * per domain held submit at 27.7-29.6 GiB/s where threads floating over the
 * node gave 23.8-36.2 run to run (the copy then on helper threads; on the
 * receive thread since, both run 46-47). */
int sha1chunk_receive_cpus(int device, unsigned slot, void *mask, size_t len, unsigned *domains);
/* Last error text of this thread ("" if none). */
const char *sha1chunk_last_error(void);
/* "gfx950:<kernels>" build identity, for logs. */
const char *sha1chunk_version(void);

#ifdef __cplusplus
}
#endif

#endif
