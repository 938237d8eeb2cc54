// sha1_runtime.hip -- the HIP backend of libsha1chunk.so (built into
// libsha1chunk_hip.so): the device half of the C-ABI batch entry points of
// include/sha1chunk.h, exported as s1be_* and reached only through the thin
// C front end (frontend.c), which dlopen()s this library on the first call
// that needs the GPU and handles the host small-call paths itself.
//
// Per device: one compute stream per pipeline slot, a device arena and a
// pinned host arena for each of two slots, so that packing/reading batch b+1
// on the host, its H2D copy, the kernel of batch b and the D2H of digests
// overlap.  Everything that hashes runs on the GPU; the host only moves
// bytes and bookkeeping (sorting by length, packing, scattering digests).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <emmintrin.h>
#include <functional>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

#include "../../include/sha1chunk.h"
#include "part_pool.hpp"
#include "sha1_kernels.h"

namespace {
using s1host::PartPool;

// First line of a sysfs file ("" if it cannot be read).
std::string sysfs_line(const char* path) {
    char buf[4096] = {0};
    if (FILE* f = fopen(path, "r")) {
        if (!fgets(buf, sizeof buf, f)) buf[0] = 0;
        fclose(f);
    }
    return buf;
}

// The CPUs of HIP device `id`'s NUMA node (the numa_node of its PCI device)
// within `allowed`, into *out; their count, 0 when the node is unknown.
int device_node_cpus(int id, const cpu_set_t& allowed, cpu_set_t* out) {
    CPU_ZERO(out);
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, sizeof bdf, id) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    for (char* c = bdf; *c; ++c) *c = static_cast<char>(tolower(static_cast<unsigned char>(*c)));
    char path[160];
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bdf);
    const std::string nl = sysfs_line(path);
    const int node = nl.empty() ? -1 : atoi(nl.c_str());
    if (node < 0) return 0;
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    return s1host::cpus_from_list(sysfs_line(path).c_str(), allowed, out);
}

bool numa_off() {
    const char* e = getenv("SHA1CHUNK_NUMA");
    return e && (!strcmp(e, "off") || !strcmp(e, "0"));
}

// Host CPUs near HIP device `id`: the CPUs of its NUMA node within this
// process's affinity mask.  The library's helper threads -- the pageable-
// batch packing, the file pipeline's preads into pinned slots, the verify
// queue's split copies when asked for (SHA1CHUNK_VQ_THREADS) -- run there,
// beside the pinned memory they write (hipHostMalloc already places it on
// the GPU's node: profiles/vq_place_r06*.jsonl) and the GPU that reads it.
// SHA1CHUNK_NUMA=off (or 0) leaves them to the scheduler.  nullptr: no
// placement (off, one node, node unknown, or none of its CPUs allowed, or
// fewer than four).
const cpu_set_t* near_cpus(int id) {
    struct Near {
        std::once_flag once;
        bool ok = false;
        cpu_set_t set;
    };
    static Near near[64];
    if (id < 0 || id >= 64) return nullptr;
    Near& n = near[id];
    std::call_once(n.once, [&] {
        if (numa_off()) return;
        cpu_set_t allowed, mine;
        if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
        // nothing to gain when every allowed CPU is on this node already,
        // and no piling of a pool's helpers onto fewer than kMinNearCpus
        constexpr int kMinNearCpus = 4;
        if (device_node_cpus(id, allowed, &mine) < kMinNearCpus || CPU_EQUAL(&mine, &allowed)) return;
        n.set = mine;
        n.ok = true;
    });
    return n.ok ? &n.set : nullptr;
}

// Receive-thread placement (sha1chunk_receive_cpus): the L3 domains of
// HIP device `id`'s node's allowed CPUs, in CPU order (of every allowed CPU
// under SHA1CHUNK_NUMA=off or when the node is unknown), once per device.
// One receive thread per domain kept `submit` at 27.7-29.6 GiB/s where
// threads floating over the node gave 23.8-36.2 (profiles/vq_l3.jsonl).
const std::vector<cpu_set_t>& receive_domains(int id) {
    struct Dom {
        std::once_flag once;
        std::vector<cpu_set_t> dom;
    };
    static Dom doms[64];
    static const std::vector<cpu_set_t> none;
    if (id < 0 || id >= 64) return none;
    Dom& d = doms[id];
    std::call_once(d.once, [&] {
        cpu_set_t allowed, base;
        if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
        if (numa_off() || device_node_cpus(id, allowed, &base) == 0) base = allowed;
        s1host::l3_domains(base, &d.dom, [](int cpu) {
            char path[128];
            snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
            return sysfs_line(path);
        });
    });
    return d.dom;
}
using s1host::pool_copy;
thread_local std::string t_err;
thread_local int t_dev = 0;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(SHA1CHUNK_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                                  \
    } while (0)

constexpr size_t kAlign = 128;  // device layout: every chunk starts on a 128-B line
// Stream (file) pipeline: a ring of slots, each read into pinned memory,
// copied H2D and hashed on its own stream.  A slot's kernel takes ~7 ms
// however few chunks it holds (one chunk's serial chain), so slots must be
// large (512 MiB: ~10 ms of PCIe) and several in flight: with 2 slots each
// read waited for the kernel 2 slots back.  3 slots keep the slot streams
// plus the copy stream within the process's 4 hardware queues (more streams
// share queues and serialise kernels).  Measured on an 8 GiB file in the
// page cache (profiles/file_vq_r01.json): 2 x 256 MiB 29.6 GiB/s, 3 x 512 MiB
// 47.9 GiB/s (PCIe H2D 53.6).
// SHA1CHUNK_STREAM_SLOTS (2..8) / SHA1CHUNK_STREAM_SLOT_MIB (16..1024) for A/B.
constexpr int kMaxSlots = 8;
int stream_slots() {
    static const int n = [] {
        const char* e = getenv("SHA1CHUNK_STREAM_SLOTS");
        return e ? std::min(kMaxSlots, std::max(2, atoi(e))) : 3;
    }();
    return n;
}
size_t stream_slot_bytes() {
    static const size_t b = [] {
        const char* e = getenv("SHA1CHUNK_STREAM_SLOT_MIB");
        const size_t mib = e ? std::min<size_t>(1024, std::max<size_t>(16, atoi(e))) : 512;
        return mib << 20;  // a multiple of SHA1CHUNK_CHUNK_LEN
    }();
    return b;
}

// H2D piece of the stream pipeline (SHA1CHUNK_STREAM_PIECE_MIB, 0 = whole slot)
size_t stream_piece_bytes() {
    static const size_t b = [] {
        const char* e = getenv("SHA1CHUNK_STREAM_PIECE_MIB");
        return static_cast<size_t>(e ? std::max(0, atoi(e)) : 64) << 20;
    }();
    return b;
}

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return SHA1CHUNK_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        bytes = round_up(std::max(bytes, size_t(1) << 20), size_t(1) << 20);
        if (hipMalloc(&p, bytes) != hipSuccess)
            return fail(SHA1CHUNK_ENOMEM, "hipMalloc(%zu) failed", bytes);
        cap = bytes;
        return SHA1CHUNK_OK;
    }
};

struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return SHA1CHUNK_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        bytes = round_up(std::max(bytes, size_t(1) << 20), size_t(1) << 20);
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess)
            return fail(SHA1CHUNK_ENOMEM, "hipHostMalloc(%zu) failed", bytes);
        cap = bytes;
        return SHA1CHUNK_OK;
    }
};

// One pipeline slot: pinned staging for [meta | data], device mirror,
// digests on both sides, its own stream and completion event.
struct Slot {
    PinBuf hpin;    // meta (offsets, lengths, order) then chunk bytes
    PinBuf hdig;    // n x 20 digests back from the device
    DevBuf dmem;    // device copy of hpin
    DevBuf ddig;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    hipEvent_t copied = nullptr;  // this slot's H2D has landed (copy stream)
    bool busy = false;
    // bookkeeping for the batch in flight
    std::vector<uint32_t> ids;  // caller chunk index of each staged entry
};

struct Device {
    std::mutex mu;
    std::atomic<bool> ready{false};  // set once, under mu, after the streams exist
    int id = -1;
    int cus = 256;
    // Host batches use slots 0-1; the stream (file) pipeline cycles through
    // stream_slots() of them.
    Slot slot[kMaxSlots];
    // Every slot's H2D goes through this one stream: copies run back to back
    // at the full PCIe rate instead of two slots splitting it (which would
    // delay the first kernel), and the next slot's copy queues behind the
    // current one while the current slot's kernel runs.
    hipStream_t copy = nullptr;
    DevBuf small;  // streaming calls: state + data
    PinBuf small_pin;
    // threads that pack pageable host chunks into pinned staging (created on
    // the first such batch, alive with the process; idle ones sleep)
    std::unique_ptr<PartPool> pack;
    // CUs held by the persistent verify-queue drains of this device (under
    // drain_mu): each drain workgroup takes a whole CU (all of its LDS)
    std::mutex drain_mu;
    int drain_cus = 0;
};

std::once_flag g_once;
int g_count = -1;  // >= 0 once probed
std::string g_probe_err;
Device* g_dev = nullptr;

void probe() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        g_count = 0;
        g_probe_err = "no HIP device visible";
        return;
    }
    int ok = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t pr;
        if (hipGetDeviceProperties(&pr, d) != hipSuccess) continue;
        if (strncmp(pr.gcnArchName, "gfx950", 6) != 0) {
            g_probe_err = std::string("device ") + std::to_string(d) + " is " + pr.gcnArchName +
                          ", this build targets gfx950 only";
            continue;
        }
        ++ok;
    }
    if (ok != n) {
        g_count = 0;
        return;
    }
    // SHA1CHUNK_VIRTUAL_DEVICES=k (testing): k logical devices over the n
    // physical ones (logical d -> physical d % n), each with its own streams,
    // slots and host thread, so the multi-device path (SHA1CHUNK_ALL_DEVICES:
    // byte-balanced slices, one thread per device) runs on a one-GPU box.
    int k = n;
    if (const char* e = getenv("SHA1CHUNK_VIRTUAL_DEVICES")) k = std::max(1, std::min(64, atoi(e)));
    g_count = k;
    g_dev = new Device[k];
    for (int d = 0; d < k; ++d) g_dev[d].id = d % n;
}

int device_count() {
    std::call_once(g_once, probe);
    return g_count;
}

// Streams and events of slots [0, n), created on first use (caller holds D.mu).
int ensure_slots(Device& D, int n) {
    for (int i = 0; i < n && i < kMaxSlots; ++i) {
        Slot& s = D.slot[i];
        if (s.stream) continue;
        HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
        HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    }
    return SHA1CHUNK_OK;
}

// The shared H2D stream of multi-slot pipelines (caller holds D.mu).
int ensure_copy(Device& D) {
    if (!D.copy) HIP_TRY(hipStreamCreateWithFlags(&D.copy, hipStreamNonBlocking));
    return SHA1CHUNK_OK;
}

// Acquire the calling thread's device (initialising it on first use).
int get_device(Device** out) {
    if (device_count() <= 0) return fail(SHA1CHUNK_ENODEV, "%s", g_probe_err.c_str());
    if (t_dev < 0 || t_dev >= g_count) return fail(SHA1CHUNK_EINVAL, "bad device %d", t_dev);
    Device& D = g_dev[t_dev];
    HIP_TRY(hipSetDevice(D.id));
    if (!D.ready.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> lk(D.mu);
        if (!D.ready.load(std::memory_order_relaxed)) {
            hipDeviceProp_t pr;
            HIP_TRY(hipGetDeviceProperties(&pr, D.id));
            D.cus = pr.multiProcessorCount;
            // Only slot 0 now: a stream costs ~12-20 ms to create
            // (profiles/startup_r01.json, init_cost_r02.jsonl), and a caller
            // whose batch fits one slot (shahash, verify_hash, the CLI on a
            // small file) copies on that slot's own stream.  Other slots and
            // the copy stream are made on first use (ensure_slots, ensure_copy).
            int rc = ensure_slots(D, 1);
            if (rc) return rc;
            D.ready.store(true, std::memory_order_release);
        }
    }
    *out = &D;
    return SHA1CHUNK_OK;
}

// Pick the kernel for a batch of n chunks on a device with `cus` CUs
// (crossovers measured on MI355X: profiles/sweep_r01.json,
// split_2prod_sweep_r01.json; DESIGN.md section 5, kernel table):
//  - up to 2 groups of 64 chunks per CU, each chunk's serial instruction
//    stream is the bound: the split kernel (rounds-only consumer wave alone
//    on its SIMD, two producer waves on others) is ~1.4x the fused kernel
//    per chunk;
//  - beyond that the SIMDs are busy and the split kernel's LDS hand-off and
//    barriers cost more than they save: the fused kernel (schedule + rounds
//    in one wave, 4 blocks of register prefetch) wins.
int choose_kernel(int kernel, size_t n, int cus) {
    if (kernel != SHA1CHUNK_KERNEL_AUTO) return kernel;
    // A/B and test hook: force one kernel behind every AUTO call site
    if (const char* f = getenv("SHA1CHUNK_FORCE_KERNEL")) {
        if (!strcmp(f, "lane")) return SHA1CHUNK_KERNEL_LANE;
        if (!strcmp(f, "fused")) return SHA1CHUNK_KERNEL_FUSED;
        if (!strcmp(f, "split")) return SHA1CHUNK_KERNEL_SPLIT;
    }
    const size_t groups = (n + 63) / 64;
    return groups <= size_t(cus) * 2 ? SHA1CHUNK_KERNEL_SPLIT : SHA1CHUNK_KERNEL_FUSED;
}

// Split-kernel shape: 4-block units (1 barrier per 4 blocks, the whole 160
// KiB LDS, two producers) at one group of 64 chunks per CU; at two groups per
// CU one 8-wave workgroup holding both, 2-block units, two producers per
// consumer sharing a SIMD and each consumer alone on its own (case 11:
// 10-11 % faster than two 2-wave workgroups, profiles/split_2prod_sweep_r01.json);
// else 1-block units (40 KiB).  SHA1CHUNK_SPLIT_UNIT forces a shape for A/B
// runs: 1, 4, 11 in the product library; the study's other shapes and
// variants only in the A/B library (`make ab`, sha1_kernels.h).  Forcing a
// shape this library does not hold fails the call (SHA1CHUNK_EINVAL,
// launch_checked) instead of timing some other kernel.
int split_unit(size_t n, int cus) {
    if (const char* e = getenv("SHA1CHUNK_SPLIT_UNIT")) return atoi(e);
    const size_t groups = (n + 63) / 64;
    if (groups <= size_t(cus)) return 4;
    if (groups <= size_t(cus) * 2) return 11;
    return 1;
}

hipError_t launch(int kernel, const BatchArgs& A, int cus, hipStream_t st) {
    switch (kernel) {
    case SHA1CHUNK_KERNEL_LANE: return launch_lane(A, st);
    case SHA1CHUNK_KERNEL_FUSED: return launch_fused(A, st);
    case SHA1CHUNK_KERNEL_SPLIT: return launch_split(A, split_unit(A.n, cus), st);
    default: return hipErrorInvalidValue;
    }
}

// Checks every launch path shares (plain kernels and the mixed kernel):
// grid sizes are computed in 32 bits ((n + 255) / 256, (n + 63) / 64), and
// digests are stored as 32-bit words.
int check_batch(const BatchArgs& A) {
    if (A.n > 0xffffffffu - 1024u)
        return fail(SHA1CHUNK_EINVAL, "batch of %u chunks: at most 2^32 - 1025 per call", A.n);
    if (A.n > 0 && (reinterpret_cast<uintptr_t>(A.dig) & 3u))
        return fail(SHA1CHUNK_EALIGN, "digest buffer must be 4-byte aligned");
    return SHA1CHUNK_OK;
}

int launch_checked(int kernel, const BatchArgs& A, hipStream_t st, int cus = 256) {
    if (kernel < SHA1CHUNK_KERNEL_LANE || kernel > SHA1CHUNK_KERNEL_SPLIT)
        return fail(SHA1CHUNK_EINVAL, "unknown kernel id %d", kernel);
    if (int rc = check_batch(A)) return rc;
    if (kernel == SHA1CHUNK_KERNEL_SPLIT && !split_unit_built(split_unit(A.n, cus)))
        return fail(SHA1CHUNK_EINVAL, "split shape %d is not in this library (A/B shapes: `make ab`)",
                    split_unit(A.n, cus));
    hipError_t e = launch(kernel, A, cus, st);
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "kernel launch: %s", hipGetErrorString(e));
    return SHA1CHUNK_OK;
}

// Mixed kernel for sorted ragged batches of more groups than CUs, unless an
// A/B hook forces a kernel behind AUTO (SHA1CHUNK_FORCE_KERNEL) or
// SHA1CHUNK_MIXED=0 turns it off (then AUTO's uniform-batch rule applies).
// SHA1CHUNK_MIXED=all also sends batches of <= CUs groups (every group its
// own CU at launch) through it (A/B).
bool use_mixed(size_t n, int cus) {
    if (getenv("SHA1CHUNK_FORCE_KERNEL")) return false;
    const char* e = getenv("SHA1CHUNK_MIXED");
    if (e && !strcmp(e, "0")) return false;
    if (e && !strcmp(e, "all")) return true;
    return (n + 63) / 64 > size_t(cus);
}

// SHA1CHUNK_MIXED_PLAN="mode,H,F" replaces the device-side plan (tests and
// A/B runs): mode 0 with H <= the model's head cap (min(groups, 4 CUs,
// 4096)) or H = groups, and F in {4, 8}; or mode 1.
// SHA1CHUNK_MIXED_DEBUG=1 prints the plan used (synchronises the stream:
// diagnostics only).
int launch_mixed_checked(const BatchArgs& A, const uint32_t* sorted_len, const BigFix* big, uint32_t* plan, int cus,
                         hipStream_t st) {
    if (int rc = check_batch(A)) return rc;
    int forced[3] = {0, 0, 0};
    bool force = false;
    if (const char* e = getenv("SHA1CHUNK_MIXED_PLAN")) {
        uint32_t hcap;
        const uint32_t groups = (A.n + 63u) / 64u;
        (void)mixed_grid(groups, cus, &hcap);
        if (sscanf(e, "%d,%d,%d", &forced[0], &forced[1], &forced[2]) != 3 || forced[0] < 0 ||
            forced[0] > 1 ||
            (forced[0] == 0 && (forced[1] < 0 || ((uint32_t)forced[1] > hcap && (uint32_t)forced[1] != groups) ||
                                (forced[2] != 4 && forced[2] != 8))))
            return fail(SHA1CHUNK_EINVAL,
                        "SHA1CHUNK_MIXED_PLAN=%s: want 0,H,F (0 <= H <= %u or H = %u, F 4|8) or 1,0,0", e,
                        hcap, groups);
        force = true;
    }
    hipError_t e = launch_mixed(A, sorted_len, big, plan, cus, force ? forced : nullptr, st);
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "mixed kernel launch: %s", hipGetErrorString(e));
    if (const char* d = getenv("SHA1CHUNK_MIXED_DEBUG"); d && atoi(d)) {
        uint32_t p[28];
        HIP_TRY(hipMemcpyAsync(p, plan, sizeof p, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        fprintf(stderr, "sha1chunk mixed plan: n=%u groups=%u cus=%d mode=%u H=%u F=%u\n", A.n,
                (A.n + 63u) / 64u, cus, p[0], p[1], p[2]);
        if (!force && p[12])  // the planner's stage end times (us since its start; the first
                              // simulation sweep, pass 2's rest, pass 3's misses) and shader kcycles
            fprintf(stderr,
                    "sha1chunk mixed planner stages: scan %.1f bounds %.1f sweep %.1f pass2 %.1f pass3 %.1f us;"
                    " kcycles %.1f %.1f %.1f %.1f %.1f (bounds: run8 %.1f prefix %.1f search %.1f; first sweep:"
                    " list %.1f bounds %.1f packed %.1f, %u candidates, longest call %.1f)\n",
                    p[8] * 0.01, p[9] * 0.01, p[10] * 0.01, p[11] * 0.01, p[12] * 0.01, p[14] * 1e-3, p[15] * 1e-3,
                    p[16] * 1e-3, p[17] * 1e-3, p[18] * 1e-3, p[24] * 1e-3, p[25] * 1e-3, p[26] * 1e-3,
                    p[20] * 1e-3, p[21] * 1e-3, p[22] * 1e-3, p[23], p[27] * 1e-3);
    }
    return SHA1CHUNK_OK;
}

// ------------------------------------------------------------ host batch --
// Host batches go through two pipeline slots (own stream each), so the H2D
// copy of slot b+1 overlaps the kernel of slot b.  A slot's bytes come
// either straight from the caller's buffer (when it is pinned and the slot's
// chunks are back to back in it: one hipMemcpyAsync, no host copy) or are
// packed into the slot's pinned staging first.  Device layout of a slot:
//   [off: u64 x m][len: u32 x m] pad to 128 | chunk bytes
// Slot size scales with the batch: a pass of the kernel takes ~7 ms however
// few chunks it has (serial per chunk), so a slot must carry enough bytes
// that its PCIe copy, not the kernel, is the longer stage.
// SHA1CHUNK_HOST_SLOT_MIB (16..1024, read per call) fixes the slot size, so
// tests can wrap the two-slot ring many times over a modest batch.
size_t slot_bytes_for(uint64_t total) {
    if (const char* e = getenv("SHA1CHUNK_HOST_SLOT_MIB"))
        return std::min<size_t>(1024, std::max<size_t>(16, atoi(e))) << 20;
    const size_t lo = size_t(256) << 20, hi = size_t(1) << 30;
    return std::min(hi, std::max(lo, static_cast<size_t>(total / 4)));
}

// The slot's stream waits for its H2D copies, issued on stream `cs` (the
// copy stream, or the slot's own stream for a batch of one fill).
int copies_issued(Slot& s, hipStream_t cs) {
    if (cs == s.stream) return SHA1CHUNK_OK;
    HIP_TRY(hipEventRecord(s.copied, cs));
    HIP_TRY(hipStreamWaitEvent(s.stream, s.copied, 0));
    return SHA1CHUNK_OK;
}

bool host_pinned(const void* p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// Pack entries [j0, j1) of a slot from pageable caller memory into pinned
// staging on the device's pack pool: one thread copies ~10 GB/s, well under
// the PCIe rate.  The entries are split into pool-width runs of about equal
// bytes.
int pack_threads() {
    const char* e = getenv("SHA1CHUNK_COPY_THREADS");
    return e ? std::max(1, atoi(e)) : 8;
}
void pack_range(PartPool& pool, uint8_t* h, const uint64_t* hoff, const uint8_t* base,
                const uint64_t* offsets, const uint32_t* lengths, const std::vector<uint32_t>& ids,
                size_t j0, size_t j1, size_t bytes) {
    const size_t T = std::min<size_t>(pool.width(), std::max<size_t>(1, bytes >> 23));
    std::vector<size_t> cut(T + 1, j1);
    cut[0] = j0;
    for (size_t t = 1, j = j0; t < T; ++t) {
        const uint64_t target = hoff[j0] + bytes * t / T;
        while (j < j1 && hoff[j] < target) ++j;
        cut[t] = j;
    }
    pool.run(T, [&](size_t t) {
        for (size_t j = cut[t]; j < cut[t + 1]; ++j)
            if (lengths[ids[j]]) memcpy(h + hoff[j], base + offsets[ids[j]], lengths[ids[j]]);
    });
}

int stage_and_launch(Device& D, Slot& s, const uint8_t* base, const uint64_t* offsets,
                     const uint32_t* lengths, const std::vector<uint32_t>& order, size_t lo,
                     size_t hi, size_t data_bytes, bool src_pinned, hipStream_t cs) {
    const size_t m = hi - lo;
    const size_t meta = round_up(m * (sizeof(uint64_t) + sizeof(uint32_t)), kAlign);
    int rc;
    s.ids.assign(order.begin() + lo, order.begin() + hi);
    // Direct mode: chunks contiguous and ascending in the pinned source, each
    // length a multiple of 16 (keeps every device chunk 16-byte aligned).
    bool direct = src_pinned;
    uint64_t span0 = offsets[s.ids[0]], span = 0;
    for (size_t j = 0; direct && j < m; ++j) {
        const uint32_t id = s.ids[j];
        direct = offsets[id] == span0 + span && (j + 1 == m || (lengths[id] & 15u) == 0);
        span += lengths[id];
    }
    const size_t dbytes = direct ? round_up(span, kAlign) : data_bytes;
    // SHA1CHUNK_HOST_DEBUG=1: one line per slot fill (tests check the mode
    // and the number of ring wraps; diagnostics only)
    if (const char* dbg = getenv("SHA1CHUNK_HOST_DEBUG"); dbg && atoi(dbg))
        fprintf(stderr, "sha1chunk host slot %d: %zu chunks %zu bytes %s\n",
                static_cast<int>(&s - D.slot), m, direct ? static_cast<size_t>(span) : data_bytes,
                direct ? "direct" : "packed");
    if ((rc = s.hpin.ensure(meta + (direct ? 0 : data_bytes))) || (rc = s.dmem.ensure(meta + dbytes)) ||
        (rc = s.hdig.ensure(m * 20)) || (rc = s.ddig.ensure(m * 20)))
        return rc;
    uint8_t* h = static_cast<uint8_t*>(s.hpin.p);
    uint64_t* hoff = reinterpret_cast<uint64_t*>(h);
    uint32_t* hlen = reinterpret_cast<uint32_t*>(h + m * sizeof(uint64_t));
    size_t cur = meta;
    for (size_t j = 0; j < m; ++j) {
        const uint32_t id = s.ids[j];
        const uint32_t L = lengths[id];
        hlen[j] = L;
        if (direct) {
            hoff[j] = meta + (offsets[id] - span0);
        } else {
            hoff[j] = cur;
            cur += round_up(L, kAlign);
        }
    }
    uint8_t* d = static_cast<uint8_t*>(s.dmem.p);
    if (direct) {
        HIP_TRY(hipMemcpyAsync(d, h, meta, hipMemcpyHostToDevice, cs));
        if (span) HIP_TRY(hipMemcpyAsync(d + meta, base + span0, span, hipMemcpyHostToDevice, cs));
    } else {
        // pack in runs of ~64 MiB and start each run's H2D as soon as it is
        // packed, so the copy engine works while the rest is packed
        if (!D.pack) D.pack.reset(new PartPool(pack_threads() - 1, near_cpus(D.id)));
        static const size_t piece = [] {  // SHA1CHUNK_PACK_PIECE_MIB, 0 = whole slot
            const char* e = getenv("SHA1CHUNK_PACK_PIECE_MIB");
            const size_t mib = e ? static_cast<size_t>(std::max(0, atoi(e))) : 64;
            return mib ? mib << 20 : ~size_t(0) >> 1;
        }();
        for (size_t j0 = 0; j0 < m;) {
            size_t j1 = j0 + 1;
            while (j1 < m && hoff[j1] - hoff[j0] < piece) ++j1;
            const size_t end = j1 < m ? hoff[j1] : cur;
            pack_range(*D.pack, h, hoff, base, offsets, lengths, s.ids, j0, j1, end - hoff[j0]);
            HIP_TRY(hipMemcpyAsync(d + hoff[j0], h + hoff[j0], end - hoff[j0], hipMemcpyHostToDevice, cs));
            j0 = j1;
        }
        HIP_TRY(hipMemcpyAsync(d, h, meta, hipMemcpyHostToDevice, cs));
    }
    if ((rc = copies_issued(s, cs))) return rc;
    BatchArgs A{};
    A.base = d;
    A.off = reinterpret_cast<const uint64_t*>(d);
    A.len = reinterpret_cast<const uint32_t*>(d + m * sizeof(uint64_t));
    A.n = static_cast<uint32_t>(m);
    A.dig = static_cast<uint8_t*>(s.ddig.p);
    // Entries are already in length order: no order[] indirection needed.
    if ((rc = launch_checked(choose_kernel(SHA1CHUNK_KERNEL_AUTO, m, D.cus), A, s.stream, D.cus)))
        return rc;
    HIP_TRY(hipMemcpyAsync(s.hdig.p, s.ddig.p, m * 20, hipMemcpyDeviceToHost, s.stream));
    HIP_TRY(hipEventRecord(s.done, s.stream));
    s.busy = true;
    return SHA1CHUNK_OK;
}

// A call that failed half-way can leave a slot in flight; its results
// belong to that call, so the next call waits for the work and drops them
// instead of scattering stale digests into its own output.
int discard_in_flight(Device& D) {
    for (auto& s : D.slot) {
        if (!s.busy) continue;
        s.busy = false;
        HIP_TRY(hipEventSynchronize(s.done));
    }
    return SHA1CHUNK_OK;
}

int drain(Slot& s, uint8_t* digests) {
    if (!s.busy) return SHA1CHUNK_OK;
    s.busy = false;
    HIP_TRY(hipEventSynchronize(s.done));
    const uint8_t* src = static_cast<const uint8_t*>(s.hdig.p);
    for (size_t j = 0; j < s.ids.size(); ++j) memcpy(digests + 20ull * s.ids[j], src + 20 * j, 20);
    return SHA1CHUNK_OK;
}

int hash_host(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths, size_t n,
              uint8_t* digests) {
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(D->mu);
    if ((rc = discard_in_flight(*D))) return rc;
    // Longest first, so every wave of 64 gets near-equal lengths (a wave
    // runs as long as its longest lane); equal lengths keep caller order.
    std::vector<uint32_t> order(n);
    std::iota(order.begin(), order.end(), 0u);
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return lengths[a] > lengths[b]; });
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) total += lengths[i];
    const size_t slot_cap = slot_bytes_for(total);
    const bool pinned = host_pinned(base);
    size_t lo = 0;
    int which = 0;
    while (lo < n) {
        size_t hi = lo, bytes = 0;
        while (hi < n) {
            const size_t b = round_up(lengths[order[hi]], kAlign);
            if (hi > lo && bytes + b > slot_cap) break;
            bytes += b;
            ++hi;
        }
        // A batch that fits one slot (a single chunk from shahash /
        // verify_hash) copies on slot 0's stream and creates no other stream;
        // larger ones share the copy stream and alternate two slots.
        const bool one_fill = lo == 0 && hi == n;
        if (!one_fill && ((rc = ensure_slots(*D, 2)) || (rc = ensure_copy(*D)))) return rc;
        Slot& s = D->slot[which];
        if ((rc = drain(s, digests))) return rc;
        if ((rc = stage_and_launch(*D, s, base, offsets, lengths, order, lo, hi, bytes, pinned,
                                   one_fill ? s.stream : D->copy)))
            return rc;
        lo = hi;
        which ^= 1;
    }
    if ((rc = drain(D->slot[which], digests))) return rc;
    return drain(D->slot[which ^ 1], digests);
}

// Shard a host batch over every device: contiguous, byte-balanced slices,
// one host thread per device, no collective.
int hash_host_all(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths, size_t n,
                  uint8_t* digests) {
    const int nd = device_count();
    if (nd <= 0) return fail(SHA1CHUNK_ENODEV, "%s", g_probe_err.c_str());
    if (nd == 1 || n < 64) return hash_host(base, offsets, lengths, n, digests);
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) total += lengths[i];
    std::vector<size_t> cut(nd + 1, n);
    cut[0] = 0;
    uint64_t acc = 0;
    int d = 1;
    for (size_t i = 0; i < n && d < nd; ++i) {
        acc += lengths[i];
        while (d < nd && acc >= total * (uint64_t)d / (uint64_t)nd) cut[d++] = i + 1;
    }
    std::vector<int> rcs(nd, 0);
    std::vector<std::string> errs(nd);
    std::vector<std::thread> th;
    for (int g = 0; g < nd; ++g) {
        th.emplace_back([&, g] {
            t_dev = g;
            const size_t a = cut[g], b = cut[g + 1];
            if (b > a) {
                std::vector<uint64_t> off(offsets + a, offsets + b);
                rcs[g] = hash_host(base, off.data(), lengths + a, b - a, digests + 20 * a);
                if (rcs[g]) errs[g] = t_err;
            }
        });
    }
    for (auto& t : th) t.join();
    for (int g = 0; g < nd; ++g)
        if (rcs[g]) return fail(rcs[g], "device %d: %s", g, errs[g].c_str());
    return SHA1CHUNK_OK;
}

}  // namespace

// ================================================================ C ABI ====
extern "C" {

int s1be_device_count(void) {
    const int n = device_count();
    if (n <= 0) fail(SHA1CHUNK_ENODEV, "%s", g_probe_err.c_str());
    return n;
}

int s1be_set_device(int device) {
    const int n = device_count();
    if (n <= 0) return fail(SHA1CHUNK_ENODEV, "%s", g_probe_err.c_str());
    if (device < 0 || device >= n) return fail(SHA1CHUNK_EINVAL, "device %d of %d", device, n);
    t_dev = device;
    return SHA1CHUNK_OK;
}

const char* s1be_last_error(void) { return t_err.c_str(); }

// PCI address of logical device `device`'s physical GPU (multi-device tests
// and bench.py's device identity: distinct ranks/threads, distinct GPUs).
int s1be_device_pci_bus_id(int device, char* buf, size_t len) {
    const int n = device_count();
    if (n <= 0) return fail(SHA1CHUNK_ENODEV, "%s", g_probe_err.c_str());
    if (device < 0 || device >= n) return fail(SHA1CHUNK_EINVAL, "device %d of %d", device, n);
    if (len > static_cast<size_t>(INT32_MAX)) len = INT32_MAX;
    HIP_TRY(hipDeviceGetPCIBusId(buf, static_cast<int>(len), g_dev[device].id));
    return SHA1CHUNK_OK;
}

// The CPUs for receive thread `slot` of device `device` (L3 domain slot mod
// their count; receive_domains), as a cpu_set_t of `len` >= its size bytes.
int s1be_receive_cpus(int device, unsigned slot, void* mask, size_t len, unsigned* domains) {
    const int n = device_count();
    if (n <= 0) return fail(SHA1CHUNK_ENODEV, "%s", g_probe_err.c_str());
    if (device < 0 || device >= n) return fail(SHA1CHUNK_EINVAL, "device %d of %d", device, n);
    const std::vector<cpu_set_t>& dom = receive_domains(g_dev[device].id);
    if (dom.empty()) return fail(SHA1CHUNK_EINVAL, "no CPU of this process's affinity mask found");
    const cpu_set_t& d = dom[slot % dom.size()];
    memset(mask, 0, len);
    memcpy(mask, &d, sizeof d);
    if (domains) *domains = static_cast<unsigned>(dom.size());
    return CPU_COUNT(&d);
}

int s1be_hash_device_async(const void* d_base, const uint64_t* d_offsets,
                                const uint32_t* d_lengths, size_t n, uint8_t* d_digests,
                                void* stream, int kernel) {
    if (n > 0xffffffffu) return fail(SHA1CHUNK_EINVAL, "n too large");
    if (n && (!d_base || !d_offsets || !d_lengths || !d_digests))
        return fail(SHA1CHUNK_EINVAL, "null device pointer");
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    BatchArgs A{};
    A.base = static_cast<const uint8_t*>(d_base);
    A.off = d_offsets;
    A.len = d_lengths;
    A.n = static_cast<uint32_t>(n);
    A.dig = d_digests;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // AUTO on a ragged batch: hash longest-first (sha1_sort.hip); with more
    // groups of 64 than CUs, through the mixed kernel and its device-side
    // plan (sha1_kernels.hip, mixed).
    if ((rc = check_batch(A))) return rc;
    void* scratch = nullptr;
    if (kernel == SHA1CHUNK_KERNEL_AUTO && n > 64) {
        const uint32_t* sorted_len = nullptr;
        uint32_t* plan = nullptr;
        BigFix big{};
        const bool mixed = use_mixed(n, D->cus);
        // the mixed path re-ranks chunks of 4 MiB and more exactly (BigFix);
        // one group per CU or fewer hash all at once, where the grouping of
        // such chunks cannot change the batch's time
        hipError_t e = sort_by_length_desc(d_lengths, A.n, &A.order, &sorted_len, &plan, &scratch,
                                           mixed ? &big : nullptr, st);
        if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "length sort: %s", hipGetErrorString(e));
        if (mixed) {
            rc = launch_mixed_checked(A, sorted_len, &big, plan, D->cus, st);
            (void)hipFreeAsync(scratch, st);
            return rc;
        }
    }
    rc = launch_checked(choose_kernel(kernel, n, D->cus), A, st, D->cus);
    if (scratch) (void)hipFreeAsync(scratch, st);
    return rc;
}

int s1be_hash_uniform_async(const void* d_base, uint32_t chunk_len, size_t n,
                                 uint8_t* d_digests, void* stream, int kernel) {
    if (n > 0xffffffffu) return fail(SHA1CHUNK_EINVAL, "n too large");
    if (n && (!d_base || !d_digests)) return fail(SHA1CHUNK_EINVAL, "null device pointer");
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    BatchArgs A{};
    A.base = static_cast<const uint8_t*>(d_base);
    A.ulen = chunk_len;
    A.n = static_cast<uint32_t>(n);
    A.dig = d_digests;
    return launch_checked(choose_kernel(kernel, n, D->cus), A, static_cast<hipStream_t>(stream), D->cus);
}

// Diagnostics (tests; no frontend entry point): the longest-first order and
// sorted lengths AUTO's ragged path hashes a batch of lengths in
// (sha1_sort.hip), copied into the caller's device arrays of n entries.
int s1be_sort_order_async(const uint32_t* d_lengths, size_t n, uint32_t* d_order, uint32_t* d_sorted_len,
                          void* stream) {
    if (n > 0xffffffffu) return fail(SHA1CHUNK_EINVAL, "n too large");
    if (n == 0) return SHA1CHUNK_OK;
    if (!d_lengths || !d_order || !d_sorted_len) return fail(SHA1CHUNK_EINVAL, "null device pointer");
    Device* D;
    if (int rc = get_device(&D)) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t *order = nullptr, *sorted_len = nullptr;
    uint32_t* plan = nullptr;
    void* scratch = nullptr;
    hipError_t e = sort_by_length_desc(d_lengths, static_cast<uint32_t>(n), &order, &sorted_len, &plan, &scratch,
                                       nullptr, st);
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "length sort: %s", hipGetErrorString(e));
    (void)sorted_len;  // group heads only: every position's length is gathered below
    e = hipMemcpyAsync(d_order, order, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = gather_sorted_lengths(d_lengths, order, d_sorted_len, static_cast<uint32_t>(n), st);
    (void)hipFreeAsync(scratch, st);
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "sort copy: %s", hipGetErrorString(e));
    return SHA1CHUNK_OK;
}

// Diagnostics (tests): the order the mixed path hashes a ragged batch in --
// the length sort, then the layout kernel's exact re-ranking of chunks of
// 4 MiB and more (BigFix) -- and the lengths in that order.  d_offsets: the
// batch's offsets (the layout summary reads them; no bytes are read).
int s1be_mixed_order_async(const uint32_t* d_lengths, const uint64_t* d_offsets, size_t n, uint32_t* d_order,
                           uint32_t* d_sorted_len, void* stream) {
    if (n > 0xffffffffu) return fail(SHA1CHUNK_EINVAL, "n too large");
    if (n == 0) return SHA1CHUNK_OK;
    if (!d_lengths || !d_offsets || !d_order || !d_sorted_len) return fail(SHA1CHUNK_EINVAL, "null device pointer");
    Device* D;
    if (int rc = get_device(&D)) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    BatchArgs A{};
    A.base = reinterpret_cast<const uint8_t*>(d_offsets);  // addresses only, never read
    A.off = d_offsets;
    A.len = d_lengths;
    A.n = static_cast<uint32_t>(n);
    const uint32_t* sorted_len = nullptr;
    uint32_t* plan = nullptr;
    void* scratch = nullptr;
    BigFix big{};
    hipError_t e = sort_by_length_desc(d_lengths, A.n, &A.order, &sorted_len, &plan, &scratch, &big, st);
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "length sort: %s", hipGetErrorString(e));
    e = launch_plan_layout(A, sorted_len, &big, plan, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_order, A.order, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = gather_sorted_lengths(d_lengths, A.order, d_sorted_len, A.n, st);
    (void)hipFreeAsync(scratch, st);
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "mixed order: %s", hipGetErrorString(e));
    return SHA1CHUNK_OK;
}

int s1be_compare_device_async(const uint8_t* d_digests, const uint8_t* d_expected, size_t n,
                                   uint8_t* d_mismatch, void* stream) {
    if (n > 0xffffffffu) return fail(SHA1CHUNK_EINVAL, "n too large");
    if (n && (!d_digests || !d_expected || !d_mismatch))
        return fail(SHA1CHUNK_EINVAL, "null device pointer");
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    hipError_t e = launch_compare(d_digests, d_expected, static_cast<uint32_t>(n), d_mismatch,
                                  static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "compare launch: %s", hipGetErrorString(e));
    return SHA1CHUNK_OK;
}

int s1be_hash_batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                         size_t n, uint8_t* digests, unsigned flags) {
    if (n == 0) return SHA1CHUNK_OK;
    if (!base || !offsets || !lengths || !digests) return fail(SHA1CHUNK_EINVAL, "null pointer");
    if (n > 0xffffffffu) return fail(SHA1CHUNK_EINVAL, "n too large");
    if (flags & SHA1CHUNK_DEVICE) {
        Device* D;
        int rc = get_device(&D);
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(D->mu);
        hipStream_t st = D->slot[0].stream;
        if ((rc = s1be_hash_device_async(base, offsets, lengths, n, digests, st,
                                              SHA1CHUNK_KERNEL_AUTO)))
            return rc;
        HIP_TRY(hipStreamSynchronize(st));
        return SHA1CHUNK_OK;
    }
    const uint8_t* b = static_cast<const uint8_t*>(base);
    if (flags & SHA1CHUNK_ALL_DEVICES) return hash_host_all(b, offsets, lengths, n, digests);
    return hash_host(b, offsets, lengths, n, digests);
}

int s1be_verify_batch(const void* base, const uint64_t* offsets, const uint32_t* lengths,
                           size_t n, const uint8_t* expected, uint8_t* mismatch, unsigned flags) {
    if (n == 0) return SHA1CHUNK_OK;
    if (!expected || !mismatch) return fail(SHA1CHUNK_EINVAL, "null pointer");
    if (flags & SHA1CHUNK_DEVICE) {
        Device* D;
        int rc = get_device(&D);
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(D->mu);
        Slot& s = D->slot[0];
        if ((rc = s.ddig.ensure(n * 20))) return rc;
        if ((rc = s1be_hash_device_async(base, offsets, lengths, n,
                                              static_cast<uint8_t*>(s.ddig.p), s.stream,
                                              SHA1CHUNK_KERNEL_AUTO)))
            return rc;
        if ((rc = s1be_compare_device_async(static_cast<uint8_t*>(s.ddig.p), expected, n,
                                                 mismatch, s.stream)))
            return rc;
        HIP_TRY(hipStreamSynchronize(s.stream));
        return SHA1CHUNK_OK;
    }
    std::vector<uint8_t> dig(n * 20);
    int rc = s1be_hash_batch(base, offsets, lengths, n, dig.data(), flags);
    if (rc) return rc;
    for (size_t i = 0; i < n; ++i) mismatch[i] = memcmp(&dig[20 * i], expected + 20 * i, 20) != 0;
    return SHA1CHUNK_OK;
}

}  // extern "C"

namespace {
// size_hint: bytes the reader will deliver, when known (regular files);
// small inputs then get a slot just big enough (the pinned allocation is a
// one-process cost the make-chunks CLI pays on every run), mid-size inputs
// are spread over all slots so reads and copies overlap.
long hash_stream_sized(sha1chunk_reader_fn reader, void* reader_ctx, sha1chunk_sink_fn sink,
                       void* sink_ctx, uint64_t size_hint) {
    if (!reader) return fail(SHA1CHUNK_EINVAL, "null reader");
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(D->mu);
    if ((rc = discard_in_flight(*D))) return rc;
    const int nslots = stream_slots();
    size_t slot_bytes = stream_slot_bytes();
    bool one_fill = false;  // a known size that fits one slot: slot 0 alone, copies on its stream
    if (size_hint) {
        const size_t L = SHA1CHUNK_CHUNK_LEN;
        const size_t whole = round_up(size_hint, L);
        const size_t spread = std::max(size_t(64) << 20, round_up(size_hint / nslots, L));
        slot_bytes = std::min({slot_bytes, whole, spread});
        one_fill = whole <= slot_bytes;
    }
    const size_t per_slot = slot_bytes / SHA1CHUNK_CHUNK_LEN;  // 1024 chunks per 512 MiB
    const size_t meta = round_up(per_slot * 12, kAlign);
    size_t next = 0;  // index of the next slot's first chunk
    size_t pend_first[kMaxSlots] = {}, pend_m[kMaxSlots] = {};
    auto finish = [&](int w) -> int {
        Slot& s = D->slot[w];
        if (!s.busy) return SHA1CHUNK_OK;
        s.busy = false;
        HIP_TRY(hipEventSynchronize(s.done));
        if (sink) sink(sink_ctx, pend_first[w], static_cast<const uint8_t*>(s.hdig.p), pend_m[w]);
        return SHA1CHUNK_OK;
    };
    int which = 0;
    bool eof = false;
    for (size_t fill = 0; !eof; ++fill) {
        // streams on first use; a reader that delivers more than size_hint
        // leaves the one-fill path at its second slot
        if (fill == 1) one_fill = false;
        if ((rc = ensure_slots(*D, which + 1)) || (!one_fill && (rc = ensure_copy(*D)))) return rc;
        Slot& s = D->slot[which];
        const hipStream_t cs = one_fill ? s.stream : D->copy;
        if ((rc = finish(which))) return rc;
        if ((rc = s.hpin.ensure(meta + slot_bytes)) || (rc = s.dmem.ensure(meta + slot_bytes)) ||
            (rc = s.hdig.ensure(per_slot * 20)) || (rc = s.ddig.ensure(per_slot * 20)))
            return rc;
        uint8_t* h = static_cast<uint8_t*>(s.hpin.p);
        uint8_t* d = static_cast<uint8_t*>(s.dmem.p);
        // Read straight into pinned memory: the fread loop of make_chunks
        // (chunk.c:22), a slot of up to 1024 chunks at a time, read in pieces
        // whose H2D copies start as soon as each piece is in, so the copy
        // engine is not idle while a whole slot is read (the first slot
        // above all); the kernel still waits for the whole slot.
        const size_t piece = stream_piece_bytes() ? stream_piece_bytes() : slot_bytes;
        size_t got = 0, sent = 0;
        while (got < slot_bytes) {
            const size_t r = reader(reader_ctx, h + meta + got, std::min(piece, slot_bytes - got));
            if (r == (size_t)-1) return fail(SHA1CHUNK_EIO, "stream read error");
            if (r == 0) {
                eof = true;
                break;
            }
            got += r;
            if (got - sent >= piece && got < slot_bytes) {
                HIP_TRY(hipMemcpyAsync(d + meta + sent, h + meta + sent, got - sent, hipMemcpyHostToDevice,
                                       cs));
                sent = got;
            }
        }
        if (got == 0) break;
        const size_t m = (got + SHA1CHUNK_CHUNK_LEN - 1) / SHA1CHUNK_CHUNK_LEN;
        uint64_t* hoff = reinterpret_cast<uint64_t*>(h);
        uint32_t* hlen = reinterpret_cast<uint32_t*>(h + m * 8);
        for (size_t j = 0; j < m; ++j) {
            hoff[j] = meta + j * SHA1CHUNK_CHUNK_LEN;
            hlen[j] = static_cast<uint32_t>(
                std::min<size_t>(SHA1CHUNK_CHUNK_LEN, got - j * SHA1CHUNK_CHUNK_LEN));
        }
        HIP_TRY(hipMemcpyAsync(d + meta + sent, h + meta + sent, got - sent, hipMemcpyHostToDevice, cs));
        HIP_TRY(hipMemcpyAsync(d, h, m * 12, hipMemcpyHostToDevice, cs));  // offsets + lengths
        if ((rc = copies_issued(s, cs))) return rc;
        BatchArgs A{};
        A.base = d;
        A.off = reinterpret_cast<const uint64_t*>(d);
        A.len = reinterpret_cast<const uint32_t*>(d + m * 8);
        A.n = static_cast<uint32_t>(m);
        A.dig = static_cast<uint8_t*>(s.ddig.p);
        if ((rc = launch_checked(choose_kernel(SHA1CHUNK_KERNEL_AUTO, m, D->cus), A, s.stream, D->cus)))
            return rc;
        HIP_TRY(hipMemcpyAsync(s.hdig.p, s.ddig.p, m * 20, hipMemcpyDeviceToHost, s.stream));
        HIP_TRY(hipEventRecord(s.done, s.stream));
        s.busy = true;
        pend_first[which] = next;
        pend_m[which] = m;
        next += m;
        which = (which + 1) % nslots;
    }
    // remaining slots complete in issue order: the sink sees ascending indices
    for (int k = 0; k < nslots; ++k)
        if ((rc = finish((which + k) % nslots))) return rc;
    return static_cast<long>(next);
}
}  // namespace

extern "C" {

long s1be_hash_stream_sized(sha1chunk_reader_fn reader, void* reader_ctx,
                                 sha1chunk_sink_fn sink, void* sink_ctx, uint64_t size_hint) {
    return hash_stream_sized(reader, reader_ctx, sink, sink_ctx, size_hint);
}

namespace {
struct FdSink {
    uint8_t* out;
    size_t max;
};
static size_t fd_reader(void* ctx, void* dst, size_t n) {
    const int fd = *static_cast<int*>(ctx);
    for (;;) {
        const ssize_t r = read(fd, dst, n);
        if (r >= 0) return static_cast<size_t>(r);
        if (errno != EINTR) return (size_t)-1;
    }
}
// Regular files: each slot is filled by several threads with pread -- one
// thread copies from the page cache at only ~5-10 GB/s, well under the PCIe
// rate the pipeline can take.  The fd offset is left at the end of what was
// read, as a read() loop would leave it.
struct ParFile {
    int fd;
    off_t pos, end;
    PartPool* pool;
};
static size_t par_reader(void* ctx, void* dst, size_t n) {
    ParFile* f = static_cast<ParFile*>(ctx);
    if (f->pos >= f->end) return 0;
    const size_t want = std::min<size_t>(n, static_cast<size_t>(f->end - f->pos));
    const size_t min_piece = size_t(8) << 20;
    const int T = static_cast<int>(std::max<size_t>(1, std::min<size_t>(f->pool->width(), want / min_piece)));
    const size_t piece = (want + T - 1) / T;
    std::vector<size_t> got(T, 0);
    std::atomic<bool> bad{false};
    auto work = [&](int t) {
        const size_t lo = std::min(want, piece * t), len = std::min(want, lo + piece) - lo;
        uint8_t* d = static_cast<uint8_t*>(dst) + lo;
        while (got[t] < len) {
            const ssize_t r = pread(f->fd, d + got[t], len - got[t], f->pos + lo + got[t]);
            if (r < 0) {
                if (errno == EINTR) continue;
                bad = true;
                return;
            }
            if (r == 0) return;  // the file shrank under us
            got[t] += static_cast<size_t>(r);
        }
    };
    f->pool->run(static_cast<size_t>(T), [&](size_t t) { work(static_cast<int>(t)); });
    if (bad) return (size_t)-1;
    // bytes read contiguously from pos (a short piece ends the file)
    size_t total = 0;
    for (int t = 0; t < T; ++t) {
        const size_t lo = std::min(want, piece * t), len = std::min(want, lo + piece) - lo;
        total += got[t];
        if (got[t] < len) {
            f->end = f->pos + static_cast<off_t>(total);
            break;
        }
    }
    f->pos += static_cast<off_t>(total);
    return total;
}
static void fd_sink(void* ctx, size_t first, const uint8_t* dig, size_t count) {
    FdSink* s = static_cast<FdSink*>(ctx);
    for (size_t j = 0; j < count; ++j)
        if (first + j < s->max && s->out) memcpy(s->out + 20 * (first + j), dig + 20 * j, 20);
}
}  // namespace

namespace {
// SHA1CHUNK_FILE_DEVICES (make_chunks on a regular file): how many devices
// share the file -- "all", or a count (default 1).  Each device hashes a
// contiguous, chunk-aligned byte range with its own pread pool, host thread
// and pipeline; digests land in disjoint slices of the caller's array (the
// chunk list split per device, SURVEY.md 8e: no collective).
int file_devices(uint64_t bytes) {
    const char* e = getenv("SHA1CHUNK_FILE_DEVICES");
    if (!e) return 1;
    const int nd = device_count();
    if (nd <= 1) return 1;
    const int want = strcmp(e, "all") == 0 ? nd : std::max(1, std::min(nd, atoi(e)));
    // at least one chunk per device
    const uint64_t chunks = (bytes + SHA1CHUNK_CHUNK_LEN - 1) / SHA1CHUNK_CHUNK_LEN;
    return static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(want, chunks)));
}

long hash_file_devices(int fd, off_t pos, off_t end, int nd, int read_threads, FdSink* sk) {
    const uint64_t L = SHA1CHUNK_CHUNK_LEN;
    const uint64_t chunks = (static_cast<uint64_t>(end - pos) + L - 1) / L;
    std::vector<long> got(nd, 0);
    std::vector<off_t> stop(nd, 0);
    std::vector<std::string> errs(nd);
    std::vector<std::thread> th;
    const int caller_dev = t_dev;
    for (int g = 0; g < nd; ++g) {
        th.emplace_back([&, g] {
            t_dev = (caller_dev + g) % device_count();
            const uint64_t c0 = chunks * g / nd, c1 = chunks * (g + 1) / nd;
            const off_t a = pos + static_cast<off_t>(c0 * L);
            const off_t b = std::min(end, pos + static_cast<off_t>(c1 * L));
            PartPool pool(std::max(1, read_threads) - 1, near_cpus(g_dev[t_dev].id));
            ParFile f{fd, a, b, &pool};
            struct Shift {
                FdSink* sk;
                uint64_t c0;
            } sh{sk, c0};
            auto sink = [](void* ctx, size_t first, const uint8_t* dig, size_t count) {
                Shift* z = static_cast<Shift*>(ctx);
                fd_sink(z->sk, z->c0 + first, dig, count);
            };
            got[g] = hash_stream_sized(par_reader, &f, sink, &sh, static_cast<uint64_t>(b - a));
            stop[g] = f.pos;
            if (got[g] < 0) errs[g] = t_err;
        });
    }
    for (auto& t : th) t.join();
    long n = 0;
    for (int g = 0; g < nd; ++g) {
        if (got[g] < 0) return fail(static_cast<int>(got[g]), "device %d: %s", g, errs[g].c_str());
        const uint64_t c0 = chunks * g / nd, c1 = chunks * (g + 1) / nd;
        n += got[g];
        // a range that came up short (the file shrank) ends the file there
        if (static_cast<uint64_t>(got[g]) < c1 - c0) {
            (void)lseek(fd, stop[g], SEEK_SET);
            return n;
        }
    }
    (void)lseek(fd, stop[nd - 1], SEEK_SET);
    return n;
}
}  // namespace


long s1be_hash_fd(int fd, uint8_t* digests, size_t max_chunks, size_t* total_chunks) {
    FdSink sk{digests, max_chunks};
    struct stat st;
    const off_t pos = lseek(fd, 0, SEEK_CUR);
    long n;
    if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && pos >= 0) {
        const char* e = getenv("SHA1CHUNK_READ_THREADS");
        const int read_threads = e ? std::max(1, atoi(e)) : 8;
        const off_t end = std::max(pos, st.st_size);
        const int nd = file_devices(static_cast<uint64_t>(end - pos));
        if (nd > 1) {
            n = hash_file_devices(fd, pos, end, nd, read_threads, &sk);
        } else {
            PartPool pool(read_threads - 1, near_cpus(g_dev[t_dev].id));
            ParFile f{fd, pos, end, &pool};
            n = hash_stream_sized(par_reader, &f, fd_sink, &sk, static_cast<uint64_t>(f.end - f.pos));
            (void)lseek(fd, f.pos, SEEK_SET);
        }
    } else {
        n = hash_stream_sized(fd_reader, &fd, fd_sink, &sk, 0);
    }
    if (n < 0) return n;
    if (total_chunks) *total_chunks = static_cast<size_t>(n);
    return static_cast<long>(std::min(static_cast<size_t>(n), max_chunks));
}

int s1be_compress_blocks(uint32_t state[5], const void* blocks, size_t nblocks) {
    if (!state || (nblocks && !blocks)) return fail(SHA1CHUNK_EINVAL, "null pointer");
    if (nblocks == 0) return SHA1CHUNK_OK;
    if (nblocks * 64 > 0xffffffffull) return fail(SHA1CHUNK_EINVAL, "too many blocks");
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(D->mu);
    const size_t bytes = nblocks * 64;
    if ((rc = D->small.ensure(64 + bytes)) || (rc = D->small_pin.ensure(64 + bytes))) return rc;
    uint8_t* h = static_cast<uint8_t*>(D->small_pin.p);
    memcpy(h, state, 20);
    memcpy(h + 64, blocks, bytes);
    hipStream_t st = D->slot[0].stream;
    HIP_TRY(hipMemcpyAsync(D->small.p, h, 64 + bytes, hipMemcpyHostToDevice, st));
    uint8_t* d = static_cast<uint8_t*>(D->small.p);
    BatchArgs A{};
    A.base = d + 64;
    A.ulen = static_cast<uint32_t>(bytes);
    A.n = 1;
    A.init_state = reinterpret_cast<const uint32_t*>(d);
    A.out_state = reinterpret_cast<uint32_t*>(d + 32);
    if ((rc = launch_checked(choose_kernel(SHA1CHUNK_KERNEL_AUTO, 1, D->cus), A, st, D->cus))) return rc;
    HIP_TRY(hipMemcpyAsync(h + 32, d + 32, 20, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    memcpy(state, h + 32, 20);
    return SHA1CHUNK_OK;
}

int s1be_finish(const uint32_t state[5], uint64_t prefix_bytes, const void* tail,
                     uint32_t tail_len, uint8_t digest[20]) {
    if (!state || !digest || (tail_len && !tail) || tail_len >= 64)
        return fail(SHA1CHUNK_EINVAL, "bad argument");
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(D->mu);
    if ((rc = D->small.ensure(256)) || (rc = D->small_pin.ensure(256))) return rc;
    uint8_t* h = static_cast<uint8_t*>(D->small_pin.p);
    memcpy(h, state, 20);
    if (tail_len) memcpy(h + 64, tail, tail_len);
    hipStream_t st = D->slot[0].stream;
    HIP_TRY(hipMemcpyAsync(D->small.p, h, 128, hipMemcpyHostToDevice, st));
    uint8_t* d = static_cast<uint8_t*>(D->small.p);
    BatchArgs A{};
    A.base = d + 64;
    A.ulen = tail_len;
    A.n = 1;
    A.init_state = reinterpret_cast<const uint32_t*>(d);
    A.prefix_bytes = prefix_bytes;
    A.dig = d + 128;
    if ((rc = launch_checked(SHA1CHUNK_KERNEL_LANE, A, st))) return rc;
    HIP_TRY(hipMemcpyAsync(h + 128, d + 128, 20, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    memcpy(digest, h + 128, 20);
    return SHA1CHUNK_OK;
}

int s1be_synth_fill_async(void* d_dst, uint64_t first, uint64_t count, uint32_t chunk_len,
                               uint64_t seed, void* stream) {
    if (count && !d_dst) return fail(SHA1CHUNK_EINVAL, "null pointer");
    if ((reinterpret_cast<uintptr_t>(d_dst) & 7u) || (chunk_len & 7u && count > 1))
        return fail(SHA1CHUNK_EALIGN, "synthetic chunks must start 8-byte aligned");
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    hipError_t e = launch_synth(static_cast<uint8_t*>(d_dst), nullptr, nullptr, chunk_len, first,
                                count, seed, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "synth launch: %s", hipGetErrorString(e));
    return SHA1CHUNK_OK;
}

int s1be_synth_fill_ragged_async(void* d_base, const uint64_t* d_offsets,
                                      const uint32_t* d_lengths, uint64_t first, uint64_t count,
                                      uint64_t seed, void* stream) {
    if (count && (!d_base || !d_offsets || !d_lengths)) return fail(SHA1CHUNK_EINVAL, "null pointer");
    Device* D;
    int rc = get_device(&D);
    if (rc) return rc;
    hipError_t e = launch_synth(static_cast<uint8_t*>(d_base), d_offsets, d_lengths, 0, first,
                                count, seed, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "synth launch: %s", hipGetErrorString(e));
    return SHA1CHUNK_OK;
}

}  // extern "C"

// ------------------------------------------------------------ verify queue --
// Three fill/flight sets per queue: while earlier sets' batches are copied
// to the device, hashed and compared, submissions fill the next one.  With
// two, a batch of 1024 chunks had to wait for its set's H2D + kernel (~15
// ms) and the queue topped out near 30 GiB/s (profiles/file_vq_r01.json).
// Set layout (pinned host and device alike): [off u64 x B][len u32 x B]
// [expected 20 x B] pad to 128 | B slots of `stride` bytes; the device side
// adds B x 20 digests and B mismatch bytes.
namespace {
constexpr int kVqSets = 3;

int vq_copy_helpers() {
    const char* e = getenv("SHA1CHUNK_VQ_THREADS");
    // threads in all, the caller included.  Default 1: the calling thread
    // copies the chunk it has just filled (hot in its own core's caches);
    // helper threads on other cores have to pull it across the fabric and
    // cost more than they add.  16384 x 512 KiB, 1484-byte fills, receive
    // threads one per L3 domain (profiles/vq_threads*_r06.jsonl): 1 / 4
    // receive threads at 1 copy thread 18.5 / 46.7 GiB/s, at 4 7.7 / 26.8
    // (persistent queue; batch mode 19.3 / 29.2 against 8.8 / 22.4, and the
    // same with a DRAM-resident source).  Round 2 had measured 4 best (16.9
    // / 46.4 / 36.5 GiB/s for 1 / 4 / 8 on one thread submitting batches of
    // 1024) on the round-2 queue.
    return std::max(0, (e ? atoi(e) : 1) - 1);
}

struct VqSet {
    PinBuf h;
    DevBuf d;
    PinBuf res;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    std::vector<uint64_t> tags;
    size_t count = 0;
    bool inflight = false;
};
}  // namespace

namespace {
struct Pvq;
}

struct s1be_vq {
    Pvq* pv = nullptr;  // the persistent drain (default), or null: batch launches (SHA1CHUNK_VQ_MODE=batch)
    int dev = 0;
    int cus = 256;
    size_t batch = 0;  // launch threshold
    size_t cap = 0;    // chunks a set holds: a batch grows up to this while the device is busy
    uint32_t maxlen = 0;
    size_t stride = 0, meta = 0;
    VqSet set[kVqSets];
    int fill = 0;
    std::deque<int> flight;  // launched sets, oldest first
    std::deque<std::pair<uint64_t, uint8_t>> ready;
    size_t pending = 0;
    PartPool* copier = nullptr;
    std::mutex mu;  // every entry point holds it: a queue may be shared by threads
    // batch mode's reservations: buffer -> (length, storage)
    std::unordered_map<void*, std::pair<uint32_t, std::unique_ptr<uint8_t[]>>> reserved;
    // SHA1CHUNK_VQ_STATS=1: per entry point (submit, reserve, commit, release,
    // poll, other) the calls, ns spent waiting for `mu` and ns holding it;
    // printed as one JSON line to stderr by destroy (diagnostics)
    bool stats = false;
    uint64_t st_calls[6] = {}, st_wait_ns[6] = {}, st_hold_ns[6] = {};
};

namespace {

uint64_t* vq_off(s1be_vq*, uint8_t* base) { return reinterpret_cast<uint64_t*>(base); }  // offsets lead the set
uint32_t* vq_len(s1be_vq* q, uint8_t* base) {
    return reinterpret_cast<uint32_t*>(base + q->cap * 8);
}
uint8_t* vq_exp(s1be_vq* q, uint8_t* base) { return base + q->cap * 12; }

int vq_launch(s1be_vq* q, int which) {
    VqSet& S = q->set[which];
    if (S.count == 0) return SHA1CHUNK_OK;
    HIP_TRY(hipSetDevice(q->dev));
    uint8_t* h = static_cast<uint8_t*>(S.h.p);
    uint8_t* d = static_cast<uint8_t*>(S.d.p);
    HIP_TRY(hipMemcpyAsync(d, h, q->meta + S.count * q->stride, hipMemcpyHostToDevice, S.stream));
    uint8_t* ddig = d + q->meta + q->cap * q->stride;
    uint8_t* dmis = ddig + q->cap * 20;
    BatchArgs A{};
    A.base = d;
    A.off = vq_off(q, d);
    A.len = vq_len(q, d);
    A.n = static_cast<uint32_t>(S.count);
    A.dig = ddig;
    int rc = launch_checked(choose_kernel(SHA1CHUNK_KERNEL_AUTO, S.count, q->cus), A, S.stream, q->cus);
    if (rc) return rc;
    hipError_t e = launch_compare(ddig, vq_exp(q, d), static_cast<uint32_t>(S.count), dmis, S.stream);
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "compare launch: %s", hipGetErrorString(e));
    HIP_TRY(hipMemcpyAsync(S.res.p, dmis, S.count, hipMemcpyDeviceToHost, S.stream));
    HIP_TRY(hipEventRecord(S.done, S.stream));
    S.inflight = true;
    q->flight.push_back(which);
    return SHA1CHUNK_OK;
}

// Move the oldest launched set's results to `ready` (blocking on it).
int vq_collect_oldest(s1be_vq* q) {
    if (q->flight.empty()) return SHA1CHUNK_OK;
    const int which = q->flight.front();
    VqSet& S = q->set[which];
    HIP_TRY(hipEventSynchronize(S.done));
    const uint8_t* r = static_cast<const uint8_t*>(S.res.p);
    for (size_t i = 0; i < S.count; ++i) q->ready.emplace_back(S.tags[i], r[i]);
    S.tags.clear();
    S.count = 0;
    S.inflight = false;
    q->flight.pop_front();
    return SHA1CHUNK_OK;
}

// Collect every launched set that has finished, oldest first, without
// blocking.
int vq_reap(s1be_vq* q) {
    while (!q->flight.empty()) {
        hipError_t e = hipEventQuery(q->set[q->flight.front()].done);
        if (e == hipErrorNotReady) break;
        if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "vq: %s", hipGetErrorString(e));
        int rc = vq_collect_oldest(q);
        if (rc) return rc;
    }
    return SHA1CHUNK_OK;
}

// Launch the fill set once it holds `batch` chunks, unless the device is
// busy with kVqSets - 1 earlier sets: then the set keeps growing, a batch at
// a time (up to `cap`), and goes at the first whole batch after one of them
// finishes.  Every launch costs at
// least one chunk's serial hash time (~6 ms), so while the device is busy a
// bigger batch is free throughput; while it is idle, `batch` bounds latency.
int vq_maybe_launch(s1be_vq* q) {
    VqSet& S = q->set[q->fill];
    // only at whole multiples of `batch`: a caller that submits whole batches
    // still gets every result back through non-blocking polls, no flush
    if (S.inflight || S.count < q->batch || S.count % q->batch) return SHA1CHUNK_OK;
    int rc = vq_reap(q);
    if (rc) return rc;
    if (S.count < q->cap && q->flight.size() >= static_cast<size_t>(kVqSets - 1)) return SHA1CHUNK_OK;
    if ((rc = vq_launch(q, q->fill))) return rc;
    q->fill = (q->fill + 1) % kVqSets;
    return SHA1CHUNK_OK;
}

// ------------------------------------------------ persistent verify queue --
// s1be_vq with a persistent drain kernel (sha1_vq_drain_kernel): the
// host copies each submitted chunk into a ring in pinned, uncached host
// memory, writes its length and expected digest next to it, and publishes
// groups of up to 64 chunks by bumping `pub`.  The drain -- one workgroup
// per CU on SHA1CHUNK_VQ_CUS CUs, (re)launched whenever work is published
// and fewer of its workgroups are alive than that, gone again after
// SHA1CHUNK_VQ_IDLE_MS (default 20) without a claim -- reads the ring over
// PCIe, hashes each group in the one-group split shape and writes
// one 0/1 per chunk plus the group's completion word back to host memory.
// No copy engine, no launch per batch: a chunk starts hashing as soon as
// its group is published.  A group is published when it holds
// min(batch, 64) chunks, or at once while fewer groups are in flight than
// the drain has workgroups (so at low rates every chunk goes alone and comes
// back after its own serial chain, ~6 ms for 512 KiB, whatever the batch
// size).  The drain takes SHA1CHUNK_VQ_CUS CUs (default 64 of 256): the
// queue is PCIe-bound (64 groups of 64 chunks in flight are far more than
// the link feeds), and the rest of the GPU stays free for the process's
// other kernels, which could not share a CU with a drain workgroup (it holds
// the CU's whole LDS).
// Positions in both rings are monotonic counters (physical = counter mod
// ring size).  A group is a run of consecutive slots that never wraps the
// slot ring; each slot points at its chunk's region of the data ring, a
// region never wraps the data ring, and regions are freed in allocation
// order (the data ring's head is the oldest region still held).
// Zero-copy receive (sha1chunk_vq_reserve / commit / release): the caller
// fills a region in place -- the peer's session buffer (reliable_udp.c:121,
// filled at :339) -- and commits it, which gives it a slot; the region stays
// the caller's after its result is collected, until the caller releases it
// (after copying the verified chunk into its job buffer, reliable_udp.c:
// 696-709).  A submitted (copied) chunk's region is freed when its result
// is collected.
constexpr uint32_t kPvqMaxGroup = 64;
struct PvqCtl {
    uint32_t pub;        // groups published (host store, release)
    uint32_t stop;       // destroy: exit once nothing is claimable
    uint32_t last_done;  // drain: index + 1 of the group it finished last
    uint32_t pad[29];
    uint8_t alive[2][1024];   // per launch slot, per workgroup (bytes: 16 per uncached read)
};
struct PvqGroup {
    uint64_t g;         // group index
    uint64_t slot0;     // first slot (monotonic)
    uint32_t count;
    bool collected;
};
// A byte range of the data ring [start, end) (monotonic positions).
struct PvqRegion {
    uint64_t start, end;
    bool reserved;   // handed out by reserve(): freed by release()
    bool committed;  // a slot refers to it: its result is pending until collected
    bool collected;
    bool released;
    std::thread::id owner;  // the thread that allocated it (reserve or submit)
};
struct Pvq {
    int dev = 0, cus = 256;  // cus: the drain's workgroups (one per CU)
    uint32_t nslots = 0;  // slot ring (chunks) = group ring entries
    uint64_t nbytes = 0;  // data ring bytes
    uint32_t maxlen = 0;
    uint32_t group_max = kPvqMaxGroup;
    uint64_t idle_ticks = 0, life_ticks = 0;
    // pinned, uncached host memory: data ring, then the per-slot and
    // per-group arrays, then the control words
    uint8_t* hmem = nullptr;
    uint8_t* data = nullptr;
    uint64_t* off = nullptr;
    uint32_t* grp = nullptr;
    uint32_t* len = nullptr;
    uint32_t* done = nullptr;
    uint8_t* exp = nullptr;
    uint8_t* res = nullptr;
    PvqCtl* ctl = nullptr;
    // device memory: digest scratch + the claim counter
    uint8_t* dmem = nullptr;
    std::vector<uint64_t> tags;
    std::vector<uint64_t> slot_reg;  // per slot: its region's id
    std::deque<PvqRegion> regions;   // allocated, not yet freed, oldest first
    uint64_t reg_base = 0;           // id of regions.front()
    std::unordered_map<uint64_t, uint64_t> held;  // reserved regions not released: ring offset -> id
    uint64_t slot_head = 0, slot_tail = 0, byte_head = 0, byte_tail = 0;
    uint32_t seen_done = 0;  // ctl->last_done at the last scan
    std::mutex* mu = nullptr;  // the queue's lock (held by every caller; pvq_wait drops it to sleep)
    std::mutex copy_mu;        // the copy helpers run one submit's copy at a time
    // counters for SHA1CHUNK_VQ_STATS
    uint64_t n_publish = 0, n_published = 0, n_copies = 0, n_launch = 0, n_scans = 0, n_sleeps = 0;
    std::atomic<uint64_t> copy_ns{0};  // submit's copies (outside the lock), all threads
    uint64_t sleep_ns = 0;             // pvq_wait's sleeps (lock dropped), all threads
    int64_t alive_scan_ns = 0;  // pvq_ensure_drain: when it last read the alive words
    int alive_seen = 0;         // and how many it found (or launched)
    uint64_t open_slot0 = 0;
    uint32_t open_count = 0;
    uint64_t next_g = 0;
    std::deque<PvqGroup> groups;  // published, oldest first
    size_t inflight = 0;          // published, not yet collected
    std::deque<std::pair<uint64_t, uint8_t>> ready;
    size_t pending = 0;
    // two launch slots, each a stream, an alive-word set and the event of
    // its last drain; a slot is reused only once that drain has ended
    hipStream_t stream[2] = {nullptr, nullptr};
    hipEvent_t ended[2] = {nullptr, nullptr};
    bool launched[2] = {false, false};
    PartPool* copier = nullptr;
    size_t hbytes = 0;
    unsigned hflags = 0;
    int budget_dev = -1;  // device whose drain CU budget this queue holds (pvq_create)
    // DMA staging (default since round 4; SHA1CHUNK_VQ_DMA=0 turns it off):
    // the data ring lives in ordinary pinned host memory (`hdata`), each
    // published group's chunks are copied by the copy engine into a device
    // mirror of the ring (`ddata`, uncached device memory, the drain reads it
    // from HBM), and the group is released to the drain (`pub`) once its copy
    // event has completed.  The drain reading the ring over PCIe tops out at
    // 26-28 GiB/s (8 receive threads, zero-copy), the copy engine at 37-45
    // (profiles/vq_dma_r04.jsonl, vq_dma_knobs_r04.log).
    bool dma = false;
    uint8_t* hdata = nullptr;
    size_t hdata_bytes = 0;
    uint8_t* ddata = nullptr;
    hipStream_t cstream = nullptr;
    std::deque<std::pair<uint64_t, hipEvent_t>> staged;  // group, its copies' event
    std::vector<hipEvent_t> spare_events;
};

uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* e = getenv(name);
    return e ? strtoull(e, nullptr, 10) : dflt;
}

int pvq_launch(Pvq* P, int k, int wgs) {
    // every workgroup of the new drain counts as alive from here on, so a
    // submit right after does not launch another one
    for (int w = 0; w < wgs; ++w) __atomic_store_n(&P->ctl->alive[k][w], uint8_t{1}, __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    VqDrainArgs Q{};
    Q.data = P->dma ? P->ddata : P->data;
    Q.off = P->off;
    Q.len = P->len;
    Q.exp = P->exp;
    Q.grp = P->grp;
    Q.pub = &P->ctl->pub;
    Q.stop = &P->ctl->stop;
    Q.alive = P->ctl->alive[k];
    Q.res = P->res;
    Q.done = P->done;
    Q.last_done = &P->ctl->last_done;
    Q.dig = P->dmem;
    Q.claim = reinterpret_cast<uint32_t*>(P->dmem + 20ull * P->nslots);
    Q.grp_ring = P->nslots;
    Q.idle_ticks = P->idle_ticks;
    Q.life_ticks = P->life_ticks;
    HIP_TRY(hipSetDevice(P->dev));
    hipError_t e = launch_vq_drain(Q, static_cast<uint32_t>(wgs), P->stream[k]);
    if (e != hipSuccess) return fail(SHA1CHUNK_EHIP, "vq drain launch: %s", hipGetErrorString(e));
    HIP_TRY(hipEventRecord(P->ended[k], P->stream[k]));
    P->launched[k] = true;
    ++P->n_launch;
    return SHA1CHUNK_OK;
}

// After `pub` moved (and while waiting): keep the drain at full strength.
// Workgroups leave when they find nothing to claim, each with the exit
// handshake of sha1_kernels.hip (so no published group is left without a
// live workgroup that sees it), and after their lifetime even under load
// (SHA1CHUNK_VQ_LIFE_MS, so that no drain holds its hardware queue for
// good); the latter relies on this call, which every submit, commit and
// poll makes while groups are in flight.  When fewer than the drain's
// workgroups are alive, the missing ones are launched on a slot whose
// previous drain has ended; the leftovers of the old one keep working.
//
// The alive flags are uncached host memory (a CPU read costs ~0.15 us, and
// every submit, commit and poll lands here under the queue's lock), so they
// are bytes read 16 at a time -- 8 reads for a 64-workgroup drain's two
// launch slots -- and a call that did not move `pub` does not read them again
// within kAliveScanNs of a scan that found the drain at full strength: a
// workgroup that leaves in that window is replaced at most that much later
// (workgroups live >= 4 ms), and the next publish rescans anyway.  A call
// that moved `pub` (publish, or a DMA-staged group released) always reads
// them: that read is the host's half of the exit handshake, so
// a group published just as the drain's last workgroups leave is never left
// unclaimed until some later call.
constexpr int64_t kAliveScanNs = 50000;

int64_t mono_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return int64_t(ts.tv_sec) * 1000000000 + ts.tv_nsec;
}

int count_alive(const uint8_t* a, int n) {
    int c = 0, w = 0;
    for (; w + 16 <= n; w += 16) {  // one 16-byte uncached read per 16 flags
        const __m128i v = _mm_load_si128(reinterpret_cast<const __m128i*>(a + w));
        c += 16 - __builtin_popcount(_mm_movemask_epi8(_mm_cmpeq_epi8(v, _mm_setzero_si128())));
    }
    for (; w < n; ++w) c += __atomic_load_n(a + w, __ATOMIC_ACQUIRE) != 0;
    return c;
}

int pvq_ensure_drain(Pvq* P, bool moved_pub = false) {
    const int64_t now = mono_ns();
    if (!moved_pub && P->alive_seen >= P->cus && now - P->alive_scan_ns < kAliveScanNs) return SHA1CHUNK_OK;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    int alive = 0;
    for (int k = 0; k < 2; ++k)  // a slot never launched has no live workgroup
        if (P->launched[k]) alive += count_alive(P->ctl->alive[k], P->cus);
    ++P->n_scans;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    P->alive_scan_ns = now;
    P->alive_seen = alive;
    if (alive >= P->cus) return SHA1CHUNK_OK;
    for (int k = 0; k < 2; ++k) {
        if (P->launched[k]) {
            const hipError_t q = hipEventQuery(P->ended[k]);
            if (q == hipErrorNotReady) continue;
            if (q != hipSuccess) return fail(SHA1CHUNK_EHIP, "vq drain: %s", hipGetErrorString(q));
        }
        P->alive_seen = P->cus;  // pvq_launch marks the new workgroups alive
        return pvq_launch(P, k, P->cus - alive);
    }
    return SHA1CHUNK_OK;  // both slots' drains still leaving: the next call launches
}

// DMA staging: release every staged group whose copies have landed, in
// order (the copy stream completes them in order), to the drain.
int pvq_release_staged(Pvq* P) {
    bool moved = false;
    while (!P->staged.empty()) {
        const hipError_t q = hipEventQuery(P->staged.front().second);
        if (q == hipErrorNotReady) break;
        if (q != hipSuccess) return fail(SHA1CHUNK_EHIP, "vq copy: %s", hipGetErrorString(q));
        __atomic_store_n(&P->ctl->pub, static_cast<uint32_t>(P->staged.front().first + 1), __ATOMIC_RELEASE);
        P->spare_events.push_back(P->staged.front().second);
        P->staged.pop_front();
        moved = true;
    }
    return moved ? pvq_ensure_drain(P, true) : SHA1CHUNK_OK;
}

// Copy the chunks of slots [slot0, slot0 + count) into the device ring and
// record the group's event.  Receive threads commit in their own order, so a
// group's regions are sorted by ring offset and copied as runs, a run taking
// in gaps of up to kStageGap bytes: one 512 KiB copy runs at ~30 GiB/s on the
// copy engine (15-19 us, profiles), a run of many at the link's rate.  A
// gap's bytes are other reservations' (filling, committed or free): their
// device copy is rewritten with the same or later bytes before any group
// that holds them is released to the drain, and none of them is in a group
// the drain is hashing unless committed (whose bytes no longer change).
constexpr uint64_t kStageGap = 1ull << 20;

int pvq_stage(Pvq* P, uint64_t g, uint64_t slot0, uint32_t count) {
    HIP_TRY(hipSetDevice(P->dev));
    std::pair<uint64_t, uint64_t> rg[kPvqMaxGroup];  // (ring offset, end)
    uint32_t n = 0;
    for (uint32_t j = 0; j < count && n < kPvqMaxGroup; ++j) {
        const PvqRegion& r = P->regions[P->slot_reg[(slot0 + j) % P->nslots] - P->reg_base];
        const uint64_t at = r.start % P->nbytes;
        rg[n++] = {at, at + (r.end - r.start)};
    }
    std::sort(rg, rg + n);
    for (uint32_t i = 0; i < n;) {
        uint64_t run_at = rg[i].first, run_end = rg[i].second;
        for (++i; i < n && rg[i].first <= run_end + kStageGap; ++i) run_end = std::max(run_end, rg[i].second);
        HIP_TRY(hipMemcpyAsync(P->ddata + run_at, P->hdata + run_at, run_end - run_at, hipMemcpyHostToDevice,
                               P->cstream));
        ++P->n_copies;
    }
    hipEvent_t ev;
    if (!P->spare_events.empty()) {
        ev = P->spare_events.back();
        P->spare_events.pop_back();
    } else {
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    HIP_TRY(hipEventRecord(ev, P->cstream));
    P->staged.emplace_back(g, ev);
    return SHA1CHUNK_OK;
}

int pvq_publish(Pvq* P) {
    if (P->open_count == 0) return SHA1CHUNK_OK;
    // the drain indexes a group's slots first..first+count with no modulo
    if (P->open_slot0 % P->nslots + P->open_count > P->nslots || P->open_count > kPvqMaxGroup)
        return fail(SHA1CHUNK_EHIP, "vq: internal: group of %u slots at %llu crosses the slot ring's end",
                    P->open_count, static_cast<unsigned long long>(P->open_slot0 % P->nslots));
    const uint64_t g = P->next_g++;
    const uint32_t gi = static_cast<uint32_t>(g % P->nslots);
    P->grp[2 * gi] = static_cast<uint32_t>(P->open_slot0 % P->nslots);
    P->grp[2 * gi + 1] = P->open_count;
    P->groups.push_back(PvqGroup{g, P->open_slot0, P->open_count, false});
    ++P->inflight;
    const uint64_t slot0 = P->open_slot0;
    const uint32_t count = P->open_count;
    ++P->n_publish;
    P->n_published += count;
    P->open_slot0 = P->slot_tail;
    P->open_count = 0;
    if (P->dma) {
        // released to the drain once its copies land (pvq_release_staged)
        if (int rc = pvq_stage(P, g, slot0, count)) return rc;
        return pvq_release_staged(P);
    }
    // the group's bytes, lengths, digests and descriptor are written: release them
    __atomic_store_n(&P->ctl->pub, static_cast<uint32_t>(g + 1), __ATOMIC_RELEASE);
    return pvq_ensure_drain(P, true);
}

// A region is free once nothing refers to it: a copied chunk once its
// result is collected; a reserved one once the caller released it and its
// result (if it was committed) is collected.
bool region_free(const PvqRegion& r) {
    if (!r.reserved) return r.collected;
    return r.released && (r.collected || !r.committed);
}

// Free the oldest regions that are free; the data ring's head follows.
void pvq_free_regions(Pvq* P) {
    while (!P->regions.empty() && region_free(P->regions.front())) {
        P->regions.pop_front();
        ++P->reg_base;
    }
    P->byte_head = P->regions.empty() ? P->byte_tail : P->regions.front().start;
}

// Collect finished groups (in any order) and free ring space up to the
// oldest unfinished one.  The drain claims groups in publication order and
// runs at most one per CU at a time, so the scan stops after 2 x CUs
// unfinished groups in a row: a submit costs O(CUs), not O(groups in flight).
int pvq_reap(Pvq* P) {
    if (P->dma && !P->staged.empty())
        if (int rc = pvq_release_staged(P)) return rc;
    // The completion words live in uncached host memory (~0.1-0.2 us per
    // CPU read); every submit, reserve and commit reaps, so scan them only
    // when the drain's last-finished word moved since the last scan (each
    // group writes its own index there, so the word changes whenever any
    // group finished).
    const uint32_t ld = __atomic_load_n(&P->ctl->last_done, __ATOMIC_ACQUIRE);
    if (ld == P->seen_done) return SHA1CHUNK_OK;
    bool whole = true;  // the scan reached the end (else scan again next time)
    size_t unfinished = 0;
    for (auto& G : P->groups) {
        if (G.collected) continue;
        const uint32_t gi = static_cast<uint32_t>(G.g % P->nslots);
        if (__atomic_load_n(&P->done[gi], __ATOMIC_ACQUIRE) != static_cast<uint32_t>(G.g + 1)) {
            if (++unfinished > 2 * static_cast<size_t>(P->cus)) {
                whole = false;
                break;
            }
            continue;
        }
        unfinished = 0;
        for (uint32_t j = 0; j < G.count; ++j) {
            const uint64_t sl = (G.slot0 + j) % P->nslots;
            P->ready.emplace_back(P->tags[sl], P->res[sl]);
            P->regions[P->slot_reg[sl] - P->reg_base].collected = true;
        }
        G.collected = true;
        --P->inflight;
    }
    while (!P->groups.empty() && P->groups.front().collected) {
        P->slot_head = P->groups.front().slot0 + P->groups.front().count;
        P->groups.pop_front();
    }
    if (P->groups.empty()) P->slot_head = P->open_slot0;
    if (whole) P->seen_done = ld;
    pvq_free_regions(P);
    return SHA1CHUNK_OK;
}

int pvq_publish(Pvq* P);

// Wait (bounded) until `pred` holds, reaping and keeping a drain alive.
// An open group is published first (its chunks hold ring space too), and a
// wait that only the caller can end -- the oldest region of the data ring
// is a reserved buffer not yet committed, or collected and not released --
// fails at once when `stuck` says so.
// Bound on any one wait (SHA1CHUNK_VQ_WAIT_S, default 120 s).
std::chrono::seconds pvq_wait_bound() {
    static const std::chrono::seconds b(std::max<uint64_t>(1, env_u64("SHA1CHUNK_VQ_WAIT_S", 120)));
    return b;
}

template <typename Pred, typename Stuck>
int pvq_wait(Pvq* P, Pred pred, const char* what, Stuck stuck) {
    const auto t0 = std::chrono::steady_clock::now();
    int rc;
    for (;;) {
        if ((rc = pvq_reap(P))) return rc;
        if (pred()) return SHA1CHUNK_OK;
        if (P->open_count && (rc = pvq_publish(P))) return rc;
        if (const char* why = stuck())
            return fail(SHA1CHUNK_ENOMEM, "vq: %s: the ring's oldest region is %s (%zu reserved buffers held)", what,
                        why, P->held.size());
        if (P->inflight && (rc = pvq_ensure_drain(P))) return rc;
        if (std::chrono::steady_clock::now() - t0 > pvq_wait_bound())
            return fail(SHA1CHUNK_EHIP, "vq: %s timed out (drain not progressing)", what);
        ++P->n_sleeps;
        // sleep without the queue's lock: the other threads' commits, polls
        // and releases are what frees the ring (each call re-checks its state
        // after the wait)
        const int64_t z0 = mono_ns();
        if (P->mu) P->mu->unlock();
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (P->mu) P->mu->lock();
        P->sleep_ns += static_cast<uint64_t>(mono_ns() - z0);
    }
}
template <typename Pred>
int pvq_wait(Pvq* P, Pred pred, const char* what) {
    return pvq_wait(P, pred, what, [] { return static_cast<const char*>(nullptr); });
}

// Queues alive at process exit (a caller that never destroys its queue):
// an exit handler raises every live drain's stop word and waits for its
// launches, so no drain wave is still polling the pinned ring when the
// runtime and the process's mappings go away.  The handler is registered at
// the first queue, after HIP's own start-up, so it runs before HIP's
// teardown (exit handlers run in reverse order).
std::mutex g_pvq_mu;
std::vector<Pvq*>* g_pvq_live = nullptr;
void pvq_stop_all_at_exit();
void pvq_track(Pvq* P, bool add) {
    std::lock_guard<std::mutex> lk(g_pvq_mu);
    if (!g_pvq_live) {
        if (!add) return;
        g_pvq_live = new std::vector<Pvq*>();
        std::atexit(pvq_stop_all_at_exit);
    }
    auto& v = *g_pvq_live;
    if (add)
        v.push_back(P);
    else
        v.erase(std::remove(v.begin(), v.end(), P), v.end());
}

// Pinned rings of destroyed queues, kept for the next queue of the same
// size: hipHostFree (like hipFree) can wait for the whole device, i.e. for
// other threads' busy drains, so a queue's destroy never frees its ring.
std::mutex g_ring_mu;
std::vector<std::tuple<uint8_t*, size_t, unsigned>> g_ring_cache;
constexpr size_t kRingCacheMax = 8;

uint8_t* ring_get(size_t bytes, unsigned flags) {
    {
        std::lock_guard<std::mutex> lk(g_ring_mu);
        for (size_t i = 0; i < g_ring_cache.size(); ++i)
            if (std::get<1>(g_ring_cache[i]) == bytes && std::get<2>(g_ring_cache[i]) == flags) {
                uint8_t* p = std::get<0>(g_ring_cache[i]);
                g_ring_cache.erase(g_ring_cache.begin() + i);
                return p;
            }
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, flags) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t*>(p);
}

void ring_put(uint8_t* p, size_t bytes, unsigned flags) {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    if (g_ring_cache.size() < kRingCacheMax) {
        g_ring_cache.emplace_back(p, bytes, flags);
        return;
    }
    (void)hipHostFree(p);  // beyond the cache: rare (more than kRingCacheMax queues destroyed at once)
}

// Device mirrors of DMA-staged rings, kept like the pinned rings (hipFree
// can wait for the whole device).
std::vector<std::tuple<int, uint8_t*, size_t>> g_dring_cache;

uint8_t* dring_get(int dev, size_t bytes) {
    {
        std::lock_guard<std::mutex> lk(g_ring_mu);
        for (size_t i = 0; i < g_dring_cache.size(); ++i)
            if (std::get<0>(g_dring_cache[i]) == dev && std::get<2>(g_dring_cache[i]) == bytes) {
                uint8_t* p = std::get<1>(g_dring_cache[i]);
                g_dring_cache.erase(g_dring_cache.begin() + i);
                return p;
            }
    }
    void* p = nullptr;
    // uncached device memory: the drain's loads go to HBM, never to an L2
    // line left from the ring's previous lap (the copy engine does not
    // invalidate the XCDs' L2)
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t*>(p);
}

void dring_put(int dev, uint8_t* p, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    if (g_dring_cache.size() < kRingCacheMax) {
        g_dring_cache.emplace_back(dev, p, bytes);
        return;
    }
    (void)hipFree(p);
}

// Share of the device's CUs a drain takes (SHA1CHUNK_VQ_CUS, default 64),
// within a per-device budget for all drains (SHA1CHUNK_VQ_CU_BUDGET,
// default half the CUs) so that queues never hold every CU: a drain
// workgroup takes a whole CU while its queue is busy, and a process's hash
// kernels and other queues need the rest.  0 when the budget is spent.
int drain_cus_take(Device* D) {
    const int want = static_cast<int>(
        std::max<uint64_t>(1, std::min<uint64_t>({static_cast<uint64_t>(D->cus), 1024, env_u64("SHA1CHUNK_VQ_CUS", 64)})));
    const int budget = static_cast<int>(std::min<uint64_t>(
        static_cast<uint64_t>(D->cus), env_u64("SHA1CHUNK_VQ_CU_BUDGET", static_cast<uint64_t>(D->cus / 2))));
    std::lock_guard<std::mutex> lk(D->drain_mu);
    const int left = budget - D->drain_cus;
    const int take = std::min(want, left);
    if (take < std::min(want, 8)) return 0;  // too few left to be worth a drain
    D->drain_cus += take;
    return take;
}

void drain_cus_give(int dev, int cus) {
    if (dev < 0 || dev >= g_count) return;
    std::lock_guard<std::mutex> lk(g_dev[dev].drain_mu);
    g_dev[dev].drain_cus -= cus;
}

void pvq_destroy(Pvq* P) {
    if (!P) return;
    pvq_track(P, false);
    (void)hipSetDevice(P->dev);
    if (P->ctl) {
        __atomic_store_n(&P->ctl->stop, 1u, __ATOMIC_RELEASE);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
    }
    // Wait for this queue's own work only (never the whole device): both
    // drain slots and the copy stream.  The device scratch (claim counter,
    // digests) is freed only after both drains have ended -- a drain still
    // running on slot 1 would otherwise write into memory the pool already
    // handed to the next queue.
    for (int k = 0; k < 2; ++k)
        if (P->stream[k]) (void)hipStreamSynchronize(P->stream[k]);
    if (P->cstream) {
        (void)hipStreamSynchronize(P->cstream);
        (void)hipStreamDestroy(P->cstream);
    }
    if (P->dmem && P->stream[0]) {
        (void)hipFreeAsync(P->dmem, P->stream[0]);
        (void)hipStreamSynchronize(P->stream[0]);
    }
    for (auto& st : P->staged) (void)hipEventDestroy(st.second);
    for (hipEvent_t ev : P->spare_events) (void)hipEventDestroy(ev);
    if (P->hdata) ring_put(P->hdata, P->hdata_bytes, hipHostMallocDefault);
    if (P->ddata) dring_put(P->dev, P->ddata, P->nbytes);
    for (int k = 0; k < 2; ++k) {
        if (P->ended[k]) (void)hipEventDestroy(P->ended[k]);
        if (P->stream[k]) (void)hipStreamDestroy(P->stream[k]);
    }
    if (P->hmem) ring_put(P->hmem, P->hbytes, P->hflags);
    drain_cus_give(P->budget_dev, P->cus);
    delete P->copier;
    delete P;
}

// Ring memory (SHA1CHUNK_VQ_RING_MEM): "uncached" (default) or "coherent"
// pinned host memory; the drain reads it over PCIe while the host writes.
unsigned ring_flags() {
    const char* e = getenv("SHA1CHUNK_VQ_RING_MEM");
    return e && !strcmp(e, "coherent") ? hipHostMallocCoherent : hipHostMallocUncached;
}

// The verify queue's own streams (its drains' two launch slots and its copy
// stream) are created at a priority of their own (SHA1CHUNK_VQ_PRIO: "low",
// the default, "normal" or "high").  HIP serves a process's streams from a
// few hardware queues (GPU_MAX_HW_QUEUES, 4) and streams of different
// priorities from different ones, so a queue's persistent drain and the
// barrier packets its copy stream's events leave behind (each waits for a
// staged copy on the copy engine) never sit in front of the caller's own
// work -- a hash batch on a stream of the default priority.
int vq_stream_create(hipStream_t* s) {
    const char* e = getenv("SHA1CHUNK_VQ_PRIO");
    const std::string want = e ? e : "low";
    if (want == "normal") return hipStreamCreateWithFlags(s, hipStreamNonBlocking) == hipSuccess ? 0 : -1;
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return -1;
    const int prio = want == "high" ? greatest : least;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, prio) == hipSuccess ? 0 : -1;
}

// The device's logical index for D (the CU budget lives there).
int device_index(Device* D) { return static_cast<int>(D - g_dev); }

Pvq* pvq_create(Device* D, size_t batch, uint32_t max_chunk_len, int cus) {
    auto* P = new Pvq();
    P->dev = D->id;
    P->cus = cus;
    P->budget_dev = device_index(D);
    P->maxlen = max_chunk_len;
    P->group_max = static_cast<uint32_t>(std::min<size_t>(batch, kPvqMaxGroup));
    P->idle_ticks = env_u64("SHA1CHUNK_VQ_IDLE_MS", 20) * 100000ull;  // s_memrealtime: 100 MHz
    P->life_ticks = std::max<uint64_t>(1, env_u64("SHA1CHUNK_VQ_LIFE_MS", 4)) * 100000ull;
    const uint64_t stride = round_up(max_chunk_len, kAlign);
    const uint64_t ring_mib = std::max<uint64_t>(env_u64("SHA1CHUNK_VQ_RING_MIB", 1024), 1);
    P->nbytes = round_up(std::max<uint64_t>(ring_mib << 20, 2 * kPvqMaxGroup * stride), kAlign);
    // slots: room for the ring's bytes in chunks of a quarter of the max length
    P->nslots = static_cast<uint32_t>(std::min<uint64_t>(
        std::max<uint64_t>(P->nbytes / std::max<uint64_t>(kAlign, stride / 4), 4 * kPvqMaxGroup), 1u << 20));
    const size_t ns = P->nslots;
    const size_t meta = round_up(ns * 45, 4096);  // off 8, grp 8, len 4, done 4, exp 20, res 1
    // with DMA staging the data ring is ordinary (cached) pinned memory of its
    // own, read only by the copy engine; the slot arrays and control words
    // stay in uncached memory the drain polls
    P->dma = env_u64("SHA1CHUNK_VQ_DMA", 1) != 0;
    const size_t inline_data = P->dma ? 0 : P->nbytes;
    P->hbytes = inline_data + meta + sizeof(PvqCtl);
    P->hflags = ring_flags();
    if (!(P->hmem = ring_get(P->hbytes, P->hflags)) &&
        (P->hflags == hipHostMallocCoherent ||
         !(P->hmem = ring_get(P->hbytes, P->hflags = hipHostMallocCoherent)))) {
        fail(SHA1CHUNK_ENOMEM, "vq: pinned ring of %zu bytes", P->hbytes);
        pvq_destroy(P);
        return nullptr;
    }
    if (P->dma) {
        P->hdata_bytes = P->nbytes;
        if (!(P->hdata = ring_get(P->nbytes, hipHostMallocDefault)) || !(P->ddata = dring_get(P->dev, P->nbytes)) ||
            vq_stream_create(&P->cstream) != 0) {
            (void)hipGetLastError();
            fail(SHA1CHUNK_ENOMEM, "vq: DMA-staged ring of %llu bytes", static_cast<unsigned long long>(P->nbytes));
            pvq_destroy(P);
            return nullptr;
        }
    }
    memset(P->hmem + inline_data, 0, meta + sizeof(PvqCtl));
    uint8_t* m = P->hmem + inline_data;
    P->data = P->dma ? P->hdata : P->hmem;
    P->off = reinterpret_cast<uint64_t*>(m);
    P->grp = reinterpret_cast<uint32_t*>(m + ns * 8);
    P->len = reinterpret_cast<uint32_t*>(m + ns * 16);
    P->done = reinterpret_cast<uint32_t*>(m + ns * 20);
    P->exp = m + ns * 24;
    P->res = m + ns * 44;
    P->ctl = reinterpret_cast<PvqCtl*>(P->hmem + inline_data + meta);
    P->tags.assign(ns, 0);
    P->slot_reg.assign(ns, 0);
    // streams first: the device scratch is allocated and cleared in stream
    // order on stream 0, so creating a queue never waits for the whole device
    // (other threads' drains and batches)
    for (int k = 0; k < 2; ++k)
        if (vq_stream_create(&P->stream[k]) != 0 ||
            hipEventCreateWithFlags(&P->ended[k], hipEventDisableTiming) != hipSuccess) {
            fail(SHA1CHUNK_EHIP, "vq: stream creation");
            pvq_destroy(P);
            return nullptr;
        }
    if (hipMallocAsync(reinterpret_cast<void**>(&P->dmem), 20ull * ns + 256, P->stream[0]) != hipSuccess ||
        hipMemsetAsync(P->dmem + 20ull * ns, 0, 256, P->stream[0]) != hipSuccess ||
        hipStreamSynchronize(P->stream[0]) != hipSuccess) {
        (void)hipGetLastError();
        fail(SHA1CHUNK_ENOMEM, "vq: device scratch");
        pvq_destroy(P);
        return nullptr;
    }
    P->copier = new PartPool(vq_copy_helpers(), near_cpus(P->dev));
    pvq_track(P, true);
    return P;
}

void pvq_stop_all_at_exit() {
    std::lock_guard<std::mutex> lk(g_pvq_mu);
    if (!g_pvq_live) return;
    for (Pvq* P : *g_pvq_live)
        if (P->ctl) __atomic_store_n(&P->ctl->stop, 1u, __ATOMIC_RELEASE);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    for (Pvq* P : *g_pvq_live) {
        (void)hipSetDevice(P->dev);
        for (int k = 0; k < 2; ++k)
            if (P->stream[k]) (void)hipStreamSynchronize(P->stream[k]);
    }
}

// Room for `len` bytes in the data ring (a region never wraps it): a bounded
// wait while in-flight groups can free space.  Returns the new region's id.
constexpr auto kHeldResultWait = std::chrono::milliseconds(2);
int pvq_alloc(Pvq* P, uint32_t len, bool reserved, uint64_t* id) {
    const uint64_t need = round_up(std::max<uint32_t>(len, 1), kAlign);
    auto pos = [&] {
        const uint64_t t = P->byte_tail;
        return (t % P->nbytes) + need > P->nbytes ? t + (P->nbytes - t % P->nbytes) : t;
    };
    // The wait is hopeless when the ring's head is
    //  * the caller's own reservation, not committed (this thread cannot
    //    commit it while it waits here), or
    //  * a reserved buffer whose result is finished but that is not released,
    //    whoever holds it: only a poll() that hands out the result and the
    //    release() after it free that room.  When every receive thread sits in
    //    reserve() nobody polls, so after a short grace (another thread may be
    //    polling and releasing right now) the call fails and its caller polls
    //    and releases (round 6: four receive threads all waiting here stalled
    //    for the whole 120 s bound).
    // Another thread's reservation not yet committed is a session still
    // filling, which that thread will commit: the call waits for
    // it as for any in-flight group (bounded, pvq_wait).
    const std::thread::id me = std::this_thread::get_id();
    std::chrono::steady_clock::time_point held_since{};
    uint64_t held_id = ~0ull;  // the head region the grace is running for
    auto stuck = [&]() -> const char* {
        if (P->regions.empty()) return nullptr;
        const PvqRegion& r = P->regions.front();
        if (!r.reserved || r.released) return nullptr;
        const char* own = "this thread's own reserved buffer, not committed or not released";
        if (!r.committed) return r.owner == me ? own : nullptr;
        if (!r.collected) return nullptr;
        if (r.owner == me) return own;
        const auto now = std::chrono::steady_clock::now();
        if (held_id != P->reg_base) {  // a new head region: its own grace
            held_id = P->reg_base;
            held_since = now;
        }
        return now - held_since >= kHeldResultWait
                   ? "a verified buffer whose result is not yet polled and released (poll() and release() free it)"
                   : nullptr;
    };
    if (int rc = pvq_wait(P, [&] { return pos() + need - P->byte_head <= P->nbytes; }, "data ring full", stuck))
        return rc;
    const uint64_t at = pos();
    P->regions.push_back(PvqRegion{at, at + need, reserved, false, false, false, me});
    P->byte_tail = at + need;
    *id = P->reg_base + P->regions.size() - 1;
    return SHA1CHUNK_OK;
}

// Give region `id` (filled, `len` bytes) the next slot, with its expected
// digest and tag, and publish when the group is full or the device idle.
int pvq_enqueue(Pvq* P, uint64_t id, uint32_t len, const uint8_t expected[20], uint64_t tag) {
    int rc;
    // A group never wraps the slot ring: an open group that ends where the
    // ring wraps is closed first.  pvq_wait sleeps without the queue's lock,
    // so another thread may fill the ring's last slot meanwhile and leave its
    // group open there: check again after every wait, under the
    // lock, until the next slot does not continue a group across the wrap.
    for (;;) {
        if (P->open_count && P->slot_tail % P->nslots == 0 && (rc = pvq_publish(P))) return rc;
        if ((rc = pvq_wait(P, [&] { return P->slot_tail + 1 - P->slot_head <= P->nslots; }, "slot ring full")))
            return rc;
        if (!(P->open_count && P->slot_tail % P->nslots == 0)) break;
    }
    PvqRegion& r = P->regions[id - P->reg_base];
    const uint64_t sl = P->slot_tail % P->nslots;
    P->off[sl] = r.start % P->nbytes;
    P->len[sl] = len;
    memcpy(P->exp + 20 * sl, expected, 20);
    P->tags[sl] = tag;
    P->slot_reg[sl] = id;
    r.committed = true;
    if (P->open_count == 0) P->open_slot0 = P->slot_tail;
    ++P->open_count;
    ++P->slot_tail;
    ++P->pending;
    if ((rc = pvq_reap(P))) return rc;
    if (P->open_count >= P->group_max || P->inflight < static_cast<size_t>(P->cus)) return pvq_publish(P);
    return SHA1CHUNK_OK;
}

// The copy runs without the queue's lock (the region is this call's until
// it is enqueued; nothing frees an uncollected region), on the helper
// threads when no other submit is using them, else on the calling thread:
// receive threads then copy side by side instead of one after another.
int pvq_submit(Pvq* P, const void* chunk, uint32_t len, const uint8_t expected[20], uint64_t tag) {
    uint64_t id;
    if (int rc = pvq_alloc(P, len, false, &id)) return rc;
    if (len) {
        uint8_t* dst = P->data + P->regions[id - P->reg_base].start % P->nbytes;
        const int64_t c0 = mono_ns();
        if (P->mu) P->mu->unlock();
        {
            // (streaming stores into the ring measured no faster: 28.3-29.2
            // against 27.5-28.9 GiB/s, profiles/vq_copy_r05.log)
            std::unique_lock<std::mutex> cl(P->copy_mu, std::try_to_lock);
            if (cl.owns_lock())
                pool_copy(*P->copier, dst, static_cast<const uint8_t*>(chunk), len);
            else
                memcpy(dst, chunk, len);
        }
        P->copy_ns.fetch_add(static_cast<uint64_t>(mono_ns() - c0), std::memory_order_relaxed);
        if (P->mu) P->mu->lock();
    }
    return pvq_enqueue(P, id, len, expected, tag);
}

void* pvq_reserve(Pvq* P, uint32_t len) {
    uint64_t id;
    if (pvq_alloc(P, len, true, &id)) return nullptr;
    const uint64_t at = P->regions[id - P->reg_base].start % P->nbytes;
    P->held[at] = id;
    return P->data + at;
}

// The reserved region `buf` points at (its id), or fails.
int pvq_held(Pvq* P, const void* buf, uint64_t* id) {
    const uint8_t* b = static_cast<const uint8_t*>(buf);
    if (b < P->data || b >= P->data + P->nbytes)
        return fail(SHA1CHUNK_EINVAL, "vq: %p is not a buffer of this queue", buf);
    auto it = P->held.find(static_cast<uint64_t>(b - P->data));
    if (it == P->held.end())
        return fail(SHA1CHUNK_EINVAL, "vq: %p is not a reserved buffer (released already?)", buf);
    *id = it->second;
    return SHA1CHUNK_OK;
}

int pvq_commit(Pvq* P, void* buf, uint32_t len, const uint8_t expected[20], uint64_t tag) {
    uint64_t id;
    if (int rc = pvq_held(P, buf, &id)) return rc;
    const PvqRegion& r = P->regions[id - P->reg_base];
    if (r.committed) return fail(SHA1CHUNK_EINVAL, "vq: buffer %p committed twice", buf);
    if (len > r.end - r.start)
        return fail(SHA1CHUNK_EINVAL, "vq: commit of %u bytes into a %llu-byte reservation", len,
                    static_cast<unsigned long long>(r.end - r.start));
    return pvq_enqueue(P, id, len, expected, tag);
}

int pvq_release(Pvq* P, void* buf) {
    uint64_t id;
    if (int rc = pvq_held(P, buf, &id)) return rc;
    P->held.erase(static_cast<uint64_t>(static_cast<uint8_t*>(buf) - P->data));
    P->regions[id - P->reg_base].released = true;
    pvq_free_regions(P);
    return SHA1CHUNK_OK;
}

long pvq_poll(Pvq* P, uint64_t* tags, uint8_t* mismatch, size_t max, int wait) {
    int rc;
    if (wait) {
        if ((rc = pvq_publish(P))) return rc;
        // every group published so far (other threads may keep publishing
        // while this one sleeps; their later groups are not waited for)
        const uint64_t target = P->next_g;
        if ((rc = pvq_wait(P, [&] { return P->groups.empty() || P->groups.front().g >= target; }, "poll(wait)")))
            return rc;
    } else {
        if ((rc = pvq_reap(P))) return rc;
        // an open group goes out once the device has room for it
        if (P->open_count && P->inflight < static_cast<size_t>(P->cus) && (rc = pvq_publish(P))) return rc;
        if (P->inflight && (rc = pvq_ensure_drain(P))) return rc;
    }
    size_t n = 0;
    while (n < max && !P->ready.empty()) {
        tags[n] = P->ready.front().first;
        mismatch[n] = P->ready.front().second;
        P->ready.pop_front();
        ++n;
    }
    P->pending -= n;
    return static_cast<long>(n);
}


size_t vq_cap(size_t batch) {
    const char* e = getenv("SHA1CHUNK_VQ_GROW");  // 0: launch at exactly `batch`
    if ((e && atoi(e) == 0) || batch >= 512) return batch;
    return std::max(batch, std::min(4 * batch, 512 / batch * batch));  // a multiple of batch
}

// Batch mode has no ring to reserve in: a reservation is a host buffer of
// the queue's, committed by copying (submit) and freed on release.
int vq_batch_submit(s1be_vq* q, const void* chunk, uint32_t len, const uint8_t expected[20], uint64_t tag) {
    if (len > q->maxlen) return fail(SHA1CHUNK_EINVAL, "vq: chunk of %u bytes > max %u", len, q->maxlen);
    VqSet* S = &q->set[q->fill];
    while (S->inflight) {  // the fill set is still on the device: drain in order
        int rc = vq_collect_oldest(q);
        if (rc) return rc;
    }
    if (S->count >= q->cap) {  // only after a failed launch
        int rc = vq_maybe_launch(q);
        if (rc) return rc;
        S = &q->set[q->fill];
        while (S->inflight) {
            if ((rc = vq_collect_oldest(q))) return rc;
        }
    }
    uint8_t* h = static_cast<uint8_t*>(S->h.p);
    const size_t i = S->count;
    vq_off(q, h)[i] = q->meta + i * q->stride;
    vq_len(q, h)[i] = len;
    memcpy(vq_exp(q, h) + 20 * i, expected, 20);
    if (len) pool_copy(*q->copier, h + q->meta + i * q->stride, static_cast<const uint8_t*>(chunk), len);
    S->tags.push_back(tag);
    ++S->count;
    ++q->pending;
    return vq_maybe_launch(q);
}

int vq_batch_flush(s1be_vq* q) {
    if (q->set[q->fill].count == 0 || q->set[q->fill].inflight) return SHA1CHUNK_OK;
    int rc = vq_launch(q, q->fill);
    if (rc) return rc;
    q->fill = (q->fill + 1) % kVqSets;
    return SHA1CHUNK_OK;
}

long vq_batch_poll(s1be_vq* q, uint64_t* tags, uint8_t* mismatch, size_t max, int wait) {
    int rc;
    if (wait) {
        if ((rc = vq_batch_flush(q))) return rc;
        while (!q->flight.empty())
            if ((rc = vq_collect_oldest(q))) return rc;
    } else {
        if ((rc = vq_reap(q))) return rc;
        if ((rc = vq_maybe_launch(q))) return rc;  // a grown batch waiting for the device
    }
    size_t n = 0;
    while (n < max && !q->ready.empty()) {
        tags[n] = q->ready.front().first;
        mismatch[n] = q->ready.front().second;
        q->ready.pop_front();
        ++n;
    }
    q->pending -= n;
    return static_cast<long>(n);
}

}  // namespace

// The backend's queue entry points take and return the queue as void*
// (the front end's handle type); every call holds the queue's lock, so any
// thread may reserve, fill, commit, release and poll on a shared queue.
extern "C" {

void s1be_vq_destroy(void* qv);

void* s1be_vq_create(size_t batch, uint32_t max_chunk_len) {
    if (batch == 0 || batch > (1u << 20) || max_chunk_len == 0) {
        fail(SHA1CHUNK_EINVAL, "vq: batch 1..2^20 and max_chunk_len > 0 required");
        return nullptr;
    }
    Device* D;
    if (get_device(&D)) return nullptr;
    auto* q = new s1be_vq();
    q->dev = D->id;
    q->stats = env_u64("SHA1CHUNK_VQ_STATS", 0) != 0;
    // the persistent drain unless SHA1CHUNK_VQ_MODE=batch (launch per batch)
    // or the device's drain CU budget is spent (then batch launches too)
    const char* mode = getenv("SHA1CHUNK_VQ_MODE");
    const int cus = mode && !strcmp(mode, "batch") ? 0 : drain_cus_take(D);
    if (cus > 0) {
        q->pv = pvq_create(D, batch, max_chunk_len, cus);
        if (q->pv) q->pv->mu = &q->mu;
        if (!q->pv) {
            delete q;
            return nullptr;
        }
        return q;
    }
    q->cus = D->cus;
    q->batch = batch;
    q->cap = vq_cap(batch);
    q->maxlen = max_chunk_len;
    q->stride = round_up(max_chunk_len, kAlign);
    q->meta = round_up(q->cap * (8 + 4 + 20), kAlign);
    q->copier = new PartPool(vq_copy_helpers(), near_cpus(D->id));
    const size_t hbytes = q->meta + q->cap * q->stride;
    for (auto& S : q->set) {
        if (S.h.ensure(hbytes) || S.d.ensure(hbytes + q->cap * 21) || S.res.ensure(q->cap) ||
            vq_stream_create(&S.stream) != 0 ||
            hipEventCreateWithFlags(&S.done, hipEventDisableTiming) != hipSuccess) {
            if (t_err.empty()) fail(SHA1CHUNK_ENOMEM, "vq: allocation failed");
            s1be_vq_destroy(q);
            return nullptr;
        }
        S.tags.reserve(q->cap);
    }
    return q;
}

enum { kOpSubmit, kOpReserve, kOpCommit, kOpRelease, kOpPoll, kOpOther };
struct VqLock {
    s1be_vq* q;
    int op;
    int64_t t1 = 0;
    VqLock(s1be_vq* q_, int op_) : q(q_), op(op_) {
        if (!q->stats) {
            q->mu.lock();
            return;
        }
        const int64_t t0 = mono_ns();
        q->mu.lock();
        t1 = mono_ns();
        ++q->st_calls[op];
        q->st_wait_ns[op] += static_cast<uint64_t>(t1 - t0);
    }
    ~VqLock() {
        if (q->stats) q->st_hold_ns[op] += static_cast<uint64_t>(mono_ns() - t1);
        q->mu.unlock();
    }
};

void vq_print_stats(const s1be_vq* q) {
    static const char* names[6] = {"submit", "reserve", "commit", "release", "poll", "other"};
    fprintf(stderr, "{\"vq_stats\": {");
    for (int i = 0; i < 6; ++i)
        fprintf(stderr, "\"%s\": [%llu, %.3f, %.3f], ", names[i], (unsigned long long)q->st_calls[i],
                q->st_wait_ns[i] * 1e-6, q->st_hold_ns[i] * 1e-6);
    const Pvq* P = q->pv;
    if (P)
        fprintf(stderr, "\"publish\": %llu, \"published\": %llu, \"copies\": %llu, \"launch\": %llu, "
                "\"scans\": %llu, \"sleeps\": %llu, \"sleep_ms\": %.3f, \"submit_copy_ms\": %.3f, ",
                (unsigned long long)P->n_publish, (unsigned long long)P->n_published,
                (unsigned long long)P->n_copies, (unsigned long long)P->n_launch,
                (unsigned long long)P->n_scans, (unsigned long long)P->n_sleeps, P->sleep_ns * 1e-6,
                P->copy_ns.load() * 1e-6);
    fprintf(stderr, "\"units\": \"[calls, ms waiting for the lock, ms holding it]\"}}\n");
}

int s1be_vq_submit(void* qv, const void* chunk, uint32_t len, const uint8_t expected[20], uint64_t tag) {
    auto* q = static_cast<s1be_vq*>(qv);
    if (!q || (len && !chunk) || !expected) return fail(SHA1CHUNK_EINVAL, "vq: null argument");
    VqLock lk(q, kOpSubmit);
    if (q->pv) {
        if (len > q->pv->maxlen)
            return fail(SHA1CHUNK_EINVAL, "vq: chunk of %u bytes > max %u", len, q->pv->maxlen);
        return pvq_submit(q->pv, chunk, len, expected, tag);
    }
    return vq_batch_submit(q, chunk, len, expected, tag);
}

void* s1be_vq_reserve(void* qv, uint32_t len) {
    auto* q = static_cast<s1be_vq*>(qv);
    if (!q) {
        fail(SHA1CHUNK_EINVAL, "vq: null queue");
        return nullptr;
    }
    VqLock lk(q, kOpReserve);
    const uint32_t maxlen = q->pv ? q->pv->maxlen : q->maxlen;
    if (len > maxlen) {
        fail(SHA1CHUNK_EINVAL, "vq: reservation of %u bytes > max %u", len, maxlen);
        return nullptr;
    }
    if (q->pv) return pvq_reserve(q->pv, len);
    auto buf = std::unique_ptr<uint8_t[]>(new (std::nothrow) uint8_t[std::max<uint32_t>(len, 1)]);
    if (!buf) {
        fail(SHA1CHUNK_ENOMEM, "vq: reservation of %u bytes", len);
        return nullptr;
    }
    void* p = buf.get();
    q->reserved.emplace(p, std::make_pair(len, std::move(buf)));
    return p;
}

int s1be_vq_commit(void* qv, void* buf, uint32_t len, const uint8_t expected[20], uint64_t tag) {
    auto* q = static_cast<s1be_vq*>(qv);
    if (!q || !buf || !expected) return fail(SHA1CHUNK_EINVAL, "vq: null argument");
    VqLock lk(q, kOpCommit);
    if (q->pv) return pvq_commit(q->pv, buf, len, expected, tag);
    auto it = q->reserved.find(buf);
    if (it == q->reserved.end()) return fail(SHA1CHUNK_EINVAL, "vq: %p is not a reserved buffer", buf);
    if (len > it->second.first)
        return fail(SHA1CHUNK_EINVAL, "vq: commit of %u bytes into a %u-byte reservation", len, it->second.first);
    return vq_batch_submit(q, buf, len, expected, tag);
}

int s1be_vq_release(void* qv, void* buf) {
    auto* q = static_cast<s1be_vq*>(qv);
    if (!q || !buf) return fail(SHA1CHUNK_EINVAL, "vq: null argument");
    VqLock lk(q, kOpRelease);
    if (q->pv) return pvq_release(q->pv, buf);
    if (!q->reserved.erase(buf)) return fail(SHA1CHUNK_EINVAL, "vq: %p is not a reserved buffer", buf);
    return SHA1CHUNK_OK;
}

int s1be_vq_flush(void* qv) {
    auto* q = static_cast<s1be_vq*>(qv);
    if (!q) return fail(SHA1CHUNK_EINVAL, "vq: null queue");
    VqLock lk(q, kOpOther);
    return q->pv ? pvq_publish(q->pv) : vq_batch_flush(q);
}

long s1be_vq_poll(void* qv, uint64_t* tags, uint8_t* mismatch, size_t max, int wait) {
    auto* q = static_cast<s1be_vq*>(qv);
    if (!q || (max && (!tags || !mismatch))) return fail(SHA1CHUNK_EINVAL, "vq: null argument");
    VqLock lk(q, kOpPoll);
    return q->pv ? pvq_poll(q->pv, tags, mismatch, max, wait) : vq_batch_poll(q, tags, mismatch, max, wait);
}

size_t s1be_vq_pending(const void* qv) {
    auto* q = static_cast<s1be_vq*>(const_cast<void*>(qv));
    if (!q) return 0;
    VqLock lk(q, kOpOther);
    return q->pv ? q->pv->pending : q->pending;
}

void s1be_vq_destroy(void* qv) {
    auto* q = static_cast<s1be_vq*>(qv);
    if (!q) return;
    if (q->stats) vq_print_stats(q);
    if (q->pv) {
        pvq_destroy(q->pv);
        delete q;
        return;
    }
    (void)hipSetDevice(q->dev);
    for (auto& S : q->set) {
        if (S.stream) (void)hipStreamSynchronize(S.stream);
        if (S.done) (void)hipEventDestroy(S.done);
        if (S.stream) (void)hipStreamDestroy(S.stream);
        if (S.h.p) (void)hipHostFree(S.h.p);
        if (S.res.p) (void)hipHostFree(S.res.p);
        if (S.d.p) (void)hipFree(S.d.p);
    }
    delete q->copier;
    delete q;
}

}  // extern "C"
