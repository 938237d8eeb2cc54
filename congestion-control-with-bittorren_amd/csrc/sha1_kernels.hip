// sha1_kernels.hip -- gfx950 kernels of the SHA-1 chunk engine.
//
// The reference hashes one chunk at a time on one CPU core (make_chunks loop
// chunk.c:22-24 -> shahash chunk.c:35-51 -> SHA1Update sha.c:453-527 ->
// SHA1Guts sha.c:176-451).  Here every lane owns one chunk and a wave hashes
// 64 chunks in lockstep.  SHA-1 is serial inside a message (Merkle-Damgard:
// sha.c:518 carries sc->hash from block to block), so the only parallelism
// is across chunks; the kernels differ in how a lane gets its 64-byte blocks
// and who computes the message schedule:
//
//   sha1_lane_kernel   each lane loads its own blocks from HBM (any byte
//                      alignment, any length); also the streaming kernel
//                      behind SHA1Update/SHA1Final (init state + no-final).
//   sha1_fused_kernel  one wave per 64 chunks, schedule + rounds in VGPRs
//                      (~627 instructions per block), two 128-byte stages of
//                      each chunk prefetched per lane.  The high-occupancy
//                      kernel: > 2 groups of 64 chunks per CU.
//   sha1_split_kernel  workgroup = consumer wave + producer wave(s) on the
//                      same 64 chunks.  Producers stream and byte-swap the
//                      blocks and expand the 80-word schedule (+K) into an
//                      LDS ring; the consumer runs only the 80 rounds (~428
//                      instructions per block instead of ~627), which is the
//                      bound when there are too few chunks to fill the
//                      SIMDs (BASELINE config 2: 4096 chunks = 64 waves).
//                      One wave's 20 ds_write_b128 per block cost ~28 cycles
//                      each on top of its VALU (tools/gen_producer_probe.py),
//                      so one producer is as slow as the consumer: each
//                      consumer gets two producers, laid out so that it has a
//                      SIMD to itself (a workgroup's waves 0-3 land on four
//                      different SIMDs, wave w + 4 on wave w's:
//                      tools/wave_placement_probe.hip).
//   sha1_mixed_kernel  ragged batches sorted longest-first with more groups
//                      than CUs: one launch whose workgroups run the split
//                      body (longest groups) or the fused body, per a
//                      device-side plan (plan_mixed_kernel) -- see `mixed`.
//
// Measured on MI355X (tools/issue_probe.hip, tools/gen_consumer_probe.py,
// DESIGN.md section 5): one wave issues at most one instruction per 4.0
// cycles; its round stream reaches that with x = e + (W+K) as a VOP2 add and
// runs at ~5 cycles per VALU with a VOP3 add3 of K; at several waves per SIMD
// v_alignbit/v_add3/v_perm cost ~1.9 ns of SIMD time per wave-instruction vs
// ~1.1 ns for v_add/v_xor/v_bitop3.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "sha1_split.hpp"

// The mixed planner's measured constants (us per block of a group of 64
// chunks, see `Makespan model` below).  The scattered fused shapes (S) were
// re-measured in round 5 after their loads moved to LDS-DMA four blocks
// ahead (1.408 -> 1.334, 2.661 -> 2.628; profiles/mixed_const_r05.jsonl).
// The same run measured the split and together-fused shapes at 0.742,
// 1.268 and 2.489 (within 1.2 % of these) and the 8-wave shape at 0.803,
// 7 % under its constant; kept, as the 8-wave mode is 12-14 % behind the
// best split-head plan at 131072 chunks either way.
#define PLAN_SPLIT4 0.743
#define PLAN_SPLIT8 0.860
#define PLAN_FUSED4T 1.254
#define PLAN_FUSED4S 1.334
#define PLAN_FUSED8T 2.502
#define PLAN_FUSED8S 2.628
// The fused constants are measured with every CU running the fused shape
// (tools/mixed_constants.sh).  In a mixed plan the fused workgroups share the
// chip with split ones and run faster: fitted over the 26 forced split-head
// plans of the config-5 law at 131072 and 262144 chunks in both layouts
// (profiles/mixed_verify_r04c.jsonl), the fused jobs take 0.955 of their
// all-fused time (simulated vs measured: rms 2.2 % instead of 4.5 %).
#define PLAN_FUSED_SHARE 0.955

// ---------------------------------------------------------------- lane ----
__global__ __launch_bounds__(256) void sha1_lane_kernel(BatchArgs A) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= A.n) return;
    const Entry en = fetch_entry(A, e);
    uint32_t h[5];
    load_init(A, en.id, h);
    lane_blocks(A, en, 0, h);
    emit(A, en.id, h);
}

// --------------------------------------------------------------- fused ----
// (body: fused_body in sha1_split.hpp)
__global__ __launch_bounds__(256) void sha1_fused_kernel(BatchArgs A) {
    fused_body(A, blockIdx.x * 256u + threadIdx.x);
}

// --------------------------------------------------------------- mixed ----
// Ragged batches with more groups of 64 than CUs, sorted longest-first
// (BASELINE config 5's shape beyond 16384 chunks).  A batch of mixed lengths
// ends with its longest chunks' serial chains, so the kernel that has the
// most throughput per CU (fused) is not the one to run them on: at several
// waves per SIMD a fused wave's chain crawls (2.4 us per block at 2 waves
// per SIMD against 0.74 us in the one-group split shape), and a batch of
// log-uniform 4 KiB .. 1 MiB chunks ran 2.5x longer fused than split
// (tools/mixed_bench.py, profiles/mixed_r02.json).  A device-side plan
// (plan_mixed_kernel, from the sorted lengths, no host round trip) splits
// the batch between the shapes; every workgroup of this kernel reserves the
// whole 160 KiB of LDS, so exactly one is resident per CU:
//   mode 0: workgroups 0 .. H-1 hash groups 0 .. H-1 (the longest) one per
//           CU in the one-group split shape (4-block units, two producers,
//           the consumer alone on its SIMD); workgroup H + j hashes groups
//           H + j*F .. H + j*F + F-1 fused, one group per wave (F = 4: one
//           wave per SIMD, chain 1.28 us per block; F = 8: two), each
//           wave loading lane-per-chunk if its chunks lie together and
//           with loads shared across the wave if not (fused_coop_body).
//   mode 1: workgroup w hashes groups 2w, 2w+1 in the 8-wave two-pair split
//           shape (AUTO's shape for C < groups <= 2C on a uniform batch).
// Blocks in dispatch order: the longest groups start first, and the
// hardware dispatcher hands the next workgroup to whichever CU frees up
// (longest-processing-time order).  The grid is one workgroup per group
// (the all-split plan); workgroups past a plan's count exit at once.
//
// Memory locality: with every lane streaming its own chunk, a load
// instruction translates 64 addresses, and when the resident chunks lie far
// apart (a sorted batch whose chunks arrived in random length order) the
// CU's translation cache (UTCL1) thrashes: 98 % misses instead of ~0 on the
// same requests, L2 unchanged (tools/tlb_probe.sh, profiles/tlb_r02.json).
// 65536 x 512 KiB with permuted offsets hashed in 29.2 ms lane-per-chunk
// against 10.4 in place.  Every shape here loads scattered chunks 8 or 16 per
// instruction (see `shared loads`): permuted, the fused tail takes 10.8 ms
// and the one-group split shape 24.3 as in place (profiles/mixed_r02.json,
// profiles/coop_split_ab_r02.json).  A fused wave whose chunks lie together
// still streams lane-per-chunk, which is faster, so the planner prices the
// fused jobs by layout (round 4: plan_layout_kernel, PLAN_FUSED*T/S).
constexpr int kMixedThreads = 512;

__global__ __launch_bounds__(kMixedThreads) void sha1_mixed_kernel(BatchArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
    const uint32_t mode = A.plan[0], H = A.plan[1], F = A.plan[2];
    const uint32_t wg = blockIdx.x;
    const uint32_t groups = (A.n + 63u) / 64u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (mode == 1) {
        if (2u * wg >= groups) return;
        split_body<2, 2, kSplit8V, 2>(A, lds, wg);
        return;
    }
    if (wg < H) {
        if (wave >= 4) return;  // the one-group shape is waves 0-3 (wave 2 empty)
        split_body<4, 1, kSplitV<4>, kSplitNProd<4>>(A, lds, wg);
        return;
    }
    const uint32_t g = H + (wg - H) * F + wave;
    if (wave >= F || g >= groups) return;
    fused_coop_body(A, g * 64u + (threadIdx.x & 63u), lds + wave * kCoopWaveBytes);
}

// Persistent-dispatch variant of the mixed kernel (BASELINE config 5 names
// "persistent-kernel dispatch"): one 512-thread
// workgroup per CU (all 160 KiB of LDS each, so one resident per CU) pulls
// the plan's jobs in order from a device counter (plan[3], zeroed by the
// planner on the same stream) until the list is empty.  The job list is the
// plan's: jobs 0 .. H-1 one split group each, then fused jobs of F groups (or
// mode 1: pairs in the 8-wave split shape).  Against the hardware dispatch
// of sha1_mixed_kernel (workgroup i goes to XCD i % 8 and waits for a CU of
// that XCD) any CU that frees takes the next job: one global greedy queue
// instead of eight.  Every wave stays in the loop, so the waves a split job
// does not use pass the same number of workgroup barriers as the job's
// waves (idle_barriers): units + 1 for a split job, plus the two of the
// 8-wave shape's length exchange.
__device__ __forceinline__ uint32_t group_units(const BatchArgs& A, uint32_t group, uint32_t U) {
    const uint32_t e = group * 64u + (threadIdx.x & 63u);
    const bool valid = e < A.n;
    Entry en = fetch_entry(A, valid ? e : fallback_entry(A, group));
    const uint32_t T = valid ? total_blocks(en.len) : 0u;
    const uint32_t Tmax = __builtin_amdgcn_readfirstlane(wave_max(T));
    return (Tmax + 2u * U - 1u) / (2u * U) * 2u;
}

__device__ __forceinline__ void idle_barriers(uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) split_barrier();
}

__global__ __launch_bounds__(kMixedThreads) void sha1_mixed_persistent_kernel(BatchArgs A, uint32_t* queue) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
    const uint32_t mode = A.plan[0], H = A.plan[1], F = A.plan[2];
    const uint32_t groups = (A.n + 63u) / 64u;
    const uint32_t jobs = mode == 1 ? (groups + 1u) / 2u : H + (groups - H + F - 1u) / F;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t* slot = reinterpret_cast<uint32_t*>(lds);  // free between jobs
    for (;;) {
        if (threadIdx.x == 0) slot[0] = atomicAdd(queue, 1u);
        __syncthreads();
        const uint32_t job = __builtin_amdgcn_readfirstlane(slot[0]);
        __syncthreads();  // every wave has the job before the LDS is reused
        if (job >= jobs) break;
        if (mode == 1) {
            if (wave == 4 || wave == 6) {  // the 8-wave shape's empty waves
                const uint32_t u = max(group_units(A, 2u * job, 2), 2u * job + 1u < groups
                                                                        ? group_units(A, 2u * job + 1u, 2)
                                                                        : 0u);
                idle_barriers(2u + u + 1u);
            } else {
                split_body<2, 2, kSplit8V, 2>(A, lds, job);
            }
        } else if (job < H) {
            if (wave == 0 || wave == 1 || wave == 3)  // the one-group shape (wave 2 empty)
                split_body<4, 1, kSplitV<4>, kSplitNProd<4>>(A, lds, job);
            else
                idle_barriers(group_units(A, job, 4) + 1u);
        } else {
            const uint32_t g = H + (job - H) * F + wave;
            if (wave < F && g < groups) fused_coop_body(A, g * 64u + (threadIdx.x & 63u), lds + wave * kCoopWaveBytes);
        }
    }
}

// ---------------------------------------------------- verify-queue drain ----
// The persistent drain of the received-chunk verify queue (SURVEY 8f rank 2;
// packet_handler.c:469-472 -> job.c:217-228 verify_hash).  One 512-thread
// workgroup per CU loops: lane 0 claims the next published group of <= 64
// chunks (a compare-and-swap on a device counter, below the host's `pub`),
// the workgroup hashes it in the one-group split shape straight out of the
// host ring (coherent pinned memory: every read goes over PCIe, nothing is
// cached), wave 0 compares the 64 digests with the expected ones and
// writes a 0/1 per chunk and the group's completion word to host memory.
// Without work a workgroup sleeps (exponential backoff up to ~50 us) and
// exits once no group has been claimed for `idle_ticks` of 100 MHz time, or
// at once when the host sets `stop`.  Exit handshake (no lost group): the
// workgroup clears its alive word, fences, and re-reads `pub`; the host
// stores `pub`, fences, and reads the alive words.  At least one of them
// sees the other: either the workgroup claims the new group or the host
// launches a new drain.
constexpr uint32_t kVqIdle = 0xffffffffu, kVqExit = 0xfffffffeu;

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// alive flags are bytes: the host reads 16 workgroups' flags per uncached load
__device__ __forceinline__ void st_sys(uint8_t* p, uint8_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Lane 0 only: a claimed group index, kVqIdle or kVqExit.  Idleness is the
// queue's, not the workgroup's: `last` is when the claim counter last moved
// (any workgroup's claim), so under load no workgroup leaves, and after a
// quiet spell the drain's workgroups leave together.
__device__ uint32_t vq_next(const VqDrainArgs& Q, uint64_t& last, uint32_t& seen, uint64_t born) {
    // Bounded lifetime: a drain that never went idle would hold its hardware
    // queue for good, and HIP serves every stream mapped onto that queue (a
    // process has GPU_MAX_HW_QUEUES = 4 of them) in order behind it -- another
    // queue's setup or drain, a hash batch.  Past life_ticks the workgroup
    // leaves between groups, work pending or not; the host relaunches the
    // drain on its next call (pvq_ensure_drain counts the live workgroups).
    if (__builtin_amdgcn_s_memrealtime() - born > Q.life_ticks) {
        st_sys(Q.alive + blockIdx.x, uint8_t{0});
        return kVqExit;
    }
    for (int round = 0; round < 2; ++round) {
        uint32_t p = ld_sys(Q.pub);
        uint32_t c = __hip_atomic_load(Q.claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c != seen) {
            seen = c;
            last = __builtin_amdgcn_s_memrealtime();
        }
        while (c < p) {
            if (__hip_atomic_compare_exchange_strong(Q.claim, &c, c + 1u, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                seen = c + 1u;
                last = __builtin_amdgcn_s_memrealtime();
                return c;
            }
        }
        if (ld_sys(Q.stop)) return kVqExit;
        if (round == 1 || __builtin_amdgcn_s_memrealtime() - last <= Q.idle_ticks) return kVqIdle;
        // idle too long: leave, unless a group was published meanwhile
        st_sys(Q.alive + blockIdx.x, uint8_t{0});
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
        if (__hip_atomic_load(Q.claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ld_sys(Q.pub)) return kVqExit;
        st_sys(Q.alive + blockIdx.x, uint8_t{1});
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
    }
    return kVqIdle;
}

__global__ __launch_bounds__(kMixedThreads) void sha1_vq_drain_kernel(VqDrainArgs Q) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[160 * 1024];
    uint32_t* slot = reinterpret_cast<uint32_t*>(lds);  // free between jobs
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    const uint64_t born = last;
    uint32_t seen = 0xffffffffu;
    uint32_t backoff = 1;
    for (;;) {
        if (threadIdx.x == 0) slot[0] = vq_next(Q, last, seen, born);
        __syncthreads();
        const uint32_t g = __builtin_amdgcn_readfirstlane(slot[0]);
        __syncthreads();  // every wave has the command before the LDS is reused
        if (g == kVqExit) break;
        if (g == kVqIdle) {
            for (uint32_t i = 0; i < backoff; ++i) __builtin_amdgcn_s_sleep(127);  // ~3.4 us each
            backoff = min(backoff * 2u, 16u);
            continue;
        }
        backoff = 1;
        const uint32_t gi = g % Q.grp_ring;
        const uint32_t first = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(Q.grp + 2 * gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        const uint32_t count = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(Q.grp + 2 * gi + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        BatchArgs A{};
        A.base = Q.data;
        A.off = Q.off + first;
        A.len = Q.len + first;
        A.n = count;
        A.dig = Q.dig + 20ull * first;
        if (wave == 0 || wave == 1 || wave == 3)  // the one-group split shape (wave 2 empty)
            split_body<4, 1, kSplitV<4>, kSplitNProd<4>>(A, lds, 0);
        else
            idle_barriers(group_units(A, 0, 4) + 1u);
        __syncthreads();
        if (wave == 0) {  // the consumer wave re-reads the digests it wrote
            uint32_t diff = 0;
            if (lane < count) {
                const uint32_t* d = reinterpret_cast<const uint32_t*>(A.dig + 20u * lane);
                const uint32_t* x = reinterpret_cast<const uint32_t*>(Q.exp + 20ull * (first + lane));
#pragma unroll
                for (int i = 0; i < 5; ++i)
                    diff |= d[i] ^ __hip_atomic_load(x + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                Q.res[first + lane] = diff ? 1 : 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (lane == 0) {
                st_sys(Q.done + gi, g + 1u);
                st_sys(Q.last_done, g + 1u);  // the host scans only after this word moved
            }
        }
    }
}

// Makespan model of a sorted ragged batch, microseconds per 64-byte block of
// a group of 64 chunks, measured on MI355X with one job of the shape on
// every CU (the clock the chip holds under that load; tools/mixed_constants.sh,
// profiles/mixed_const_r04.jsonl):
//   chain: time of one group's block when it runs in that shape
//   cu:    CU-time per group-block (the CU's throughput in that shape)
// The fused shapes stream a group lane-per-chunk when its chunks lie
// together and share each load across the wave when they lie scattered
// (fused_coop_body), which costs a few per cent more: two constants each.
constexpr double kChainSplit4 = PLAN_SPLIT4, kCuSplit4 = PLAN_SPLIT4;
constexpr double kChainFused4T = PLAN_FUSED4T * PLAN_FUSED_SHARE, kChainFused4S = PLAN_FUSED4S * PLAN_FUSED_SHARE;
constexpr double kChainFused8T = PLAN_FUSED8T * PLAN_FUSED_SHARE, kChainFused8S = PLAN_FUSED8S * PLAN_FUSED_SHARE;
constexpr double kChainSplit8 = PLAN_SPLIT8, kCuSplit8 = PLAN_SPLIT8 / 2;

__device__ __forceinline__ double fused_chain(uint32_t F, bool together) {
    return F == 4 ? (together ? kChainFused4T : kChainFused4S) : (together ? kChainFused8T : kChainFused8S);
}

__device__ __forceinline__ uint32_t group_blocks(const uint32_t* sorted_len, uint32_t g) {
    return total_blocks(sorted_len[64ull * g]);  // a group's first lane is its longest
}

// The workgroups of a plan are jobs that the dispatcher starts in index
// order on whichever CU frees first.  Job i of mode 0 (H split groups, then
// fused workgroups of F groups) and of mode 1 (pairs): its duration.
// (blocks: the planner's LDS copy of group_blocks for groups < kSimMaxG)
constexpr uint32_t kSimMaxG = 16384;  // groups whose blocks the planner keeps in LDS

__device__ __forceinline__ uint32_t plan_blocks(const uint32_t* sorted_len, const uint32_t* blocks, uint32_t g) {
    return g < kSimMaxG ? blocks[g] & 0x0fffffffu : group_blocks(sorted_len, g);  // bits 28-31: the run (sim_xcd)
}

// Whether group g's chunks lie together: the rule fused_coop_body applies
// per wave (address span <= 2 x their bytes + 2 MiB).  A wave per group,
// a lane per chunk, all groups in parallel over the chip (the planner's
// single workgroup walking 64 dependent entries per group cost it up to
// ~0.5 ms at 262144 chunks).  Workgroup w summarises groups 32w .. 32w+31:
// bits[w] (bit i: group 32w+i lies together) and tb[w] (the blocks of those
// groups, the planner's together share).
constexpr int kLayoutThreads = 1024;  // two groups per wave (eight at 256 threads: 16.5 us at 2048 groups)
constexpr uint32_t kLayoutGroupsPerWave = 32 / (kLayoutThreads / 64);

// The workgroups holding positions below kBigExact (2048 per workgroup)
// first re-rank the chunks whose sort keys clamped (BigFix, sha1_kernels.h):
// m = the tiles' clamped counts summed; for 0 < m <= kBigExact every such
// workgroup sorts the m (exact block count, caller position) pairs in LDS
// (bitonic) and rewrites the order, and the group-head sorted lengths, of its
// own positions below m, then summarises its groups from the re-ranked
// entries.  No other workgroup, and no batch without chunks of 4 MiB and
// more, does anything extra.
constexpr uint32_t kLayoutPositions = 32u * 64u;  // positions per layout workgroup

__global__ __launch_bounds__(kLayoutThreads) void plan_layout_kernel(BatchArgs A, const uint32_t* sorted_len,
                                                                     BigFix B, uint64_t* tb, uint32_t* bits,
                                                                     uint32_t* gblk) {
    const uint32_t lane = threadIdx.x % 64u, wave = threadIdx.x / 64u;
    const uint32_t G = (A.n + 63u) / 64u;
    __shared__ uint32_t tog[32], blk[32];
    __shared__ uint64_t bk[kBigExact];  // (0x7ffffff - blocks) << 32 | caller position, sorted
    __shared__ uint32_t bm;
    // The wave's groups' entries first, all in flight together: each is two
    // dependent global reads (order, then offset and length), and taking
    // the groups one at a time cost ~17 us at 2048 groups.
    Entry en[kLayoutGroupsPerWave];
#pragma unroll
    for (uint32_t k = 0; k < kLayoutGroupsPerWave; ++k) {
        const uint32_t e = 64u * (32u * blockIdx.x + wave * kLayoutGroupsPerWave + k) + lane;
        if (e < A.n) {
            en[k] = fetch_entry(A, e);
        } else {
            en[k].p = nullptr;
            en[k].len = 0;
        }
    }
    // position 0 holds the largest key: below the clamp, no chunk clamped and
    // nothing more to read (one load, in flight with the entries')
    if (B.cnt && blockIdx.x * kLayoutPositions < kBigExact && total_blocks(sorted_len[0]) >= 65535u) {
        const uint32_t t = threadIdx.x;
        if (t < 64u) {
            uint32_t v = 0;
            for (uint32_t i = t; i < B.tiles; i += 64u) v += B.cnt[i];
#pragma unroll
            for (uint32_t o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
            if (t == 0) bm = v;
        }
        __syncthreads();
        const uint32_t m = bm;
        if (m > 0 && m <= kBigExact && blockIdx.x * kLayoutPositions < m) {
            uint32_t P = 64;
            while (P < m) P <<= 1;
            for (uint32_t j = t; j < P; j += kLayoutThreads)
                bk[j] = j < m ? (uint64_t)(0x07ffffffu - total_blocks(B.len[j])) << 32 | j : ~0ull;
            __syncthreads();
            // ascending bitonic sort: longest first, then caller order
            for (uint32_t k2 = 2; k2 <= P; k2 <<= 1)
                for (uint32_t j2 = k2 >> 1; j2 > 0; j2 >>= 1) {
                    for (uint32_t i = t; i < P; i += kLayoutThreads) {
                        const uint32_t ixj = i ^ j2;
                        if (ixj > i) {
                            const uint64_t a = bk[i], b = bk[ixj];
                            if ((a > b) == ((i & k2) == 0u)) {
                                bk[i] = b;
                                bk[ixj] = a;
                            }
                        }
                    }
                    __syncthreads();
                }
            const uint32_t r0 = blockIdx.x * kLayoutPositions, r1 = min(m, r0 + kLayoutPositions);
            for (uint32_t r = r0 + t; r < r1; r += kLayoutThreads) {
                const uint32_t j = static_cast<uint32_t>(bk[r]);
                B.order[r] = B.id[j];
                if ((r & 63u) == 0u) B.sorted_len[r] = B.len[j];
            }
#pragma unroll
            for (uint32_t k = 0; k < kLayoutGroupsPerWave; ++k) {
                const uint32_t e = 64u * (32u * blockIdx.x + wave * kLayoutGroupsPerWave + k) + lane;
                if (e < m) {
                    const uint32_t j = static_cast<uint32_t>(bk[e]);
                    const uint32_t id = B.id[j];
                    en[k].p = A.base + A.off[id];
                    en[k].len = B.len[j];
                }
            }
        }
    }
#pragma unroll
    for (uint32_t k = 0; k < kLayoutGroupsPerWave; ++k) {
        const uint32_t slot = wave * kLayoutGroupsPerWave + k;
        const uint32_t g = 32u * blockIdx.x + slot;
        if (g >= G) {  // wave-uniform
            if (lane == 0) tog[slot] = blk[slot] = 0u;
            continue;
        }
        const uint32_t e = 64u * g + lane;
        uint64_t lo = ~0ull, hi = 0, bytes = 0;
        if (e < A.n) {
            lo = reinterpret_cast<uint64_t>(en[k].p);
            hi = lo + en[k].len;
            bytes = en[k].len;
        }
#pragma unroll
        for (uint32_t m = 1; m < 64; m *= 2) {
            lo = min(lo, (uint64_t)__shfl_xor((unsigned long long)lo, m));
            hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, m));
            bytes += (uint64_t)__shfl_xor((unsigned long long)bytes, m);
        }
        if (lane == 0) {
            tog[slot] = hi - lo <= 2 * bytes + (2ull << 20) ? 1u : 0u;
            // the head's blocks from its entry (lane 0 holds position 64g: the
            // length sorted_len[64g] holds, or a re-ranked head's), written
            // for the planner as one coalesced array
            const uint32_t b = total_blocks(en[k].len);
            blk[slot] = b;
            gblk[g] = b;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t w = 0;
        uint64_t b = 0;
        for (uint32_t i = 0; i < 32; ++i) {
            w |= tog[i] << i;
            b += tog[i] ? blk[i] : 0u;
        }
        bits[blockIdx.x] = w;
        tb[blockIdx.x] = b;
    }
}

// The planner's layout knowledge: per group g < kSimMaxG (in LDS) how many
// of groups g .. g+7 in a row lie together (groups past the batch count as
// together, groups from kSimMaxG on as `rest`), and for the groups beyond,
// whether most blocks lie together.
struct PlanLayout {
    const uint8_t* run;
    bool rest;
    // a fused job of F <= 8 groups from g streams lane-per-chunk if all of them do
    __device__ bool job_together(uint32_t g, uint32_t F, uint32_t G) const {
        return g < kSimMaxG ? run[g] >= F : rest;
    }
};

// Branch-free (a wave's lanes price plans of both modes; the same values
// as the three-way branch it replaced, which ran each side in turn).
__device__ __forceinline__ double job_time(const uint32_t* sorted_len, const uint32_t* blocks, const PlanLayout& L,
                                           uint32_t G, uint32_t mode, uint32_t H, uint32_t F, uint32_t i) {
    const bool split = mode == 1 || i < H;
    const uint32_t g = mode == 1 ? 2u * i : (i < H ? i : H + (i - H) * F);
    const double fc = fused_chain(F, L.job_together(g, F, G));
    const double c = mode == 1 ? kChainSplit8 : (split ? kChainSplit4 : fc);
    return plan_blocks(sorted_len, blocks, g) * c;
}

// Estimated makespan of a plan: the largest of
//   W / C                         total CU-time over C CUs (work bound)
//   p_0, p_H                      the longest split job, the longest fused job
//   (k + 1) p_{kC}, k >= 1        jobs 0 .. kC on C CUs: some CU runs k + 1
//                                 of them back to back (rounds bound; exact
//                                 for equal lengths)
// where W = cu_split4 * P_H + cu_fusedF * (P_G - P_H) in mode 0 and
// cu_split8 * P_G in mode 1 (P_H: blocks of groups 0 .. H-1; cu_fusedF the
// together / scattered constants weighted by the batch's share `ft` of
// blocks in groups whose chunks lie together).
__device__ double makespan(const uint32_t* sorted_len, const uint32_t* blocks, const PlanLayout& L, double ft,
                           uint32_t G, uint32_t C, uint32_t mode, uint32_t H, uint32_t F, uint64_t PH, uint64_t PG) {
    double W;
    uint32_t J;
    if (mode == 1) {
        W = kCuSplit8 * (double)PG;
        J = (G + 1u) / 2u;
    } else {
        const double cu = (ft * fused_chain(F, true) + (1.0 - ft) * fused_chain(F, false)) / F;
        W = kCuSplit4 * (double)PH + cu * (double)(PG - PH);
        J = H + (G - H + F - 1u) / F;
    }
    double m = fmax(W / C, job_time(sorted_len, blocks, L, G, mode, H, F, 0));
    if (mode == 0 && H > 0 && H < G) m = fmax(m, job_time(sorted_len, blocks, L, G, mode, H, F, H));
    // the rounds bound four k at a time, their reads in flight together (a
    // k past the jobs prices job J - 1 and counts 0; the maximum is the same
    // in any order: every term is finite and >= 0)
    for (uint32_t k = 1; (uint64_t)k * C < J; k += 4u) {
        double v[4];
#pragma unroll
        for (uint32_t u = 0; u < 4u; ++u) {
            const uint64_t i = (uint64_t)(k + u) * C;
            const double t = job_time(sorted_len, blocks, L, G, mode, H, F, i < J ? (uint32_t)i : J - 1u);
            v[u] = i < J ? (k + u + 1) * t : 0.0;
        }
        m = fmax(m, fmax(fmax(v[0], v[1]), fmax(v[2], v[3])));
    }
    return m;
}

// The bounds above are lower bounds: with 160 KiB of LDS per workgroup a CU
// runs one job at a time, and a long fused job that a CU picks up late ends
// late (config-5 law at 131072 chunks: bounds 13.0 ms for H = 257, measured
// 17.4, while H = 160 measured 13.8).  So the planner then simulates the
// dispatch of a short list of candidate plans exactly and keeps the
// shortest: workgroup i goes to XCD i % 8 (round-robin), and each XCD starts
// its jobs in index order on whichever of its CUs frees first.  One lane
// per (candidate, XCD) keeps its CUs' free times sorted in 32 registers;
// fp32, restated bit for bit in tests/test_gpu_mixed.py.  Candidates whose
// bounds already exceed the simulated time of the bounds' best plan are not
// simulated.
constexpr uint32_t kSimXcds = 8, kSimCus = 32;      // CUs per XCD the lane tracks at most
constexpr float kChainSplit4f = (float)kChainSplit4, kChainSplit8f = (float)kChainSplit8;
constexpr float kChainFused4Tf = (float)kChainFused4T, kChainFused4Sf = (float)kChainFused4S,
                kChainFused8Tf = (float)kChainFused8T, kChainFused8Sf = (float)kChainFused8S;

__device__ __forceinline__ uint32_t plan_jobs(uint32_t G, uint32_t mode, uint32_t H, uint32_t F) {
    return mode == 1 ? (G + 1u) / 2u : H + (G - H + F - 1u) / F;
}

// v_med3_u32 (no builtin for the unsigned form); volatile, so the LDS
// reads sim_xcd issues ahead of an insert stay ahead of it.
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Job j's duration from its group's word (blocks, run in bits 28-31): the
// split constant while j < Hs, then the fused one by whether the job's F
// groups lie together; the fp32 product rounded before the insert's add.
__device__ __forceinline__ float sim_dur(uint32_t v, uint32_t j, uint32_t Hs, uint32_t F, float cs, float cT,
                                         float cS) {
#pragma clang fp contract(off)
    const uint32_t b = v & 0x0fffffffu, r = v >> 28;
    const float c = j < Hs ? cs : (r >= F ? cT : cS);
    return (float)b * c;
}

// A job of duration d on the CU that frees first: t ascending, the new t[i]
// is the job's end clamped to [t[i], t[i+1]].
__device__ __forceinline__ void sim_insert(uint32_t (&t)[kSimCus], float d) {
#pragma clang fp contract(off)
    const uint32_t nx = __float_as_uint(__uint_as_float(t[0]) + d);
#pragma unroll
    for (uint32_t i = 0; i + 1 < kSimCus; ++i) t[i] = umed3(t[i], nx, t[i + 1]);
    t[kSimCus - 1] = max(t[kSimCus - 1], nx);
}

// Jobs x, x + 8, .. of a plan on one XCD's `per` CUs: the time its last CU
// frees.  t holds the free times in ascending order (+inf past `per`); a
// job starts at t[0] and its end is inserted in order.  Simulated only for
// G <= kSimMaxG, so every job's group has its blocks and run in LDS.
//
// Job j runs group g_j: split jobs (j < Hs) g = m*j (m = 2 for the 8-wave
// mode's pairs), fused jobs g = Hs + (j - Hs)*F; its duration is the
// group's blocks times the shape's chain constant (fused: by whether the F
// groups from g lie together), the fp32 product rounded before the add
// (contract off; tests/test_gpu_mixed.py restates it bit for bit).
// Branch-free (the lanes of a wave simulate different candidates, and a
// per-mode branch with its own read and wait, round 4's form, cost ~3x
// this), one LDS word per job read ahead of the insert before it.
__device__ __forceinline__ float sim_xcd(const uint32_t* blocks, uint32_t G, uint32_t mode, uint32_t H, uint32_t F,
                                         uint32_t x, uint32_t per) {
#pragma clang fp contract(off)
    typedef const volatile __attribute__((address_space(3))) uint32_t lds_u32;
    // Free times as the bits of non-negative floats, which order as
    // unsigned integers (+inf above every finite time), so the insert is
    // v_med3_u32: ~205 shader cycles per job against ~300 for v_med3_f32 and
    // ~400 for v_min_u32 + v_max_u32 pairs (one wave, tools/insert_probe.hip,
    // profiles/insert_probe_r05.log).
    uint32_t t[kSimCus];
#pragma unroll
    for (uint32_t i = 0; i < kSimCus; ++i) t[i] = i < per ? 0u : 0x7f800000u;
    const uint32_t J = plan_jobs(G, mode, H, F);
    const uint32_t Hs = mode == 1 ? J : H, m = mode == 1 ? 2u : 1u;
    const float cs = mode == 1 ? kChainSplit8f : kChainSplit4f;
    const float cT = F == 8 ? kChainFused8Tf : kChainFused4Tf, cS = F == 8 ? kChainFused8Sf : kChainFused4Sf;
    // g = m*j while j < Hs, Hs + (j - Hs)*F after (m, F powers of two; mode 1
    // never leaves the first phase): shifts, min and max, no branch (the
    // ternary compiled to two branches and a 64-bit multiply per job, which
    // doubled the insert's ~265 cycles, profiles/fixed_cost_planner_r05.log)
    const uint32_t msh = m == 2u ? 1u : 0u, fsh = F == 8u ? 3u : 2u;
    auto group = [&](uint32_t j) { return (min(j, Hs) << msh) + ((max(j, Hs) - Hs) << fsh); };
    // each group's blocks with its run in bits 28-31 (one read per job), two
    // jobs ahead (measured the same as one: 43.0 against 43.2 kcycles for
    // the longest call; what had slowed the sweep to ~470 cycles per job was
    // two waves per SIMD, see plan_mixed_kernel's first sweep)
    auto read = [&](uint32_t j) { return *(lds_u32*)(&blocks[group(j)]); };
    uint32_t va = 0, vb = 0;
    if (x < J) {
        va = read(x);
        vb = read(x + kSimXcds < J ? x + kSimXcds : x);
    }
    // job j from v (its group's word), whose register then takes the job two
    // ahead (a job of this lane's past the end); two jobs per iteration so
    // the two words alternate with no register copy (a copy waited for the
    // newest read)
    for (uint32_t j = x; j < J; j += 2u * kSimXcds) {
        {
            const float d = sim_dur(va, j, Hs, F, cs, cT, cS);
            va = read(j + 2u * kSimXcds < J ? j + 2u * kSimXcds : j);
            sim_insert(t, d);
        }
        {  // past the end a job of duration 0, which ends at t[0]: no change
            // (unconditional, so both reads are always in flight and the wait
            // before the first step is for the older one only)
            const uint32_t k = j + kSimXcds < J ? j + kSimXcds : j;
            const float d = j + kSimXcds < J ? sim_dur(vb, k, Hs, F, cs, cT, cS) : 0.0f;
            vb = read(k + 2u * kSimXcds < J ? k + 2u * kSimXcds : k);
            sim_insert(t, d);
        }
    }
    uint32_t last = 0u;
#pragma unroll
    for (uint32_t i = 0; i < kSimCus; ++i)
        if (i < per) last = max(last, t[i]);
    return __uint_as_float(last);
}

// One workgroup, two stages.  Bounds: every mode-0 plan (H in [0, hcap] or
// H = G, F in {4, 8}) gets the makespan bounds above, the smallest wins
// (ties: smaller H, then F = 4).  Simulation (up to kSimMaxG groups on 8 XCDs of <= 32
// CUs): ~80 candidates around it are simulated and the shortest wins, or
// all-split within 0.5 % of it; beyond that, the bounds' plan or mode 1 by
// the same bounds.  The plan depends on the lengths and, through the fused
// shapes' two constants, on whether each group's chunks lie together
// (round 4: laid out longest-first, the fused tail streams lane-per-chunk
// and a split head + fused tail beats the 8-wave mode).  forced: write
// {fmode, fh, ff} as given (tests, A/B).
constexpr int kPlanThreads = 1024;
constexpr uint32_t kPlanMaxH = 4096;  // largest split head the model search considers
// (H, F) pairs whose bounds the search keeps for the candidates: every pair
// while the head cap (mixed_grid: min(G, 4 x CUs, 4096)) is <= 1024, as on
// 256 CUs; the candidates of a larger cap recompute theirs
constexpr uint32_t kPairStore = 2u * 1025u + 1u;

__global__ __launch_bounds__(kPlanThreads) void plan_mixed_kernel(BatchArgs A, const uint32_t* sorted_len,
                                                                  uint32_t cus, uint32_t hcap, int forced,
                                                                  uint32_t fmode, uint32_t fh, uint32_t ff,
                                                                  uint32_t* plan, const uint64_t* lay_tb,
                                                                  const uint32_t* lay_bits, const uint32_t* lay_blk) {
    const uint32_t n = A.n;
    const uint32_t t = threadIdx.x;
    if (t == 0) plan[3] = 0u;  // the persistent kernel's job counter
    // stage end times (s_memrealtime, 100 MHz; plan[8..12], thread 0) for
    // SHA1CHUNK_MIXED_DEBUG: scan, bounds search, the first simulation
    // sweep, pass 2's rest, pass 3's misses
    uint64_t ts[6] = {0, 0, 0, 0, 0, 0};
    // and the shader-clock cycles at the same points (plan[14..18])
    uint64_t cs[6] = {0, 0, 0, 0, 0, 0};
    if (t == 0) {
        ts[0] = __builtin_amdgcn_s_memrealtime();
        cs[0] = __builtin_amdgcn_s_memtime();
    }
    if (forced) {
        if (t == 0) {
            plan[0] = fmode;
            plan[1] = fh;
            plan[2] = ff;
        }
        return;
    }
    __shared__ uint64_t scan[kPlanThreads];
    __shared__ double best_m[kPlanThreads / 64];
    __shared__ uint32_t best_h[kPlanThreads / 64], best_f[kPlanThreads / 64];
    __shared__ uint64_t prefix[kPlanMaxH + 1];
    const uint32_t G = (n + 63u) / 64u;
    const uint32_t per = (G + kPlanThreads - 1) / kPlanThreads;
    const uint32_t g0 = min(G, t * per), g1 = min(G, g0 + per);
    uint64_t local = 0, local_t = 0;
    __shared__ uint32_t blocks[kSimMaxG];  // group_blocks of groups < kSimMaxG, for the simulation
    __shared__ uint32_t togw[kSimMaxG / 32];  // plan_layout_kernel's bits, groups < kSimMaxG
    for (uint32_t g = g0; g < g1; ++g) {
        const uint32_t b = lay_blk[g];  // group_blocks(sorted_len, g), coalesced (plan_layout_kernel)
        if (g < kSimMaxG) blocks[g] = b;
        local += b;
    }
    const uint32_t W = (G + 31u) / 32u;
    for (uint32_t w = t; w < W; w += kPlanThreads) {
        if (w < kSimMaxG / 32) togw[w] = lay_bits[w];
        local_t += lay_tb[w];
    }
    // inclusive scan of the threads' block counts: in the wave, then over
    // the 16 wave totals (Hillis-Steele over the workgroup took 20 barriers)
    const uint32_t lane = t & 63u, wv = t >> 6;
    __shared__ uint64_t wtot[kPlanThreads / 64];
    __shared__ uint64_t wtog[kPlanThreads / 64];  // per-wave toggled-block sums, added after the barrier
    uint64_t inc = local;
#pragma unroll
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint64_t v = __shfl_up(inc, d);
        if (lane >= d) inc += v;
    }
    for (uint32_t m = 32; m >= 1; m >>= 1) local_t += __shfl_xor(local_t, m);
    if (lane == 63u) wtot[wv] = inc;
    if (lane == 0u) wtog[wv] = local_t;
    __syncthreads();
    uint64_t before = 0, PG = 0, tog_blocks = 0;
#pragma unroll
    for (uint32_t w = 0; w < kPlanThreads / 64; ++w) {
        before += w < wv ? wtot[w] : 0ull;
        PG += wtot[w];
        tog_blocks += wtog[w];
    }
    scan[t] = before + inc;
    const double ft = PG ? (double)tog_blocks / (double)PG : 1.0;
    if (t == 0) {
        ts[1] = __builtin_amdgcn_s_memrealtime();
        cs[1] = __builtin_amdgcn_s_memtime();
    }
    __shared__ uint8_t run8[kSimMaxG];
    for (uint32_t g = t; g < min(G, kSimMaxG); g += kPlanThreads) {
        uint32_t r = 0;
        for (uint32_t i = g; i < g + 8u; ++i, ++r) {
            const bool tg = i >= G || (i < kSimMaxG ? ((togw[i >> 5] >> (i & 31u)) & 1u) != 0 : ft >= 0.5);
            if (!tg) break;
        }
        run8[g] = static_cast<uint8_t>(r);
        blocks[g] |= r << 28;  // for sim_xcd, one LDS read per job (blocks < 2^27)
    }
    __syncthreads();
    const PlanLayout L{run8, ft >= 0.5};
    uint64_t bsub[3] = {0, 0, 0};  // shader-clock stamps inside the bounds stage (plan[24..26])
    if (t == 0) bsub[0] = __builtin_amdgcn_s_memtime();
    // P_H for every candidate H <= hcap, then each thread takes H = t, t + 1024, ..
    uint64_t P = scan[t] - local;  // P_{g0}
    for (uint32_t g = g0; g <= g1 && g <= hcap; ++g) {
        prefix[g] = P;
        if (g < g1) P += plan_blocks(sorted_len, blocks, g);
    }
    __syncthreads();
    if (t == 0) bsub[1] = __builtin_amdgcn_s_memtime();
    // every (H, F): H in [0, hcap] with F = 4 and, below G, 8, and H = G
    // (every group split) beyond hcap; pair w = 2H + (F == 8), the last one
    // H = G, dealt evenly over the threads (thread 0 took H = 0, 1024 and G
    // at 2048 groups: 5 bounds against 2)
    double bm = 1e300;
    uint32_t bh = 0, bf = 4;
    const uint32_t npair = 2u * (hcap + 1u) + (G > hcap ? 1u : 0u);
    __shared__ double pbnd[kPairStore];  // pair w's bound, for the candidates' (same call, same value)
    __shared__ double m1b;               // the 8-wave mode's bound
    for (uint32_t w = t; w < npair; w += kPlanThreads) {
        const bool all = w == 2u * (hcap + 1u);  // H = G beyond hcap
        const uint32_t H = all ? G : w / 2u, F = all ? 4u : 4u + 4u * (w & 1u);
        if (F == 8u && H >= G) continue;  // H = G: every group split, F = 4 only
        const double m = makespan(sorted_len, blocks, L, ft, G, cus, 0, H, F, all ? PG : prefix[H], PG);
        if (w < kPairStore) pbnd[w] = m;
        if (m < bm || (m == bm && (H < bh || (H == bh && F < bf)))) { bm = m; bh = H; bf = F; }
    }
    // the last thread has the fewest pairs (or as many as any)
    if (t == kPlanThreads - 1) m1b = makespan(sorted_len, blocks, L, ft, G, cus, 1, 0, 0, 0, PG);
    if (t == 0) bsub[2] = __builtin_amdgcn_s_memtime();
    // the smallest (bound, head, F) over the workgroup: in the wave, then
    // over the 16 waves' bests
#pragma unroll
    for (uint32_t m = 32; m >= 1; m >>= 1) {
        const double mo = __shfl_xor(bm, m);
        const uint32_t ho = __shfl_xor(bh, m), fo = __shfl_xor(bf, m);
        if (mo < bm || (mo == bm && (ho < bh || (ho == bh && fo < bf)))) {
            bm = mo;
            bh = ho;
            bf = fo;
        }
    }
    if (lane == 0u) {
        best_m[wv] = bm;
        best_h[wv] = bh;
        best_f[wv] = bf;
    }
    __syncthreads();
    if (t < 64) {  // the 16 waves' bests, reduced by wave 0
        constexpr uint32_t kW = kPlanThreads / 64;
        bm = t < kW ? best_m[t] : 1e300;
        bh = t < kW ? best_h[t] : 0xffffffffu;
        bf = t < kW ? best_f[t] : 8u;
#pragma unroll
        for (uint32_t m = kW / 2; m >= 1; m >>= 1) {
            const double mo = __shfl_xor(bm, m);
            const uint32_t ho = __shfl_xor(bh, m), fo = __shfl_xor(bf, m);
            if (mo < bm || (mo == bm && (ho < bh || (ho == bh && fo < bf)))) {
                bm = mo;
                bh = ho;
                bf = fo;
            }
        }
        if (t == 0) {
            best_m[0] = bm;
            best_h[0] = bh;
            best_f[0] = bf;
        }
    }
    __syncthreads();
    if (t == 0) {
        ts[2] = __builtin_amdgcn_s_memrealtime();
        cs[2] = __builtin_amdgcn_s_memtime();
    }
    const bool simulate = G <= kSimMaxG && cus % kSimXcds == 0 && cus / kSimXcds <= kSimCus;
    if (!simulate) {
        if (t == 0) {
            const bool split8 = m1b < best_m[0];
            plan[0] = split8 ? 1u : 0u;
            plan[1] = split8 ? 0u : best_h[0];
            plan[2] = split8 ? 0u : best_f[0];
#pragma unroll
            for (int i = 8; i < 13; ++i) plan[i] = 0u;  // no simulation stages
        }
        return;
    }
    // Candidates, in the order every pass and the final choice index them
    // (tests/test_gpu_mixed.py candidates()): 0 the bounds' best plan, 1 the
    // 8-wave mode, 2 all-split, then heads hb - d, hb + d for d = 1, 2, 4 ..
    // 64 while in range (only H <= hcap: prefix[] holds P_H there -- when
    // the best is all-split beyond hcap, hb - d would be neither a searched
    // head nor all-split), then a grid of 32 heads up to 2C at F = 4 and,
    // below G, 8.  Wave 0 builds the list in parallel (positions from
    // ballots), then each candidate's makespan bounds are computed once.
    constexpr uint32_t kMaxCand = kPlanThreads / kSimXcds;
    // heads hb -/+ 1..12 simulated in the first sweep: with the bounds' plan
    // and the near candidates they are <= 32 candidates, four waves, one per
    // SIMD (44 candidates put two waves on some SIMDs: 38.6 against 25.4
    // kcycles, tools/sim_probe.hip, profiles/sim_probe2_r05.log)
    constexpr uint32_t kSpec = 24;
    __shared__ uint32_t cmode[kMaxCand], chead[kMaxCand], cf[kMaxCand], ncand, nref, npend, nmiss, nrun;
    __shared__ float cmk[kMaxCand], scmk[kSpec];
    __shared__ double clb[kMaxCand];
    __shared__ uint8_t cstate[kMaxCand], sval[kSpec];
    __shared__ uint8_t runidx[kMaxCand];  // the first sweep's work: slot, or 128 + early head
    __shared__ uint32_t simcyc;  // debug: the longest simulate call of the first sweep (plan[27])
    const uint32_t hb = best_h[0], fb = best_f[0];
    const double mb = best_m[0];
    auto put = [&](uint32_t k, uint32_t m, uint32_t h, uint32_t f) {
        cmode[k] = m;
        chead[k] = h;
        cf[k] = h == G ? 4u : f;
    };
    if (t < kMaxCand) cstate[t] = 0;
    if (t == 0) simcyc = 0;
    if (t < 64) {
        // lanes 0..13: the d entries (lane 2q: hb - 2^q, 2q + 1: hb + 2^q);
        // lanes 14..45: grid head i = lane - 14 (at F = 4, and 8 below G)
        uint32_t cnt = 0, h0 = 0, f0 = 0;
        if (t < 14) {
            const uint32_t d = 1u << (t >> 1);
            if ((t & 1u) == 0u ? (hb >= d && hb - d <= hcap) : (hb + d <= hcap)) {
                cnt = 1;
                h0 = (t & 1u) == 0u ? hb - d : hb + d;
                f0 = fb;
            }
        } else if (t < 46) {
            h0 = (t - 14u) * min(hcap, 2u * cus) / 31u;
            f0 = 4;
            cnt = h0 < G ? 2u : 1u;
        }
        const uint64_t below = (1ull << t) - 1ull;
        const uint32_t pos = 3u + __popcll(__ballot(cnt >= 1u) & below) + __popcll(__ballot(cnt == 2u) & below);
        if (cnt >= 1u) put(pos, 0, h0, f0);
        if (cnt == 2u) put(pos + 1u, 0, h0, 8);
        if (t == 0) {
            put(0, 0, hb, fb);
            put(1, 1, 0, 0);
            put(2, 0, G, 4);
            npend = 0;
            nmiss = 0;
        }
        if (t == 63) ncand = pos + cnt;
    } else if (t < 64 + kSpec) {
        // pass 3's heads if the bounds' best stays the best split-head plan
        const uint32_t q = t - 64u, d = q / 2u + 1u;
        const bool ok = hb < G && ((q & 1u) == 0u ? hb >= d : (hb + d <= hcap && hb + d < G));
        sval[q] = ok ? 1 : 0;
    }
    __syncthreads();
    uint64_t sub[3] = {0, 0, 0};  // shader-clock stamps inside the first sweep's stage (plan[20..22])
    if (t == 0) sub[0] = __builtin_amdgcn_s_memtime();
    if (t >= 1 && t < ncand) {  // the search's bounds (a call costs ~5 k cycles of latency)
        const uint32_t m = cmode[t], h = chead[t], f = cf[t];
        const uint32_t w = h <= hcap ? 2u * h + (f == 8u ? 1u : 0u) : 2u * (hcap + 1u);  // its pair
        clb[t] = m == 1 ? m1b
                        : (w < kPairStore ? pbnd[w]
                                          : makespan(sorted_len, blocks, L, ft, G, cus, 0, h, f,
                                                     h <= hcap ? prefix[h] : PG, PG));
    }
    __syncthreads();
    if (t == 0) sub[1] = __builtin_amdgcn_s_memtime();
    // the first sweep's work, packed onto the fewest waves (8 lanes each):
    // the bounds' plan, candidates within 5 % of its bounds, early heads
    // (and no longer chain than 1.25x its: a sweep lasts as long as its
    // longest candidate, and all-split's 2048 jobs at 2048 groups, often
    // within 5 % by its bounds, tripled it)
    const double early = mb * 1.05;
    const uint32_t jcap = plan_jobs(G, 0, hb, fb) + plan_jobs(G, 0, hb, fb) / 4u;
    if (t < 64) {
        uint32_t off = 0;
        for (uint32_t i = t; i < kMaxCand + kSpec; i += 64) {
            bool w = i < kMaxCand ? (i == 0 || (i < ncand && clb[i] < early &&
                                                plan_jobs(G, cmode[i], chead[i], cf[i]) <= jcap))
                                  : sval[i - kMaxCand] != 0;
            if (w && i >= 1u && i < kMaxCand && cmode[i] == 0u && cf[i] == fb) {
                // the same plan as the bounds' one or an early head: copied
                // from that one's result after the sweep, not run twice
                const uint32_t h = chead[i], e = h < hb ? hb - h : h - hb;
                if (e == 0u) {
                    cstate[i] = 5;
                    w = false;
                } else if (e <= kSpec / 2u && sval[2u * (e - 1u) + (h > hb ? 1u : 0u)]) {
                    cstate[i] = 4;
                    w = false;
                }
            }
            const uint64_t bal = __ballot(w);
            if (w) {
                runidx[off + __popcll(bal & ((1ull << t) - 1ull))] = static_cast<uint8_t>(i);
                if (i < kMaxCand) cstate[i] = 3;  // simulated in the first sweep
            }
            off += __popcll(bal);
        }
        if (t == 0) nrun = off;  // <= 1 + 80 + 24 (kMaxCand + kSpec slots fit the uint8 indices)
    }
    __syncthreads();
    if (t == 0) sub[2] = __builtin_amdgcn_s_memtime();
    // Pass 1 simulates the bounds' plan; pass 2 every other candidate whose
    // bounds are below that time (the rest cannot beat it; a 4096-group
    // all-split candidate alone is ~100 us of simulation); pass 3 the heads
    // next to the best split-head plan after pass 2.  Simulating is the
    // same for every candidate whenever it runs, so the first sweep takes
    // the bounds' plan, every candidate whose bounds are within 5 % of it
    // (pass 2's usual survivors) and pass 3's heads as they would be if the
    // bounds' best stays the best split head; pass 2's rest and pass 3's
    // misses follow only if needed.  Each sweep is the longest candidate's
    // chain of inserts, so this is one sweep instead of three in the usual
    // case.  The choice is the same as passes 1-3 in order.
    const uint32_t c = t / kSimXcds, x = t % kSimXcds, xcus = cus / kSimXcds;
    {
        const bool run = c < nrun;
        const uint32_t i = run ? runidx[c] : 0u, q = i - kMaxCand, d = q / 2u + 1u;
        const bool main = i < kMaxCand;
        // one call: two (one per kind of work) ran one after the other in a wave holding both
        const uint32_t sm = main ? cmode[i] : 0u, sh = main ? chead[i] : ((q & 1u) == 0u ? hb - d : hb + d);
        const uint32_t sf = main ? cf[i] : fb;
        float mk = __builtin_inff();
        const uint64_t w0 = __builtin_amdgcn_s_memtime();
        if (run) mk = sim_xcd(blocks, G, sm, sh, sf, x, xcus);
        const uint64_t w1 = __builtin_amdgcn_s_memtime();
        if (run && (t & 63u) == 0u) atomicMax(&simcyc, static_cast<uint32_t>(w1 - w0));
#pragma unroll
        for (uint32_t m = 1; m < kSimXcds; m *= 2) mk = fmaxf(mk, __shfl_xor(mk, m));
        if (x == 0 && run) {
            if (main)
                cmk[i] = mk;
            else
                scmk[q] = mk;
        }
        __syncthreads();
        if (t == 0) {
            ts[3] = __builtin_amdgcn_s_memrealtime();
            cs[3] = __builtin_amdgcn_s_memtime();
        }
    }
    // pass 2's rule: bounds at or above the bounds' plan's simulated time
    // rule a candidate out (cmk = inf, simulated early or not)
    if (t >= 1 && t < ncand) {
        if (cstate[t] >= 4) {  // a copy of the bounds' plan or of an early head
            const uint32_t h = chead[t], e = h < hb ? hb - h : h - hb;
            cmk[t] = cstate[t] == 5 ? cmk[0] : scmk[2u * (e - 1u) + (h > hb ? 1u : 0u)];
            cstate[t] = 3;
        }
        if (!(clb[t] < (double)cmk[0])) {
            cmk[t] = __builtin_inff();
        } else if (cstate[t] != 3) {
            cstate[t] = 1;
            atomicAdd(&npend, 1u);
        }
    }
    __syncthreads();
    if (npend) {
        const bool run = c < ncand && cstate[c] == 1;
        float mk = __builtin_inff();
        if (run) mk = sim_xcd(blocks, G, cmode[c], chead[c], cf[c], x, xcus);
#pragma unroll
        for (uint32_t m = 1; m < kSimXcds; m *= 2) mk = fmaxf(mk, __shfl_xor(mk, m));
        if (x == 0 && run) cmk[c] = mk;
        __syncthreads();
    }
    if (t == 0) {
        ts[4] = __builtin_amdgcn_s_memrealtime();
        cs[4] = __builtin_amdgcn_s_memtime();
    }
    // Pass 3: heads next to the shortest split-head plan so far (same F;
    // whichever plan is shortest overall).  The simulated
    // time is jagged in H -- a head that fills the XCDs' CUs evenly beats its
    // neighbours by several percent (config-5 law at 131072 chunks in
    // arrival order: H = 187 simulated 13.88 ms and measured 13.92, mode 1
    // 14.09 / 14.27, H = 176 14.35 / 14.41) and the grid above steps ~16
    // heads, so every head within 8 of the best split-head plan is tried
    // (taken from the first sweep when it simulated that head).
    // bi: the shortest mode-0 candidate with a fused tail, first on ties --
    // the smallest (time bits, index) over the slots (times are >= 0 or
    // +inf, so their bits order as unsigned integers)
    __shared__ uint64_t red[kMaxCand / 64];
    if (t < kMaxCand) {
        const bool el = t < ncand && cmode[t] == 0 && chead[t] < G;
        uint64_t key = el ? (uint64_t)__float_as_uint(cmk[t]) << 32 | t : ~0ull;
#pragma unroll
        for (uint32_t m = 32; m >= 1; m >>= 1) key = min(key, (uint64_t)__shfl_xor(key, m));
        if (lane == 0u) red[wv] = key;
    }
    __syncthreads();
    if (t < 64) {  // the 16 heads, lane j: d = j / 2 + 1, below (j even) or above bi's head
        uint64_t key = red[0];
#pragma unroll
        for (uint32_t w = 1; w < kMaxCand / 64; ++w) key = min(key, red[w]);
        const bool have = (uint32_t)(key >> 32) < 0x7f800000u;  // some candidate, and finite
        const uint32_t bi = (uint32_t)key;
        const uint32_t h2 = have ? chead[bi] : 0u, f2 = have ? cf[bi] : 4u, d = t / 2u + 1u;
        const bool lo = (t & 1u) == 0u;
        const bool ok = have && t < 16u && (lo ? h2 >= d : (h2 + d <= hcap && h2 + d < G));
        const uint32_t h = lo ? h2 - d : h2 + d;
        const uint32_t k = ncand + __popcll(__ballot(ok) & ((1ull << t) - 1ull));  // < kMaxCand: ncand <= 81
        bool miss = false;
        if (ok) {
            put(k, 0, h, f2);
            const uint32_t e = h < hb ? hb - h : h - hb;  // its early slot, if any
            const uint32_t q = e >= 1u ? 2u * (e - 1u) + (h > hb ? 1u : 0u) : 0u;
            if (f2 == fb && h == hb) {
                cmk[k] = cmk[0];
            } else if (f2 == fb && e >= 1u && e <= kSpec / 2u && sval[q]) {
                cmk[k] = scmk[q];
            } else {
                cstate[k] = 2;
                miss = true;
            }
        }
        const uint64_t ballot_ok = __ballot(ok), ballot_miss = __ballot(miss);
        if (t == 0) {
            nref = ncand + __popcll(ballot_ok);
            nmiss = __popcll(ballot_miss);
        }
    }
    __syncthreads();
    if (nmiss) {
        const bool run = c >= ncand && c < nref && cstate[c] == 2;
        float mk = __builtin_inff();
        if (run) mk = sim_xcd(blocks, G, cmode[c], chead[c], cf[c], x, xcus);
#pragma unroll
        for (uint32_t m = 1; m < kSimXcds; m *= 2) mk = fmaxf(mk, __shfl_xor(mk, m));
        if (x == 0 && run) cmk[c] = mk;
        __syncthreads();
    }
    // the shortest of all, first on ties
    if (t < kMaxCand) {
        uint64_t key = t < nref ? (uint64_t)__float_as_uint(cmk[t]) << 32 | t : ~0ull;
#pragma unroll
        for (uint32_t m = 32; m >= 1; m >>= 1) key = min(key, (uint64_t)__shfl_xor(key, m));
        if (lane == 0u) red[wv] = key;
    }
    __syncthreads();
    if (t == 0) {
        ts[5] = __builtin_amdgcn_s_memrealtime();
        cs[5] = __builtin_amdgcn_s_memtime();
        uint64_t key = red[0];
#pragma unroll
        for (uint32_t w = 1; w < kMaxCand / 64; ++w) key = min(key, red[w]);
        uint32_t bi = (uint32_t)key;
        // All-split (candidate 2) within 0.5 % of the best is taken instead:
        // a chain-bound batch then runs with no fused waves heating the chip
        // (65536 chunks of the config-5 law: 12.14 ms all-split against 12.50
        // for a split head + fused tail simulated as equal).
        if (cmk[2] <= cmk[bi] * 1.005f) bi = 2;
        plan[0] = cmode[bi];
        plan[1] = cmode[bi] == 1 ? 0u : chead[bi];
        plan[2] = cmode[bi] == 1 ? 0u : cf[bi];
#pragma unroll
        for (int i = 1; i < 6; ++i) plan[7 + i] = static_cast<uint32_t>(ts[i] - ts[0]);
#pragma unroll
        for (int i = 1; i < 6; ++i) plan[13 + i] = static_cast<uint32_t>(cs[i] - cs[0]);
#pragma unroll
        for (int i = 0; i < 3; ++i) plan[20 + i] = static_cast<uint32_t>(sub[i] - cs[0]);
        plan[23] = nrun;
#pragma unroll
        for (int i = 0; i < 3; ++i) plan[24 + i] = static_cast<uint32_t>(bsub[i] - cs[0]);
        plan[27] = simcyc;
    }
}

// ------------------------------------------------------------ utilities ---
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// One workgroup per chunk: chunk c (global index first + blockIdx.x) of
// length len is written at dst + off.  dst + off must be 8-byte aligned.
__global__ __launch_bounds__(256) void synth_fill_kernel(uint8_t* dst, const uint64_t* off,
                                                         const uint32_t* lens, uint32_t ulen,
                                                         uint64_t first, uint64_t seed) {
    const uint64_t c = blockIdx.x;
    const uint32_t len = lens ? lens[c] : ulen;
    uint8_t* out = dst + (off ? off[c] : c * (uint64_t)ulen);
    const uint64_t key = seed ^ ((first + c) << 24);
    const uint32_t nw = len >> 3;
    uint64_t* o = reinterpret_cast<uint64_t*>(out);
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) o[w] = splitmix64(key ^ (uint64_t)w);
    const uint32_t rem = len & 7u;
    if (rem && threadIdx.x == 0) {
        const uint64_t v = splitmix64(key ^ (uint64_t)nw);
        for (uint32_t b = 0; b < rem; ++b) out[8ull * nw + b] = (uint8_t)(v >> (8 * b));
    }
}

__global__ __launch_bounds__(256) void compare_kernel(const uint8_t* dig, const uint8_t* exp,
                                                      uint32_t n, uint8_t* mismatch) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t diff = 0;
#pragma unroll
    for (int b = 0; b < 20; ++b) diff |= (uint32_t)(dig[20ull * i + b] ^ exp[20ull * i + b]);
    mismatch[i] = diff ? 1 : 0;
}

// ------------------------------------------------------------ launchers ---
hipError_t launch_lane(const BatchArgs& A, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t grid = (A.n + 255u) / 256u;
    hipLaunchKernelGGL(sha1_lane_kernel, dim3(grid), dim3(256), 0, st, A);
    return hipGetLastError();
}

hipError_t launch_fused(const BatchArgs& A, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    hipLaunchKernelGGL(sha1_fused_kernel, dim3((A.n + 255u) / 256u), dim3(256), 0, st, A);
    return hipGetLastError();
}

// Split shapes beyond the product's (the A/B library, tools/ab_kernels.hip,
// `make ab`, overrides these weak definitions; the product library holds only
// what AUTO dispatches: units 1, 4, 11).
__attribute__((weak)) bool split_unit_study_built(int) { return false; }
__attribute__((weak)) hipError_t launch_split_study(const BatchArgs&, int, hipStream_t) {
    return hipErrorInvalidValue;
}

bool split_unit_built(int u) { return u == 1 || u == 4 || u == 11 || split_unit_study_built(u); }

hipError_t launch_split(const BatchArgs& A, int unit_blocks, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t groups = (A.n + 63u) / 64u;
    switch (unit_blocks) {
    case 1: hipLaunchKernelGGL((sha1_split_kernel<1, 1>), dim3(groups), dim3(128), 0, st, A); break;
    case 4:  // two producers per consumer (kSplitNProd<4>), wave 2 empty: 256 threads
        hipLaunchKernelGGL((sha1_split_kernel<4, 1, kSplitV<4>, kSplitNProd<4>>), dim3(groups),
                           dim3(64 * (1 + kSplitNProd<4>) + ((kSplitV<4> & kVSkipWave2) ? 64 : 0)), 0,
                           st, A);
        break;
    case 11:  // <= 2 groups per CU: 2 pairs x (consumer + 2 producers), 2-block
              // units, 8-wave layout, producer SIMDs crossed between the pairs.
              // Chunks back to back (the uniform layout): lane-per-chunk producer
              // loads -- no TLB thrash to avoid, and the shared loads' LDS
              // transpose adds to this shape's LDS contention (LDS-issue stall
              // 9.8 % of wave time against 1.9 % at one group per CU): 6.33
              // against 6.41 ms at 32768 chunks, steady clock
              // (profiles/shard_ab_r03.json).  Ragged (possibly scattered)
              // chunks keep the shared loads.
        if (A.off == nullptr && A.order == nullptr)
            hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V & ~kVCoop, 2>), dim3((groups + 1) / 2), dim3(512),
                               0, st, A);
        else
            hipLaunchKernelGGL((sha1_split_kernel<2, 2, kSplit8V, 2>), dim3((groups + 1) / 2), dim3(512), 0,
                               st, A);
        break;
    default: return launch_split_study(A, unit_blocks, st);
    }
    return hipGetLastError();
}

uint32_t mixed_grid(uint32_t groups, int cus, uint32_t* hcap) {
    *hcap = std::min<uint32_t>(std::min<uint32_t>(groups, 4u * (uint32_t)cus), kPlanMaxH);
    // the largest workgroup count of any plan: every group split (H = G)
    return groups;
}

hipError_t launch_plan_layout(const BatchArgs& A, const uint32_t* sorted_len, const BigFix* big, uint32_t* plan,
                              hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t groups = (A.n + 63u) / 64u;
    // plan area (mixed_plan_bytes): 64 plan words, then the layout summary
    const uint32_t words = (groups + 31u) / 32u;
    uint64_t* lay_tb = reinterpret_cast<uint64_t*>(plan + 64);
    uint32_t* lay_bits = reinterpret_cast<uint32_t*>(lay_tb + words);
    uint32_t* lay_blk = lay_bits + words;
    hipLaunchKernelGGL(plan_layout_kernel, dim3(words), dim3(kLayoutThreads), 0, st, A, sorted_len,
                       big ? *big : BigFix{}, lay_tb, lay_bits, lay_blk);
    return hipGetLastError();
}

hipError_t launch_mixed(const BatchArgs& A, const uint32_t* sorted_len, const BigFix* big, uint32_t* plan, int cus,
                        const int* forced, hipStream_t st) {
    if (A.n == 0) return hipSuccess;
    const uint32_t groups = (A.n + 63u) / 64u;
    uint32_t hcap;
    const uint32_t grid = mixed_grid(groups, cus, &hcap);
    // plan area (mixed_plan_bytes): 64 plan words, then the layout summary
    const uint32_t words = (groups + 31u) / 32u;
    uint64_t* lay_tb = reinterpret_cast<uint64_t*>(plan + 64);
    uint32_t* lay_bits = reinterpret_cast<uint32_t*>(lay_tb + words);
    const uint32_t* lay_blk = lay_bits + words;
    if (!forced) {
        const hipError_t le = launch_plan_layout(A, sorted_len, big, plan, st);
        if (le != hipSuccess) return le;
    }
    hipLaunchKernelGGL(plan_mixed_kernel, dim3(1), dim3(kPlanThreads), 0, st, A, sorted_len,
                       (uint32_t)cus, hcap, forced ? 1 : 0, forced ? (uint32_t)forced[0] : 0u,
                       forced ? (uint32_t)forced[1] : 0u, forced ? (uint32_t)forced[2] : 0u, plan, lay_tb,
                       lay_bits, lay_blk);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    BatchArgs B = A;
    B.plan = plan;
    // Default: the persistent work-queue variant (one workgroup per CU
    // pulling the plan's jobs).  SHA1CHUNK_MIXED_DISPATCH=hw launches one
    // workgroup per job instead (the hardware dispatcher's order).  The two
    // measure the same plan for plan: geometric mean 0.999, -2.8 .. +1.8 %
    // over 92 (plan, size, layout) points (profiles/mixed_dispatch_ab_r03.json).
    const char* disp = getenv("SHA1CHUNK_MIXED_DISPATCH");
    const bool persistent = !(disp && !strcmp(disp, "hw"));
    if (persistent)
        hipLaunchKernelGGL(sha1_mixed_persistent_kernel, dim3((uint32_t)cus), dim3(kMixedThreads), 0, st, B,
                           plan + 3);
    else
        hipLaunchKernelGGL(sha1_mixed_kernel, dim3(grid), dim3(kMixedThreads), 0, st, B);
    return hipGetLastError();
}

hipError_t launch_vq_drain(const VqDrainArgs& Q, uint32_t grid, hipStream_t st) {
    hipLaunchKernelGGL(sha1_vq_drain_kernel, dim3(grid), dim3(kMixedThreads), 0, st, Q);
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* dst, const uint64_t* off, const uint32_t* lens, uint32_t ulen,
                        uint64_t first, uint64_t count, uint64_t seed, hipStream_t st) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_fill_kernel, dim3((uint32_t)count), dim3(256), 0, st, dst, off, lens,
                       ulen, first, seed);
    return hipGetLastError();
}

hipError_t launch_compare(const uint8_t* dig, const uint8_t* exp, uint32_t n, uint8_t* mismatch,
                          hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(compare_kernel, dim3((n + 255u) / 256u), dim3(256), 0, st, dig, exp, n,
                       mismatch);
    return hipGetLastError();
}

#ifdef SHA1CHUNK_CHECKED
// Bounds violations counted by the checked build's fetch_entry on every
// device since the last reset (reset != 0 zeroes the counters after reading).
// Exported by the checked backend only: tests/conftest.py reads it after each
// GPU test when SHA1CHUNK_CHECKED=1.
extern "C" __attribute__((visibility("default"))) long long s1be_checked_violations(int reset) {
    int cur = 0, nd = 0;
    if (hipGetDevice(&cur) != hipSuccess || hipGetDeviceCount(&nd) != hipSuccess) return -1;
    long long total = 0;
    for (int d = 0; d < nd; ++d) {
        unsigned int v = 0;
        if (hipSetDevice(d) != hipSuccess ||
            hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_checked_oob), sizeof v, 0, hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
        total += v;
        const unsigned int zero = 0;
        if (reset && hipMemcpyToSymbol(HIP_SYMBOL(g_checked_oob), &zero, sizeof zero, 0, hipMemcpyHostToDevice) !=
                         hipSuccess)
            return -1;
    }
    (void)hipSetDevice(cur);
    return total;
}
#endif
