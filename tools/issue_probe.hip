// issue_probe.hip -- diagnostic only (not part of the product): what one
// wave's instruction stream costs per instruction on gfx950 when nothing
// but issue limits it.  Straight-line blocks of 2048 instructions (no loop
// branch inside the timed region), timed with s_memtime (shader clock) and
// s_memrealtime (100 MHz) around the block, second launch (warm I-cache).
// Compares against tools/microbench.hip's 128-instruction loops, whose
// ~4.63 cycles per instruction is the split consumer's measured cadence.
//   hipcc --offload-arch=gfx950 -O3 tools/issue_probe.hip -o tools/issue_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

#define R2(x) x x
#define R4(x) R2(R2(x))
#define R16(x) R4(R4(x))
#define R256(x) R16(R16(x))

// Eight independent chains so no instruction waits on the one before it.
#define ADD8 "v_add_u32 v10, v10, v1\n v_add_u32 v11, v11, v1\n v_add_u32 v12, v12, v1\n v_add_u32 v13, v13, v1\n v_add_u32 v14, v14, v1\n v_add_u32 v15, v15, v1\n v_add_u32 v16, v16, v1\n v_add_u32 v17, v17, v1\n"
#define ADDF8 "v_add_f32 v10, v10, v1\n v_add_f32 v11, v11, v1\n v_add_f32 v12, v12, v1\n v_add_f32 v13, v13, v1\n v_add_f32 v14, v14, v1\n v_add_f32 v15, v15, v1\n v_add_f32 v16, v16, v1\n v_add_f32 v17, v17, v1\n"
#define ADD38 "v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_add3_u32 v12, v12, v1, v2\n v_add3_u32 v13, v13, v1, v2\n v_add3_u32 v14, v14, v1, v2\n v_add3_u32 v15, v15, v1, v2\n v_add3_u32 v16, v16, v1, v2\n v_add3_u32 v17, v17, v1, v2\n"
#define ALIGN8 "v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_alignbit_b32 v14, v14, v14, 27\n v_alignbit_b32 v15, v15, v15, 27\n v_alignbit_b32 v16, v16, v16, 27\n v_alignbit_b32 v17, v17, v17, 27\n"
#define NOP8 "s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"
#define ADD3S8 "v_add3_u32 v10, v10, v1, s2\n v_add3_u32 v11, v11, v1, s2\n v_add3_u32 v12, v12, v1, s2\n v_add3_u32 v13, v13, v1, s2\n v_add3_u32 v14, v14, v1, s2\n v_add3_u32 v15, v15, v1, s2\n v_add3_u32 v16, v16, v1, s2\n v_add3_u32 v17, v17, v1, s2\n"
// one SHA-1-like round, register-renamed over 8 slots: two dependent pairs
#define ROUND8 "v_alignbit_b32 v20, v10, v10, 27\n v_bitop3_b32 v21, v11, v12, v13 bitop3:0x96\n v_add_u32 v22, v14, v1\n v_add3_u32 v14, v20, v21, v22\n v_alignbit_b32 v11, v11, v11, 2\n v_alignbit_b32 v23, v14, v14, 27\n v_bitop3_b32 v24, v10, v11, v12 bitop3:0x96\n v_add_u32 v25, v13, v1\n"

#define KERNEL(NAME, BODY)                                                           \
    __global__ void NAME(uint64_t* st) {                                             \
        uint64_t t0, t1, q0, q1;                                                     \
        asm volatile("v_mov_b32 v1, 3\n v_mov_b32 v2, 5\n s_mov_b32 s2, 7\n"         \
                     "s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)"        \
                     : "=s"(t0), "=s"(q0)::"v1", "v2", "s2");                        \
        asm volatile(R256(BODY)::: "v10", "v11", "v12", "v13", "v14", "v15", "v16",   \
                     "v17", "v20", "v21", "v22", "v23", "v24", "v25");               \
        asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)"         \
                     : "=s"(t1), "=s"(q1));                                          \
        if (threadIdx.x == 0) {                                                      \
            st[0] = t1 - t0;                                                         \
            st[1] = q1 - q0;                                                         \
        }                                                                            \
    }

KERNEL(k_add, ADD8)
KERNEL(k_addf, ADDF8)
KERNEL(k_add3, ADD38)
KERNEL(k_add3s, ADD3S8)
KERNEL(k_align, ALIGN8)
KERNEL(k_nop, NOP8)
KERNEL(k_round, ROUND8)


// Same SHA-1 round mix with the consumer's schedule traffic folded in: 20
// LDS reads (or VMEM loads) of 16 B per lane per 400 VALU, the bytes one
// block's W+K needs.  The destination registers are never read by the VALU
// stream, so only issue / register-write costs can show.
#define RD128 "ds_read_b128 v[40:43], v30 offset:1024\n"
#define RD64 "ds_read_b64 v[40:41], v30 offset:2048\n"
#define RD32 "ds_read_b32 v40, v30 offset:4096\n"
#define GL128 "global_load_dwordx4 v[40:43], v[32:33], off\n"
#define WAIT "s_waitcnt lgkmcnt(4)\n"
#define VWAIT "s_waitcnt vmcnt(4)\n"
// 40 VALU (5 x ROUND8) + 2 x b128 spread = 20 per 400
#define MIX_SPREAD ROUND8 ROUND8 RD128 ROUND8 ROUND8 ROUND8 RD128 WAIT
// 100 VALU then a burst of 5 b128 (the consumer's grouping), 5 per 100
#define MIX_BURST ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 "v_add_u32 v26, v26, v1\n v_add_u32 v27, v27, v1\n v_add_u32 v28, v28, v1\n v_add_u32 v29, v29, v1\n" RD128 RD128 RD128 RD128 RD128 "s_waitcnt lgkmcnt(5)\n"
#define V100 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 ROUND8 "v_add_u32 v26, v26, v1\n v_add_u32 v27, v27, v1\n v_add_u32 v28, v28, v1\n v_add_u32 v29, v29, v1\n"
// 200 VALU then 10 reads; 400 VALU then 20 reads (the lgkm counter holds 15)
#define MIX_BURST10 V100 V100 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 "s_waitcnt lgkmcnt(10)\n"
#define MIX_BURST20 V100 V100 V100 V100 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 RD128 "s_waitcnt lgkmcnt(10)\n"
// bursts of 5, but each read's data waited for before the next burst
#define MIX_BURST5W V100 RD128 RD128 RD128 RD128 RD128 "s_waitcnt lgkmcnt(0)\n"
#define MIX_B64 ROUND8 ROUND8 RD64 ROUND8 RD64 ROUND8 RD64 ROUND8 RD64 WAIT
#define MIX_B32 ROUND8 RD32 RD32 ROUND8 RD32 RD32 ROUND8 RD32 RD32 ROUND8 RD32 RD32 ROUND8 RD32 RD32 WAIT
#define MIX_GL ROUND8 ROUND8 GL128 ROUND8 ROUND8 ROUND8 GL128 VWAIT

#define KERNEL_MEM(NAME, BODY, REPS, NVALU)                                          \
    __global__ void NAME(uint64_t* st, const uint32_t* g) {                          \
        __shared__ uint32_t lds[16384];                                              \
        lds[threadIdx.x] = threadIdx.x;                                              \
        __syncthreads();                                                             \
        uint64_t t0, t1, q0, q1;                                                     \
        const uint32_t a = (uint32_t)(uintptr_t)lds + threadIdx.x * 16;              \
        const uint32_t* gp = g + threadIdx.x * 4;                                    \
        asm volatile("v_mov_b32 v1, 3\n v_mov_b32 v2, 5\n v_mov_b32 v30, %2\n"        \
                     "v_mov_b32 v32, %3\n v_mov_b32 v33, %4\n"                        \
                     "s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)"        \
                     : "=s"(t0), "=s"(q0)                                            \
                     : "v"(a), "v"((uint32_t)(uintptr_t)gp),                         \
                       "v"((uint32_t)((uintptr_t)gp >> 32))                          \
                     : "v1", "v2", "v30", "v32", "v33");                             \
        asm volatile(REPS(BODY) "s_waitcnt lgkmcnt(0) vmcnt(0)\n" ::: "v10", "v11",   \
                     "v12", "v13", "v14", "v15", "v16", "v17", "v20", "v21", "v22",  \
                     "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v40", "v41",  \
                     "v42", "v43", "memory");                                        \
        asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)"         \
                     : "=s"(t1), "=s"(q1));                                          \
        if (threadIdx.x == 0) {                                                      \
            st[0] = t1 - t0;                                                         \
            st[1] = q1 - q0;                                                         \
            st[2] = NVALU;                                                           \
        }                                                                            \
    }

#define R5(x) x x x x x
#define R50(x) R5(R5(R2(x)))
#define R20(x) R5(R4(x))
KERNEL_MEM(m_spread, MIX_SPREAD, R50, 50 * 40)
KERNEL_MEM(m_burst, MIX_BURST, R20, 20 * 100)
KERNEL_MEM(m_b64, MIX_B64, R50, 50 * 40)
#define R10(x) R5(R2(x))
KERNEL_MEM(m_burst10, MIX_BURST10, R10, 10 * 200)
KERNEL_MEM(m_burst20, MIX_BURST20, R5, 5 * 400)
KERNEL_MEM(m_burst5w, MIX_BURST5W, R20, 20 * 100)
KERNEL_MEM(m_b32, MIX_B32, R50, 50 * 40)
KERNEL_MEM(m_gl, MIX_GL, R50, 50 * 40)
KERNEL_MEM(m_none, ROUND8 ROUND8 ROUND8 ROUND8 ROUND8, R50, 50 * 40)

static void run_mem(const char* name, void (*k)(uint64_t*, const uint32_t*), int lanes = 64) {
    uint64_t* st;
    uint32_t* g;
    CHECK(hipMalloc(&st, 32));
    CHECK(hipMalloc(&g, 64 * 16));
    CHECK(hipMemset(g, 0, 64 * 16));
    uint64_t best_c = ~0ull, best_q = 0, nv = 1;
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(lanes), 0, 0, st, g);
        CHECK(hipDeviceSynchronize());
        uint64_t h[3];
        CHECK(hipMemcpy(h, st, 24, hipMemcpyDeviceToHost));
        if (rep > 0 && h[0] < best_c) {
            best_c = h[0];
            best_q = h[1];
            nv = h[2];
        }
    }
    printf("{\"probe\": \"%s\", \"lanes\": %d, \"valu\": %llu, \"cycles_per_valu\": %.3f, "
           "\"ns_per_valu\": %.3f, \"clock_ghz\": %.3f}\n",
           name, lanes, (unsigned long long)nv, (double)best_c / nv, best_q * 10.0 / nv,
           best_c / (best_q * 10.0));
    CHECK(hipFree(st));
    CHECK(hipFree(g));
}


// operand-bank and dependency probes (bank = VGPR index mod 4)
#define ADD3_NOCONF "v_add3_u32 v10, v1, v2, v3\n v_add3_u32 v11, v1, v2, v3\n v_add3_u32 v12, v1, v2, v3\n v_add3_u32 v13, v1, v2, v3\n v_add3_u32 v14, v1, v2, v3\n v_add3_u32 v15, v1, v2, v3\n v_add3_u32 v16, v1, v2, v3\n v_add3_u32 v17, v1, v2, v3\n"
#define ADD3_CONF2 "v_add3_u32 v10, v1, v5, v3\n v_add3_u32 v11, v1, v5, v3\n v_add3_u32 v12, v1, v5, v3\n v_add3_u32 v13, v1, v5, v3\n v_add3_u32 v14, v1, v5, v3\n v_add3_u32 v15, v1, v5, v3\n v_add3_u32 v16, v1, v5, v3\n v_add3_u32 v17, v1, v5, v3\n"
#define ADD3_CONF3 "v_add3_u32 v10, v1, v5, v9\n v_add3_u32 v11, v1, v5, v9\n v_add3_u32 v12, v1, v5, v9\n v_add3_u32 v13, v1, v5, v9\n v_add3_u32 v14, v1, v5, v9\n v_add3_u32 v15, v1, v5, v9\n v_add3_u32 v16, v1, v5, v9\n v_add3_u32 v17, v1, v5, v9\n"
#define ALIGN_DUP "v_alignbit_b32 v10, v1, v1, 27\n v_alignbit_b32 v11, v2, v2, 27\n v_alignbit_b32 v12, v3, v3, 27\n v_alignbit_b32 v13, v1, v1, 27\n v_alignbit_b32 v14, v2, v2, 27\n v_alignbit_b32 v15, v3, v3, 27\n v_alignbit_b32 v16, v1, v1, 27\n v_alignbit_b32 v17, v2, v2, 27\n"
#define ALIGN_DIST "v_alignbit_b32 v10, v1, v2, 27\n v_alignbit_b32 v11, v2, v3, 27\n v_alignbit_b32 v12, v3, v1, 27\n v_alignbit_b32 v13, v1, v2, 27\n v_alignbit_b32 v14, v2, v3, 27\n v_alignbit_b32 v15, v3, v1, 27\n v_alignbit_b32 v16, v1, v2, 27\n v_alignbit_b32 v17, v2, v3, 27\n"
#define ALIGN_DUP_ADD "v_alignbit_b32 v10, v1, v1, 27\n v_add_u32 v11, v2, v3\n v_alignbit_b32 v12, v3, v3, 27\n v_add_u32 v13, v1, v2\n v_alignbit_b32 v14, v2, v2, 27\n v_add_u32 v15, v3, v1\n v_alignbit_b32 v16, v1, v1, 27\n v_add_u32 v17, v2, v3\n"
// dependent chains, conflict-free banks: each instruction consumes the previous result
#define DEP_ADD3 "v_add3_u32 v10, v13, v2, v3\n v_add3_u32 v13, v10, v2, v3\n v_add3_u32 v10, v13, v2, v3\n v_add3_u32 v13, v10, v2, v3\n v_add3_u32 v10, v13, v2, v3\n v_add3_u32 v13, v10, v2, v3\n v_add3_u32 v10, v13, v2, v3\n v_add3_u32 v13, v10, v2, v3\n"
#define DEP_ADD "v_add_u32 v10, v13, v2\n v_add_u32 v13, v10, v2\n v_add_u32 v10, v13, v2\n v_add_u32 v13, v10, v2\n v_add_u32 v10, v13, v2\n v_add_u32 v13, v10, v2\n v_add_u32 v10, v13, v2\n v_add_u32 v13, v10, v2\n"
#define DEP_ALIGN "v_alignbit_b32 v10, v13, v13, 27\n v_alignbit_b32 v13, v10, v10, 27\n v_alignbit_b32 v10, v13, v13, 27\n v_alignbit_b32 v13, v10, v10, 27\n v_alignbit_b32 v10, v13, v13, 27\n v_alignbit_b32 v13, v10, v10, 27\n v_alignbit_b32 v10, v13, v13, 27\n v_alignbit_b32 v13, v10, v10, 27\n"
#define DEP_BITOP3 "v_bitop3_b32 v10, v13, v2, v3 bitop3:0x96\n v_bitop3_b32 v13, v10, v2, v3 bitop3:0x96\n v_bitop3_b32 v10, v13, v2, v3 bitop3:0x96\n v_bitop3_b32 v13, v10, v2, v3 bitop3:0x96\n v_bitop3_b32 v10, v13, v2, v3 bitop3:0x96\n v_bitop3_b32 v13, v10, v2, v3 bitop3:0x96\n v_bitop3_b32 v10, v13, v2, v3 bitop3:0x96\n v_bitop3_b32 v13, v10, v2, v3 bitop3:0x96\n"
// distance-2 dependency: two interleaved chains
#define DEP2_ADD3 "v_add3_u32 v10, v13, v2, v3\n v_add3_u32 v11, v14, v2, v3\n v_add3_u32 v13, v10, v2, v3\n v_add3_u32 v14, v11, v2, v3\n v_add3_u32 v10, v13, v2, v3\n v_add3_u32 v11, v14, v2, v3\n v_add3_u32 v13, v10, v2, v3\n v_add3_u32 v14, v11, v2, v3\n"
#define DEP2_ALIGN "v_alignbit_b32 v10, v13, v13, 27\n v_alignbit_b32 v11, v14, v14, 27\n v_alignbit_b32 v13, v10, v10, 27\n v_alignbit_b32 v14, v11, v11, 27\n v_alignbit_b32 v10, v13, v13, 27\n v_alignbit_b32 v11, v14, v14, 27\n v_alignbit_b32 v13, v10, v10, 27\n v_alignbit_b32 v14, v11, v11, 27\n"
#define KERNEL2(NAME, BODY)                                                          \
    __global__ void NAME(uint64_t* st) {                                             \
        uint64_t t0, t1, q0, q1;                                                     \
        asm volatile("v_mov_b32 v1, 3\n v_mov_b32 v2, 5\n v_mov_b32 v3, 7\n v_mov_b32 v5, 9\n v_mov_b32 v9, 11\n v_mov_b32 v13, 1\n v_mov_b32 v14, 2\n" \
                     "s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)"        \
                     : "=s"(t0), "=s"(q0)::"v1", "v2", "v3", "v5", "v9", "v13", "v14"); \
        asm volatile(R256(BODY)::: "v10", "v11", "v12", "v13", "v14", "v15", "v16",   \
                     "v17");                                                         \
        asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)"         \
                     : "=s"(t1), "=s"(q1));                                          \
        if (threadIdx.x == 0) {                                                      \
            st[0] = t1 - t0;                                                         \
            st[1] = q1 - q0;                                                         \
        }                                                                            \
    }
KERNEL2(b_add3_noconf, ADD3_NOCONF)
KERNEL2(b_add3_conf2, ADD3_CONF2)
KERNEL2(b_add3_conf3, ADD3_CONF3)
KERNEL2(b_align_dup, ALIGN_DUP)
KERNEL2(b_align_dist, ALIGN_DIST)
KERNEL2(b_align_dup_add, ALIGN_DUP_ADD)
KERNEL2(d_add3, DEP_ADD3)
KERNEL2(d_add, DEP_ADD)
KERNEL2(d_align, DEP_ALIGN)
KERNEL2(d_bitop3, DEP_BITOP3)
KERNEL2(d2_add3, DEP2_ADD3)
KERNEL2(d2_align, DEP2_ALIGN)

static void run(const char* name, void (*k)(uint64_t*)) {
    uint64_t* st;
    CHECK(hipMalloc(&st, 16));
    uint64_t best_c = ~0ull, best_q = 0;
    for (int rep = 0; rep < 5; ++rep) {  // first launch warms the I-cache
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, st);
        CHECK(hipDeviceSynchronize());
        uint64_t h[2];
        CHECK(hipMemcpy(h, st, 16, hipMemcpyDeviceToHost));
        if (rep > 0 && h[0] < best_c) {
            best_c = h[0];
            best_q = h[1];
        }
    }
    const double n = 2048.0;
    printf("{\"probe\": \"%s\", \"instr\": 2048, \"cycles_per_instr\": %.3f, \"ns_per_instr\": %.3f, "
           "\"clock_ghz\": %.3f}\n",
           name, best_c / n, best_q * 10.0 / n, best_c / (best_q * 10.0));
    CHECK(hipFree(st));
}

int main() {
    run("v_add_u32 x8 chains", k_add);
    run("v_add_f32 x8 chains", k_addf);
    run("v_add3_u32 x8 chains", k_add3);
    run("v_add3_u32 sgpr operand", k_add3s);
    run("v_alignbit_b32 x8 chains", k_align);
    run("s_nop 0", k_nop);
    run("sha1 round mix", k_round);
    run("add3 operands in 3 banks", b_add3_noconf);
    run("add3 two operands share a bank", b_add3_conf2);
    run("add3 three operands share a bank", b_add3_conf3);
    run("alignbit x,x (rotate)", b_align_dup);
    run("alignbit x,y distinct banks", b_align_dist);
    run("alignbit x,x alternating with v_add", b_align_dup_add);
    run("dependent chain v_add3 (distance 1)", d_add3);
    run("dependent chain v_add_u32 (distance 1)", d_add);
    run("dependent chain v_alignbit rotate (distance 1)", d_align);
    run("dependent chain v_bitop3 (distance 1)", d_bitop3);
    run("two chains v_add3 (distance 2)", d2_add3);
    run("two chains v_alignbit (distance 2)", d2_align);
    run_mem("round mix, no schedule traffic", m_none);
    run_mem("+ ds_read_b128 spread (20/400 VALU)", m_spread);
    run_mem("+ ds_read_b128 bursts of 5 (20/400 VALU)", m_burst);
    run_mem("+ ds_read_b64 (40/400 VALU)", m_b64);
    run_mem("+ ds_read_b32 (80/400 VALU)", m_b32);
    run_mem("+ global_load_dwordx4 L2-hot (20/400 VALU)", m_gl);
    run_mem("+ ds_read_b128 bursts of 10 (20/400 VALU)", m_burst10);
    run_mem("+ ds_read_b128 one burst of 20 (20/400 VALU)", m_burst20);
    run_mem("+ ds_read_b128 bursts of 5, lgkmcnt(0) after each", m_burst5w);
    return 0;
}
