// microbench.hip -- diagnostic only (not part of the product): per-wave VALU
// issue cost and in-kernel clock on gfx950, to size the SHA-1 kernels'
// serial (single-wave) bound.  Clock = d(s_memtime) / d(s_memrealtime) x 100 MHz.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o tools/microbench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../congestion-control-with-bittorren_amd/csrc/sha1_device.hpp"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__device__ __forceinline__ uint64_t memtime() {
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ uint64_t realtime() {
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// MODE 0: 8 independent v_add chains; MODE 1: one dependent v_add3 chain;
// MODE 2: sha1-like round body (alignbit, bitop3, add3, add3, alignbit).
template <int MODE>
__global__ void issue_kernel(uint32_t* out, uint64_t* stamps, int iters) {
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
             r6 = r0 + 6, r7 = r0 + 7;
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t t0 = memtime(), q0 = realtime();
    __builtin_amdgcn_sched_barrier(0);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if constexpr (MODE == 0) {
                asm volatile(
                    "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\t"
                    "v_add_u32 %3, %3, %8\n\tv_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\t"
                    "v_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                    : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                    : "v"(r0));
            } else if constexpr (MODE == 1) {
                asm volatile(
                    "v_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %0, %0, %1, %2\n\t"
                    "v_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %0, %0, %1, %2\n\t"
                    "v_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %0, %0, %1, %2\n\t"
                    "v_add3_u32 %0, %0, %1, %2\n\tv_add3_u32 %0, %0, %1, %2"
                    : "+v"(r0)
                    : "v"(r1), "v"(r2));
            } else {
                // one round: r5 = rotl(a,5); f = bitop3(b,c,d); x = e+w+k; a' = add3; b = rotl(b,30)
                asm volatile(
                    "v_alignbit_b32 %5, %0, %0, 27\n\t"
                    "v_bitop3_b32 %6, %1, %2, %3 bitop3:0x96\n\t"
                    "v_add3_u32 %7, %4, %1, %2\n\t"
                    "v_add3_u32 %4, %5, %6, %7\n\t"
                    "v_alignbit_b32 %1, %1, %1, 2\n\t"
                    "v_alignbit_b32 %5, %4, %4, 27\n\t"
                    "v_bitop3_b32 %6, %0, %1, %2 bitop3:0x96\n\t"
                    "v_add3_u32 %7, %3, %0, %1\n\t"
                    "v_add3_u32 %3, %5, %6, %7\n\t"
                    "v_alignbit_b32 %0, %0, %0, 2"
                    : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t t1 = memtime(), q1 = realtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
    if ((threadIdx.x & 63) == 0) {
        const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        stamps[2 * w] = t1 - t0;
        stamps[2 * w + 1] = q1 - q0;
    }
}


// Per-opcode issue cost for one wave: 8 independent copies of OP per step.
#define OPK(NAME, ASM)                                                                   \
    __global__ void op_##NAME(uint32_t* out, uint64_t* stamps, int iters) {              \
        uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4,   \
                 r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7, s = r0 * 3, t = r0 * 5;           \
        __builtin_amdgcn_sched_barrier(0);                                               \
        const uint64_t t0 = memtime();                                                   \
        __builtin_amdgcn_sched_barrier(0);                                               \
        for (int i = 0; i < iters; ++i) {                                                \
            _Pragma("unroll") for (int j = 0; j < 16; ++j) {                             \
                asm volatile(ASM(0) ASM(1) ASM(2) ASM(3) ASM(4) ASM(5) ASM(6) ASM(7)      \
                             : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), \
                               "+v"(r6), "+v"(r7)                                        \
                             : "v"(s), "v"(t));                                          \
            }                                                                            \
        }                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                               \
        const uint64_t t1 = memtime();                                                   \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7; \
        if ((threadIdx.x & 63) == 0)                                                     \
            stamps[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;              \
    }
#define A_ADD(i) "v_add_u32 %" #i ", %" #i ", %8\n\t"
#define A_ADD3(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n\t"
#define A_ALIGN(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 27\n\t"
#define A_BITOP3(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x96\n\t"
#define A_XOR(i) "v_xor_b32 %" #i ", %" #i ", %8\n\t"
#define A_XOR3(i) "v_xor3_b32 %" #i ", %" #i ", %8, %9\n\t"
#define A_BFI(i) "v_bfi_b32 %" #i ", %" #i ", %8, %9\n\t"
#define A_PERM(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n\t"
#define A_LSHLADD(i) "v_lshl_add_u32 %" #i ", %" #i ", 5, %8\n\t"
#define A_MOVDPP(i) "v_mov_b32_dpp %" #i ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define A_NOP(i) "s_nop 0\n\t"
#define A_ALIGN2(i) "v_alignbit_b32 %" #i ", %8, %8, 27\n\t"
#define A_ALIGN3(i) "v_alignbit_b32 %" #i ", %8, %9, 27\n\t"
#define A_ALIGN4(i) "v_alignbit_b32 %" #i ", %" #i ", %8, 27\n\t"
#define A_ALIGN5(i) "v_alignbit_b32 %" #i ", %8, %" #i ", 27\n\t"
#define A_LSHL64(i) "v_lshlrev_b64 v[40:41], 5, v[42:43]\n\t"
#define A_PKMOV(i) "v_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\n\t"
#define A_ADD3S(i) "v_add3_u32 %" #i ", %" #i ", %8, 0x5a827999\n\t"
#define A_ADDSAME(i) "v_add3_u32 %" #i ", %" #i ", %" #i ", %8\n\t"
OPK(add, A_ADD)
OPK(add3, A_ADD3)
OPK(alignbit, A_ALIGN)
OPK(bitop3, A_BITOP3)
OPK(xor, A_XOR)
OPK(bfi, A_BFI)
OPK(perm, A_PERM)
OPK(lshl_add, A_LSHLADD)
OPK(mov_dpp, A_MOVDPP)
OPK(snop, A_NOP)
OPK(align_ss, A_ALIGN2)
OPK(align_st, A_ALIGN3)
OPK(align_rs, A_ALIGN4)
OPK(align_sr, A_ALIGN5)
OPK(lshl64, A_LSHL64)
OPK(pkmov, A_PKMOV)
OPK(add3_same, A_ADDSAME)

static void run_op(const char* name, void (*k)(uint32_t*, uint64_t*, int)) {
    const int iters = 2000;
    uint32_t* out;
    uint64_t* st;
    CHECK(hipMalloc(&out, 4 * 64));
    CHECK(hipMalloc(&st, 16));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, st, 10);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, st, iters);
    CHECK(hipDeviceSynchronize());
    uint64_t h;
    CHECK(hipMemcpy(&h, st, 8, hipMemcpyDeviceToHost));
    printf("{\"op\": \"%s\", \"cycles_per_instr_1wave\": %.3f}\n", name, (double)h / (iters * 16.0 * 8));
    CHECK(hipFree(out));
    CHECK(hipFree(st));
}


// Round mix with explicit registers: BANKS=0 -> every 3-source op reads three
// different banks (v40..v47 chosen by bank); BANKS=1 -> all sources in one
// bank (v40, v44, v48, v52 ...).
template <int BANKS>
__global__ void bank_kernel(uint32_t* out, uint64_t* stamps, int iters) {
    const uint64_t t0 = memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if constexpr (BANKS == 0) {
                asm volatile(
                    "v_alignbit_b32 v45, v40, v40, 27\n\t"
                    "v_bitop3_b32 v46, v41, v42, v43 bitop3:0x96\n\t"
                    "v_add3_u32 v47, v44, v49, v50\n\t"
                    "v_add3_u32 v44, v45, v46, v47\n\t"
                    "v_alignbit_b32 v41, v41, v41, 2\n\t"
                    "v_alignbit_b32 v45, v44, v44, 27\n\t"
                    "v_bitop3_b32 v46, v40, v41, v42 bitop3:0x96\n\t"
                    "v_add3_u32 v47, v43, v49, v50\n\t"
                    "v_add3_u32 v43, v45, v46, v47\n\t"
                    "v_alignbit_b32 v40, v40, v40, 2" ::: "v40", "v41", "v42", "v43", "v44",
                    "v45", "v46", "v47", "v49", "v50");
            } else {
                asm volatile(
                    "v_alignbit_b32 v60, v40, v40, 27\n\t"
                    "v_bitop3_b32 v64, v44, v48, v52 bitop3:0x96\n\t"
                    "v_add3_u32 v68, v56, v72, v76\n\t"
                    "v_add3_u32 v56, v60, v64, v68\n\t"
                    "v_alignbit_b32 v44, v44, v44, 2\n\t"
                    "v_alignbit_b32 v60, v56, v56, 27\n\t"
                    "v_bitop3_b32 v64, v40, v44, v48 bitop3:0x96\n\t"
                    "v_add3_u32 v68, v52, v72, v76\n\t"
                    "v_add3_u32 v52, v60, v64, v68\n\t"
                    "v_alignbit_b32 v40, v40, v40, 2" ::: "v40", "v44", "v48", "v52", "v56",
                    "v60", "v64", "v68", "v72", "v76");
            }
        }
    }
    const uint64_t t1 = memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = 0;
    if ((threadIdx.x & 63) == 0) stamps[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

template <int BANKS>
static void run_bank(const char* name, int blocks, int threads) {
    const int iters = 2000, waves = blocks * threads / 64;
    uint32_t* out;
    uint64_t* st;
    CHECK(hipMalloc(&out, 4 * blocks * threads));
    CHECK(hipMalloc(&st, 8 * waves));
    hipLaunchKernelGGL(bank_kernel<BANKS>, dim3(blocks), dim3(threads), 0, 0, out, st, 10);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(bank_kernel<BANKS>, dim3(blocks), dim3(threads), 0, 0, out, st, iters);
    CHECK(hipDeviceSynchronize());
    uint64_t* h = (uint64_t*)malloc(8 * waves);
    CHECK(hipMemcpy(h, st, 8 * waves, hipMemcpyDeviceToHost));
    double c = 0;
    for (int w = 0; w < waves; ++w) c += (double)h[w];
    c /= waves;
    printf("{\"bank_test\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_instr_per_wave\": %.3f}\n", name,
           threads / 256 > 0 ? threads / 256 : 1, c / (iters * 16.0 * 10));
    free(h);
    CHECK(hipFree(out));
    CHECK(hipFree(st));
}


// The real compression (schedule + 80 rounds, ~613 VALU) on register data,
// no memory traffic: isolates the VALU mix from the load path.
__global__ void compress_kernel(uint32_t* out, uint64_t* stamps, int iters) {
    uint32_t h[5];
    s1::init_state(h);
    uint32_t seed = threadIdx.x * 0x9e3779b9u + blockIdx.x;
    const uint64_t t0 = memtime(), q0 = realtime();
    for (int i = 0; i < iters; ++i) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = s1::bswap(seed + j * 0x01000193u + (uint32_t)i);
        s1::compress(h, w);
        seed ^= h[0];
    }
    const uint64_t t1 = memtime(), q1 = realtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
    if ((threadIdx.x & 63) == 0) {
        const int w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        stamps[2 * w] = t1 - t0;
        stamps[2 * w + 1] = q1 - q0;
    }
}

static void run_compress(int blocks, int threads) {
    const int iters = 400, waves = blocks * threads / 64;
    uint32_t* out;
    uint64_t* st;
    CHECK(hipMalloc(&out, 4 * blocks * threads));
    CHECK(hipMalloc(&st, 16 * waves));
    hipLaunchKernelGGL(compress_kernel, dim3(blocks), dim3(threads), 0, 0, out, st, 4);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(compress_kernel, dim3(blocks), dim3(threads), 0, 0, out, st, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipDeviceSynchronize());
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    uint64_t* h = (uint64_t*)malloc(16 * waves);
    CHECK(hipMemcpy(h, st, 16 * waves, hipMemcpyDeviceToHost));
    double c = 0, q = 0;
    for (int w = 0; w < waves; ++w) {
        c += (double)h[2 * w];
        q += (double)h[2 * w + 1];
    }
    c /= waves;
    q /= waves;
    const double lanes = (double)blocks * threads;
    printf("{\"compress_test\": \"%d x %d\", \"cycles_per_block_per_wave\": %.1f, "
           "\"clock_ghz\": %.3f, \"wave_ms\": %.3f, \"kernel_ms\": %.3f, \"GBps_equiv\": %.1f}\n",
           blocks, threads, c / iters, c / q * 0.1, q * 1e-5, ms,
           lanes * 64.0 * iters / (ms * 1e-3) / 1e9);
    free(h);
    CHECK(hipFree(out));
    CHECK(hipFree(st));
}


static void run_op_full(const char* name, void (*k)(uint32_t*, uint64_t*, int), int blocks, int threads) {
    const int iters = 1000, waves = blocks * threads / 64;
    uint32_t* out;
    uint64_t* st;
    CHECK(hipMalloc(&out, 4 * blocks * threads));
    CHECK(hipMalloc(&st, 8 * waves));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, st, 10);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, st, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipDeviceSynchronize());
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    uint64_t* h = (uint64_t*)malloc(8 * waves);
    CHECK(hipMemcpy(h, st, 8 * waves, hipMemcpyDeviceToHost));
    double c = 0;
    for (int w = 0; w < waves; ++w) c += (double)h[w];
    c /= waves;
    const double n = iters * 16.0 * 8;
    const double simd_instr = (double)waves / 1024.0 * n;  // wave-instructions per SIMD
    printf("{\"op_full\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_instr_per_wave\": %.3f, "
           "\"ns_per_simd_instr\": %.4f, \"clock_ghz\": %.3f}\n",
           name, waves / 1024, c / n, ms * 1e6 / simd_instr, c / (ms * 1e-3) / 1e9);
    free(h);
    CHECK(hipFree(out));
    CHECK(hipFree(st));
}

template <int MODE>
static void run(const char* name, int blocks, int threads, int instr_per_iter) {
    const int iters = 2000;
    uint32_t* out;
    uint64_t* st;
    const int waves = blocks * threads / 64;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * threads));
    CHECK(hipMalloc(&st, sizeof(uint64_t) * 2 * waves));
    hipLaunchKernelGGL(issue_kernel<MODE>, dim3(blocks), dim3(threads), 0, 0, out, st, 10);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(issue_kernel<MODE>, dim3(blocks), dim3(threads), 0, 0, out, st, iters);
    CHECK(hipDeviceSynchronize());
    uint64_t* h = (uint64_t*)malloc(sizeof(uint64_t) * 2 * waves);
    CHECK(hipMemcpy(h, st, sizeof(uint64_t) * 2 * waves, hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int w = 0; w < waves; ++w) {
        cyc += (double)h[2 * w];
        real += (double)h[2 * w + 1];
    }
    cyc /= waves;
    real /= waves;
    const double n_instr = (double)iters * 16 * instr_per_iter;
    printf("{\"test\": \"%s\", \"blocks\": %d, \"threads\": %d, \"cycles_per_instr\": %.3f, "
           "\"clock_ghz\": %.3f, \"ns_per_instr\": %.3f}\n",
           name, blocks, threads, cyc / n_instr, cyc / real * 0.1, real * 10.0 / n_instr);
    free(h);
    CHECK(hipFree(out));
    CHECK(hipFree(st));
}

int main() {
    run_op_full("v_add_u32", op_add, 256, 1024);
    run_op_full("v_xor_b32", op_xor, 256, 1024);
    run_op_full("v_add3_u32", op_add3, 256, 1024);
    run_op_full("v_bitop3_b32", op_bitop3, 256, 1024);
    run_op_full("v_alignbit_b32", op_alignbit, 256, 1024);
    run_op_full("v_alignbit s,s", op_align_ss, 256, 1024);
    run_op_full("v_perm_b32", op_perm, 256, 1024);
    run_op_full("v_bfi_b32", op_bfi, 256, 1024);
    run_op_full("v_lshl_add_u32", op_lshl_add, 256, 1024);
    run_op_full("v_add_u32 2/SIMD", op_add, 256, 512);
    run_op_full("v_add3_u32 2/SIMD", op_add3, 256, 512);
    run_op_full("v_alignbit 2/SIMD", op_alignbit, 256, 512);
    run_op_full("v_add_u32 8/SIMD", op_add, 512, 1024);
    run_op_full("v_add3_u32 8/SIMD", op_add3, 512, 1024);
    run_compress(1, 64);
    run_compress(256, 256);
    run_compress(256, 512);
    run_compress(256, 1024);
    run_compress(512, 1024);
    run_bank<0>("distinct_banks", 1, 64);
    run_bank<1>("same_bank", 1, 64);
    run_bank<0>("distinct_banks", 256, 256);
    run_bank<1>("same_bank", 256, 256);
    run_bank<0>("distinct_banks", 256, 512);
    run_bank<1>("same_bank", 256, 512);
    run_bank<0>("distinct_banks", 256, 1024);
    run_bank<1>("same_bank", 256, 1024);
    run_op("v_add_u32", op_add);
    run_op("v_add3_u32", op_add3);
    run_op("v_alignbit_b32", op_alignbit);
    run_op("v_bitop3_b32", op_bitop3);
    run_op("v_xor_b32", op_xor);
    run_op("v_bfi_b32", op_bfi);
    run_op("v_perm_b32", op_perm);
    run_op("v_lshl_add_u32", op_lshl_add);
    run_op("v_mov_b32_dpp", op_mov_dpp);
    run_op("s_nop", op_snop);
    run_op("alignbit s,s (dst r)", op_align_ss);
    run_op("alignbit s,t", op_align_st);
    run_op("alignbit r,s", op_align_rs);
    run_op("alignbit s,r", op_align_sr);
    run_op("v_lshlrev_b64", op_lshl64);
    run_op("v_pk_mov_b32", op_pkmov);
    run_op("add3 r,r,r,s", op_add3_same);
    // one wave alone on the chip / per CU; waves of one 256-thread block sit on 4 SIMDs
    run<0>("indep_add_1wave", 1, 64, 8);
    run<1>("dep_add3_1wave", 1, 64, 8);
    run<2>("round_1wave", 1, 64, 10);
    run<0>("indep_add_64waves_1perCU", 64, 64, 8);
    run<2>("round_64waves_1perCU", 64, 64, 10);
    // 8 waves per workgroup -> 2 waves on each SIMD of the CU
    run<0>("indep_add_2perSIMD", 64, 512, 8);
    run<2>("round_2perSIMD", 64, 512, 10);
    run<2>("round_1perSIMD_fullchip", 256, 256, 10);
    run<2>("round_2perSIMD_fullchip", 256, 512, 10);
    run<2>("round_4perSIMD_fullchip", 256, 1024, 10);
    return 0;
}
