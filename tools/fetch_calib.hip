// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950
// against reads and writes of a known byte count, in the access patterns the
// SHA-1 kernels use, so that the traffic figures in profiles/traffic_*.json
// rest on a measurement committed here rather than on a quoted factor.
//
//   stream_read  coalesced: consecutive lanes read consecutive 16-byte pieces
//                (global_load_dwordx4), XOR-folded, one dword per thread out.
//   lane_read    the hash kernels' pattern: lane i owns chunk i (chunks
//                chunk_len apart), 16-byte loads, 128 contiguous bytes per
//                lane per stage (8 x dwordx4), 20 bytes written per chunk.
//
// Each kernel is launched REPS times on its own.  Run under separate
// rocprofv3 passes (tools/fetch_calib.sh) and divide the per-dispatch
// counter by the byte counts this program prints (tools/fetch_calib_summary.py).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ __launch_bounds__(256) void stream_read(const uint4* __restrict__ src, size_t n16,
                                                   uint32_t* __restrict__ out) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (size_t i = tid; i < n16; i += stride) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[tid] = acc;
}

__global__ __launch_bounds__(64) void lane_read(const uint8_t* __restrict__ base, uint32_t chunk_len,
                                                uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const uint4* p = reinterpret_cast<const uint4*>(base + (size_t)c * chunk_len);
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0;
    for (uint32_t s = 0; s < chunk_len / 128; ++s) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = p[8 * s + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            a0 ^= v[j].x;
            a1 += v[j].y;
            a2 ^= v[j].z;
            a3 += v[j].w;
            a4 ^= v[j].x + v[j].w;
        }
    }
    uint32_t* o = out + 5ull * c;  // 20 bytes per chunk, like a digest
    o[0] = a0;
    o[1] = a1;
    o[2] = a2;
    o[3] = a3;
    o[4] = a4;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 4096;  // chunks
    const uint32_t L = 524288;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    const size_t bytes = (size_t)n * L;
    uint8_t* buf = nullptr;
    uint32_t* out = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    const int sgrid = 256 * 8, sblock = 256;  // 8 workgroups per CU
    const size_t out_words = (size_t)sgrid * sblock > 5ull * n ? (size_t)sgrid * sblock : 5ull * n;
    CHECK(hipMalloc(&out, out_words * 4));
    CHECK(hipMemset(buf, 0x5a, bytes));
    CHECK(hipDeviceSynchronize());
    for (int r = 0; r < reps; ++r) {
        stream_read<<<sgrid, sblock>>>(reinterpret_cast<const uint4*>(buf), bytes / 16, out);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
    }
    for (int r = 0; r < reps; ++r) {
        lane_read<<<(n + 63) / 64, 64>>>(buf, L, n, out);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
    }
    printf("{\"chunks\": %u, \"chunk_bytes\": %u, \"reps\": %d, "
           "\"stream_read\": {\"read_bytes\": %zu, \"write_bytes\": %zu}, "
           "\"lane_read\": {\"read_bytes\": %zu, \"write_bytes\": %zu}}\n",
           n, L, reps, bytes, (size_t)sgrid * sblock * 4, bytes, (size_t)n * 20);
    CHECK(hipFree(out));
    CHECK(hipFree(buf));
    return 0;
}
