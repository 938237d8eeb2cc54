#!/usr/bin/env python3
"""Diagnostic only: generate tools/consumer_probe.hip, a single-wave replica
of the split kernel's consumer (80 SHA-1 rounds per 64-byte block on W+K
held in VGPRs, the next block's schedule streamed from LDS into the other
register set) as explicit-register inline asm, in several schedules of the
20 ds_read_b128 per block.  Each variant runs 8 blocks straight-line per
timed pass; the probe prints cycles per block next to the 409-VALU issue
floor (4 cycles each), to find how much of the consumer's measured ~1990
cycles per block is the schedule hand-off and which placement hides it.

    python3 tools/gen_consumer_probe.py && \
    hipcc --offload-arch=gfx950 -O3 tools/consumer_probe.hip -o tools/consumer_probe
"""
from __future__ import annotations

import os

HERE = os.path.dirname(os.path.abspath(__file__))
K = ["s20", "s21", "s22", "s23"]
ST = [0, 1, 2, 3, 4]          # v0..v4: working state a..e (rotating)
R5, F, X = 5, 6, 7            # temporaries
WSET = [8, 88]                # two 80-register W sets
ADDR = 170                    # LDS address (lane * 16)
H = [180, 181, 182, 183, 184]  # chaining value


def round_asm(t: int, wbase: int, fop: str, order: str = "O1", wk: bool = False) -> list[str]:
    ia = (5 - t % 5) % 5
    ib, ic, id_, ie = (ia + 1) % 5, (ia + 2) % 5, (ia + 3) % 5, (ia + 4) % 5
    a, b, c, d, e = (f"v{ST[i]}" for i in (ia, ib, ic, id_, ie))
    k = K[t // 20]
    if t < 20:
        f = f"v_bfi_b32 v{F}, {b}, {c}, {d}" if fop == "bfi" else \
            f"v_bitop3_b32 v{F}, {b}, {c}, {d} bitop3:0xca"
    elif t < 40 or t >= 60:
        f = f"v_bitop3_b32 v{F}, {b}, {c}, {d} bitop3:0x96"
    else:
        f = f"v_bitop3_b32 v{F}, {b}, {c}, {d} bitop3:0xe8"
    ins = {
        "r5": f"v_alignbit_b32 v{R5}, {a}, {a}, 27",
        "f": f,
        "x": (f"v_add_u32 v{X}, {e}, v{wbase + t}" if wk is True else
              f"v_add3_u32 v{X}, {e}, v{wbase + t}, v{171 + t // 20}" if wk == "vk" else
              f"v_add3_u32 v{X}, {e}, v{wbase + t}, {k}"),
        "t": f"v_add3_u32 {e}, v{R5}, v{F}, v{X}",
        "r30": f"v_alignbit_b32 {b}, {b}, {b}, 2",
    }
    seq = {"O1": ["r5", "f", "x", "t", "r30"], "O2": ["x", "f", "r5", "r30", "t"],
           "O3": ["x", "r5", "f", "r30", "t"], "O4": ["f", "x", "r5", "t", "r30"],
           "O5": ["r5", "x", "f", "t", "r30"], "O6": ["x", "r5", "f", "t", "r30"]}[order]
    return [ins[n] for n in seq]


def block_asm(blk: int, sched: str, fop: str, order: str = "O1", wk: bool = False) -> list[str]:
    cur, nxt = WSET[blk % 2], WSET[(blk + 1) % 2]
    slot = (blk + 1) % 2  # ds offsets are 16-bit: two 20 KiB slots
    reads = [f"ds_read_b128 v[{nxt + 4 * q}:{nxt + 4 * q + 3}], v{ADDR} offset:{slot * 20480 + q * 1024}"
             for q in range(20)]
    # where each of the 20 reads goes: before round r
    if sched == "burst5":        # the compiler's placement: 5 before rounds 0/20/40/60
        at = {0: reads[0:5], 20: reads[5:10], 40: reads[10:15], 60: reads[15:20]}
    elif sched == "burst10":
        at = {0: reads[0:10], 40: reads[10:20]}
    elif sched == "spread":      # one read every 4 rounds
        at = {4 * q: [reads[q]] for q in range(20)}
    elif sched == "early15":     # 15 at the block start, 5 at round 40
        at = {0: reads[0:15], 40: reads[15:20]}
    elif sched == "none":
        at = {}
    else:
        raise ValueError(sched)
    out = []
    # set `cur` was filled during the previous block: all of those reads must
    # have landed before round 0 uses it; the reads issued just now may not
    first = at.get(0, [])
    out += first
    if sched != "none":
        out.append(f"s_waitcnt lgkmcnt({min(len(first), 15)})")
    for h, s in zip(H, ST):
        pass
    for t in range(80):
        if t and t in at:
            out += at[t]
        out += round_asm(t, cur, fop, order, wk)
    # feed-forward (state registers hold the block's result)
    for i in range(5):
        out.append(f"v_add_u32 v{H[i]}, v{H[i]}, v{ST[i]}")
    for i in range(5):
        out.append(f"v_mov_b32 v{ST[i]}, v{H[i]}")
    return out


def kernel(name: str, sched: str, fop: str, order: str = "O1", wk: bool = False, nblk: int = 8) -> str:
    body = []
    for blk in range(nblk):
        body += block_asm(blk, sched, fop, order, wk)
    body.append("s_waitcnt lgkmcnt(0)")
    asm = "\\n".join(body)
    clobbers = ", ".join(f'"v{i}"' for i in list(range(0, 168)) + H)
    return f'''
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void {name}(uint64_t* st) {{
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 20480];
    for (int i = threadIdx.x; i < 2 * 20480 / 4; i += 64) reinterpret_cast<uint32_t*>(lds)[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t a = (uint32_t)(uintptr_t)lds + threadIdx.x * 16;
    uint64_t t0, t1, q0, q1;
    asm volatile("v_mov_b32 v{ADDR}, %0\\n s_mov_b32 s20, 0x5a827999\\n s_mov_b32 s21, 0x6ed9eba1\\n"
                 "s_mov_b32 s22, 0x8f1bbcdc\\n s_mov_b32 s23, 0xca62c1d6\\n"
                 "v_mov_b32 v0, 1\\n v_mov_b32 v1, 2\\n v_mov_b32 v2, 3\\n v_mov_b32 v3, 4\\n v_mov_b32 v4, 5\\n"
                 "v_mov_b32 v180, 1\\n v_mov_b32 v181, 2\\n v_mov_b32 v182, 3\\n v_mov_b32 v183, 4\\n v_mov_b32 v184, 5\\n"
                 "v_mov_b32 v171, 0x5a827999\\n v_mov_b32 v172, 0x6ed9eba1\\n v_mov_b32 v173, 0x8f1bbcdc\\n v_mov_b32 v174, 0xca62c1d6"
                 :: "v"(a) : "v{ADDR}", "s20", "s21", "s22", "s23", "v0", "v1", "v2", "v3", "v4",
                   "v180", "v181", "v182", "v183", "v184", "v171", "v172", "v173", "v174");
    asm volatile("s_memtime %0\\n s_memrealtime %1\\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(q0));
    asm volatile("{asm}" ::: {clobbers}, "memory");
    asm volatile("s_memtime %0\\n s_memrealtime %1\\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(q1));
    if (threadIdx.x == 0) {{ st[0] = t1 - t0; st[1] = q1 - q0; st[2] = {nblk}; }}
}}
'''


VARIANTS = []
for order in ("O1", "O2"):
    for wk in (False, True, "vk"):
        for sched in ("none", "burst5", "burst10"):
            tag = {False: "sk", True: "wk", "vk": "vk"}[wk]
            VARIANTS.append((f"c_{order}_{tag}_{sched}", sched, "bfi", order, wk))


def main():
    parts = ['''// consumer_probe.hip -- GENERATED by tools/gen_consumer_probe.py (diagnostic only).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \\
    fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
''']
    for name, sched, fop, order, wk in VARIANTS:
        parts.append(kernel(name, sched, fop, order, wk))
    parts.append('''
static void run(const char* name, void (*k)(uint64_t*)) {
    uint64_t* st;
    CHECK(hipMalloc(&st, 32));
    uint64_t best_c = ~0ull, best_q = 0, nb = 1;
    for (int rep = 0; rep < 6; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, st);
        CHECK(hipDeviceSynchronize());
        uint64_t h[3];
        CHECK(hipMemcpy(h, st, 24, hipMemcpyDeviceToHost));
        if (rep > 0 && h[0] < best_c) { best_c = h[0]; best_q = h[1]; nb = h[2]; }
    }
    printf("{\\"consumer_probe\\": \\"%s\\", \\"cycles_per_block\\": %.1f, \\"ns_per_block\\": %.1f, "
           "\\"cycles_per_valu\\": %.3f, \\"clock_ghz\\": %.3f}\\n", name, (double)best_c / nb,
           best_q * 10.0 / nb, (double)best_c / nb / 410.0, best_c / (best_q * 10.0));
    CHECK(hipFree(st));
}
int main() {
''')
    for name, *_ in VARIANTS:
        parts.append(f'    run("{name}", {name});\n')
    parts.append("    return 0;\n}\n")
    with open(os.path.join(HERE, "consumer_probe.hip"), "w") as f:
        f.write("".join(parts))


if __name__ == "__main__":
    main()
