#!/usr/bin/env python3
"""Diagnostic only: generate tools/producer_probe.hip, a single-wave replica
of the split kernel's producer (per 64-byte block: 16 v_perm byte swaps, the
64-word schedule expansion as v_bitop3 + v_xor + v_alignbit, W+K adds, and
20 ds_write_b128 of the block's W+K into the LDS ring) as explicit-register
inline asm, to find what the compiled producer's ~1878 cycles per block
(against ~1320 for its ~330 instructions at the 4-cycle issue floor) are
spent on.  Variants: no LDS writes; every write sourcing the same 4-VGPR
quad (what hipcc emits: `ds_write_b128 v96, v[32:35]` twenty times per block,
the next group's adds overwriting the quad the write still has to read)
vs rotating quads; the XOR temporary in a fixed bank vs bank-aware.

    python3 tools/gen_producer_probe.py && \
    hipcc --offload-arch=gfx950 -O3 tools/producer_probe.hip -o tools/producer_probe
"""
from __future__ import annotations

import os

HERE = os.path.dirname(os.path.abspath(__file__))
KS = [0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xCA62C1D6]
WBASE = 16     # W ring: W[t] in v(16 + t % 16)
MSG = 64       # fake message words v64..v79 (the loaded stage)
QBASE = 40     # data quads for the writes: v40.. (up to 6 quads -> v63)
ADDR = 8       # LDS address (lane * 16)
ADDR2 = 9      # v8 + (block slot / 2048-byte window) for ds_write2 (8-bit offsets)


def write_asm(kind: str, qb: int, off: int) -> list[str]:
    """One group's 16 bytes per lane (4 W+K words in v[qb:qb+3]) to LDS."""
    if kind == "b128":
        return [f"ds_write_b128 v{ADDR}, v[{qb}:{qb + 3}] offset:{off}"]
    if kind == "b64":
        return [f"ds_write_b64 v{ADDR}, v[{qb}:{qb + 1}] offset:{off}",
                f"ds_write_b64 v{ADDR}, v[{qb + 2}:{qb + 3}] offset:{off + 8}"]
    if kind == "write2_b64":  # offsets in units of 8 bytes, 8-bit each: keep them small
        return [f"ds_write2_b64 v{ADDR2}, v[{qb}:{qb + 1}], v[{qb + 2}:{qb + 3}] offset0:{(off % 2048) // 8} "
                f"offset1:{(off % 2048) // 8 + 1}"]
    if kind == "b32":
        return [f"ds_write_b32 v{ADDR}, v{qb + i} offset:{off + 4 * i}" for i in range(4)]
    if kind == "b96":
        return [f"ds_write_b96 v{ADDR}, v[{qb}:{qb + 2}] offset:{off}",
                f"ds_write_b32 v{ADDR}, v{qb + 3} offset:{off + 12}"]
    raise ValueError(kind)


def block_asm(blk: int, writes: bool, quads: int, tmp_mode: str, kind: str = "b128",
              burst: bool = False) -> list[str]:
    out = []
    pending = []
    slot = (blk % 2) * 20480

    def q(g):  # quad register base for write group g
        return QBASE + 4 * (g % quads)

    def tmp(t):
        return 4 + ((t + 3) % 4) if tmp_mode == "bank" else 4

    # W[0..15]: byte swap of the message words (into the W ring) and W+K
    for j in range(16):
        out.append(f"v_perm_b32 v{WBASE + j}, 0, v{MSG + j}, s10")
    for t in range(80):
        if t >= 16:
            a, b, c, d = (WBASE + (t - 3) % 16, WBASE + (t - 8) % 16,
                          WBASE + (t - 14) % 16, WBASE + t % 16)
            x = tmp(t)
            out.append(f"v_bitop3_b32 v{x}, v{a}, v{b}, v{c} bitop3:0x96")
            out.append(f"v_xor_b32 v{x}, v{d}, v{x}")
            out.append(f"v_alignbit_b32 v{d}, v{x}, v{x}, 31")
        g = t // 4
        out.append(f"v_add_u32 v{q(g) + t % 4}, s{20 + t // 20}, v{WBASE + t % 16}")
        if t % 4 == 3 and writes:
            w = write_asm(kind, q(g), slot + g * 1024)
            (pending if burst else out).extend(w)
    return out + pending


def kernel(name: str, writes: bool, quads: int, tmp_mode: str, kind: str = "b128",
           burst: bool = False, nblk: int = 8) -> str:
    body = []
    for blk in range(nblk):
        body += block_asm(blk, writes, quads, tmp_mode, kind, burst)
    body.append("s_waitcnt lgkmcnt(0)")
    asm = "\\n".join(body)
    msg_movs = " ".join(f'"v_mov_b32 v{MSG + j}, {0x01020304 * (j + 1) & 0xffffffff}\\n"' for j in range(16))
    msg_clob = ", ".join(f'"v{MSG + j}"' for j in range(16))
    regs = list(range(4, 8)) + list(range(WBASE, WBASE + 16)) + list(range(QBASE, QBASE + 24))
    clobbers = ", ".join(f'"v{i}"' for i in regs)
    return f'''
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void {name}(uint64_t* st) {{
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 20480];
    for (int i = threadIdx.x; i < 2 * 20480 / 4; i += 64) reinterpret_cast<uint32_t*>(lds)[i] = 0;
    __syncthreads();
    const uint32_t a = (uint32_t)(uintptr_t)lds + threadIdx.x * 16;
    uint64_t t0, t1, q0, q1;
    asm volatile("v_mov_b32 v{ADDR}, %0\\n v_mov_b32 v{ADDR2}, %0\\n s_mov_b32 s10, 0x10203\\n"
                 "s_mov_b32 s20, 0x5a827999\\n s_mov_b32 s21, 0x6ed9eba1\\n"
                 "s_mov_b32 s22, 0x8f1bbcdc\\n s_mov_b32 s23, 0xca62c1d6\\n"
                 {msg_movs}
                 :: "v"(a) : "v{ADDR}", "v{ADDR2}", "s10", "s20", "s21", "s22", "s23",
                 {msg_clob});
    asm volatile("s_memtime %0\\n s_memrealtime %1\\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(q0));
    asm volatile("{asm}" ::: {clobbers}, "memory");
    asm volatile("s_memtime %0\\n s_memrealtime %1\\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(q1));
    if (threadIdx.x == 0) {{ st[0] = t1 - t0; st[1] = q1 - q0; st[2] = {nblk}; }}
}}
'''


VARIANTS = [
    ("p_nowrite_bank", False, 1, "bank"),
    ("p_nowrite_fixed", False, 1, "fixed"),
    ("p_samequad_fixed", True, 1, "fixed"),
    ("p_samequad_bank", True, 1, "bank"),
    ("p_2quads_bank", True, 2, "bank"),
    ("p_3quads_bank", True, 3, "bank"),
    ("p_5quads_bank", True, 5, "bank"),
    ("p_b64", True, 2, "bank", "b64"),
    ("p_b32", True, 2, "bank", "b32"),
    ("p_write2_b64", True, 2, "bank", "write2_b64"),
    ("p_b96_b32", True, 2, "bank", "b96"),
    ("p_b128_burst_end", True, 6, "bank", "b128", True),
]
NWR = {"b128": 20, "b64": 40, "b32": 80, "write2_b64": 20, "b96": 40}


def main():
    parts = ['''// producer_probe.hip -- GENERATED by tools/gen_producer_probe.py (diagnostic only).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \\
    fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
''']
    for v in VARIANTS:
        parts.append(kernel(*v))
    parts.append('''
static void run(const char* name, void (*k)(uint64_t*), int writes) {
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
    const double instr = 288.0 + writes;
    printf("{\\"producer_probe\\": \\"%s\\", \\"cycles_per_block\\": %.1f, \\"ns_per_block\\": %.1f, "
           "\\"instr_per_block\\": %.0f, \\"cycles_per_instr\\": %.3f, \\"clock_ghz\\": %.3f}\\n", name,
           (double)best_c / nb, best_q * 10.0 / nb, instr, (double)best_c / nb / instr,
           best_c / (best_q * 10.0));
    CHECK(hipFree(st));
}
int main() {
''')
    for name, writes, _q, _t, *rest in VARIANTS:
        nw = NWR[rest[0] if rest else "b128"] if writes else 0
        parts.append(f'    run("{name}", {name}, {nw});\n')
    parts.append("    return 0;\n}\n")
    with open(os.path.join(HERE, "producer_probe.hip"), "w") as f:
        f.write("".join(parts))


if __name__ == "__main__":
    main()
