#!/usr/bin/env python3
"""Per-block instruction mix of each kernel's hot loop, read from the gfx950
assembly that `make -C congestion-control-with-bittorren_amd isa` writes.

For every loop (hipcc's "Loop Header" labels up to the branch back to them)
of the named kernels the instructions are counted by opcode and divided by
the number of 64-byte blocks one trip covers (80 rounds per block: the trip's
byte swaps / 16 in the fused kernel, its rotates / 160 in the rounds-only
consumer).  The result feeds the
issue-floor models in bench.py:

  * split consumer: instructions per block one wave issues (serial floor at
    one instruction per 4 cycles per wave);
  * fused: VALU cycles per block on one SIMD, full-rate ops at 2 cycles per
    wave64 instruction and half-rate ops (alignbit, add3, perm, bfi, lshl_add)
    at 4 (SIMD-32, MI355X_MICROARCH.md "Wave scheduling"; the half-rate class
    measured in tools/microbench.hip, profiles/microbench_ops_r01.json).

usage: tools/isa_mix.py [asm.s] > profiles/isa_mix_rNN.json
"""
import collections
import json
import re
import sys

ASM = sys.argv[1] if len(sys.argv) > 1 else \
    "congestion-control-with-bittorren_amd/build/sha1_kernels-hip-amdgcn-amd-amdhsa-gfx950.s"
HALF_RATE = {"v_alignbit_b32", "v_add3_u32", "v_perm_b32", "v_bfi_b32", "v_lshl_add_u32",
             "v_alignbyte_b32", "v_lshl_or_b32", "v_and_or_b32", "v_xad_u32"}
KERNELS = {
    "fused": "_Z17sha1_fused_kernel9BatchArgs",
    # <= 1 group of 64 chunks per CU: 4-block units, two producers
    "split_u4_2prod": "_Z17sha1_split_kernelILi4ELi1ELi8269ELi2EEv9BatchArgs",
    # <= 2 groups per CU: 8-wave workgroup, 2-block units (split_unit case 11)
    "split_u2_8wave": "_Z17sha1_split_kernelILi2ELi2ELi8581ELi2EEv9BatchArgs",
}


def functions(lines):
    out, cur = {}, None
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            cur = m.group(1)
            out[cur] = [i, None]
        if cur and l.startswith(".Lfunc_end"):
            out[cur][1] = i
            cur = None
    return out


def loops(lines, lo, hi):
    for i in range(lo, hi):
        m = re.match(r"^(\.LBB\d+_\d+):", lines[i])
        if not m or "Loop Header" not in lines[i] + lines[i + 1]:
            continue
        lab = m.group(1)
        for j in range(i + 1, hi):
            if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\s*$", lines[j]):
                body = [x.strip() for x in lines[i + 1:j + 1]]
                body = [x for x in body if x and not x.startswith((";", ".")) and not re.match(r"^\S+:", x)]
                yield lab, collections.Counter(x.split()[0].replace("_e32", "").replace("_e64", "")
                                               for x in body)
                break


def main():
    lines = open(ASM).read().split("\n")
    fns = functions(lines)
    res = {"source": ASM.split("/")[-1], "half_rate_ops": sorted(HALF_RATE), "kernels": {}}
    for name, sym in KERNELS.items():
        lo, hi = fns[sym]
        # the steady-state bulk loop: among loops that run whole rounds
        # (>= 160 alignbit = 2 rotates x 80 rounds per block), the one with
        # the fewest instructions per block (the masked tail loops carry
        # extra v_cndmask commits)
        best = None
        for lab, c in loops(lines, lo, hi):
            if c.get("v_alignbit_b32", 0) < 160:
                continue
            blocks = c["v_perm_b32"] / 16 if name == "fused" else c["v_alignbit_b32"] / 160
            if best is None or sum(c.values()) / blocks < sum(best[1].values()) / best[2]:
                best = (lab, c, blocks)
        lab, c, blocks = best
        per = {k: v / blocks for k, v in sorted(c.items(), key=lambda kv: -kv[1])}
        valu = {k: v for k, v in per.items() if k.startswith("v_")}
        half = sum(v for k, v in valu.items() if k in HALF_RATE)
        full = sum(valu.values()) - half
        res["kernels"][name] = {
            "symbol": sym, "loop": lab, "blocks_per_trip": blocks,
            "per_block": {k: round(v, 2) for k, v in per.items()},
            "instructions_per_block": round(sum(per.values()), 2),
            "valu_per_block": round(sum(valu.values()), 2),
            "valu_half_rate_per_block": round(half, 2), "valu_full_rate_per_block": round(full, 2),
            "simd_cycles_per_wave_block": round(4 * half + 2 * full, 1),
        }
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
