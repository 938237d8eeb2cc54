#!/bin/bash
# Disassemble the gfx950 code object inside a hipcc object file:
#   tools/dump_isa.sh build/sha1_kernels.o out.s
set -e
B=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fat.bin "$1"
$B/clang-offload-bundler --unbundle --type=o --input=$tmp/fat.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/k.co
$B/llvm-objdump -d $tmp/k.co > "$2"
rm -rf $tmp
