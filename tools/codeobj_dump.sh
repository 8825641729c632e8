#!/bin/bash
# Device code of every object of the library build, as disassembled text with
# addresses stripped: tools/codeobj_dump.sh <build dir> <out dir>.  Two dumps
# diff equal when a source change (e.g. deleting a disabled variant) leaves
# the product kernels' machine code unchanged.
B=${1:-dav1d-mirror_amd/build}
O=${2:-/tmp/codeobj}
mkdir -p "$O"
L=/opt/rocm/lib/llvm/bin
for f in "$B"/*.o; do
    n=$(basename "$f" .o)
    [ "$n" = stamp ] && continue
    # (an output file is named: without one llvm-objcopy rewrites the input)
    "$L/llvm-objcopy" --dump-section .hip_fatbin="$O/$n.fatbin" "$f" "$O/$n.copy.o" 2>/dev/null || continue
    rm -f "$O/$n.copy.o"
    "$L/clang-offload-bundler" --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$O/$n.fatbin" \
        --output="$O/$n.gfx950.o" --unbundle 2>/dev/null || continue
    rm -f "$O/$n.fatbin"
    "$L/llvm-objdump" -d --no-show-raw-insn --no-leading-addr "$O/$n.gfx950.o" 2>/dev/null \
        | sed -e 's/<[^>]*+0x[0-9a-f]*>//g' -e 's/0x[0-9a-f]\{6,\}//g' > "$O/$n.s"
    rm -f "$O/$n.gfx950.o"
done
