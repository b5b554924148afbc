#!/bin/bash
# Per-kernel VGPR / SGPR / scratch / LDS of one gfx950 object (librmc build):
#   tools/kernel_resources.sh raft.tla_amd/_obj/rmc_kernels_3_4.o [name-regex]
set -e
obj=$1; pat=${2:-.}
d=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$d/fat.bin "$obj"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$d/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$d/co.elf
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $d/co.elf | python3 -c '
import sys, re
txt = sys.stdin.read()
pat = re.compile(sys.argv[1])
for blk in txt.split("- .agpr_count")[1:]:
    def g(k):
        m = re.search(r"\.%s:\s+(\S+)" % k, blk)
        return m.group(1) if m else "?"
    name = g("name")
    if not pat.search(name): continue
    v, s_, p_, l_ = g("vgpr_count"), g("sgpr_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size")
    ss = g("sgpr_spill_count")
    print("%4s vgpr %4s sgpr %4s sgpr-spill %5s scratch %6s lds  %s" % (v, s_, ss, p_, l_, name[:150]))
' "$pat"
rm -rf $d
