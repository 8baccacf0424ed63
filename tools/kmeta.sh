# registers, spills and static LDS of the search kernels in a built fsclg.o: bash tools/kmeta.sh <fsclg.o>
set -e
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | python3 -c '
import sys, re
txt = sys.stdin.read()
for blk in re.split(r"\n\s+- \.", txt):
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or "search_maxpos" not in m.group(1): continue
    g = lambda k: (re.search(k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print(m.group(1)[:60], "vgpr", g(r"\.vgpr_count"), "spill", g(r"\.vgpr_spill_count"), "lds", g(r"\.group_segment_fixed_size"))
'
rm -rf $T
