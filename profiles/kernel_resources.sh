#!/bin/bash
# Per-kernel register / scratch use of a built object (gfx950 code object notes):
#   bash profiles/kernel_resources.sh fuzzy-aho-corasick-rs_amd/csrc/build/search_kernels.o [name-regex]
set -eo pipefail
OBJ=${1:?object}
PAT=${2:-.}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin="$T/fb" "$OBJ"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --input="$T/fb" --output="$T/co" --unbundle \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/co" | python3 -c '
import re, sys
pat = re.compile(sys.argv[1])
txt = sys.stdin.read()
for blk in txt.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or not pat.search(name.group(1)):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    vals = [g(k) for k in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size", "group_segment_fixed_size")]
    print("%-90s vgpr %s sgpr %s vspill %s sspill %s scratch %s lds %s" % ((name.group(1)[:90],) + tuple(vals)))
' "$PAT"
rm -rf "$T"
