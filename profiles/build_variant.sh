#!/bin/bash
# Compile-time A/B variants of the search kernels (run here, on the CPU, before a gpurun call):
#   bash profiles/build_variant.sh NAME "-DMACRO=value ..."
# builds fuzzy_aho_corasick/_lib/libfac_NAME.so from the current sources with the extra flags on
# search_kernels.hip (the other objects from the regular build); select it with FAC_LIB=<that path>.
set -eo pipefail
NAME=${1:?name}
FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/fuzzy-aho-corasick-rs_amd/csrc
make -s -C "$C" >/dev/null
mkdir -p "$C/build/var"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
  --offload-arch=gfx950 -fno-gpu-flush-denormals-to-zero -fno-gpu-rdc $FLAGS -c -o "$C/build/var/sk_$NAME.o" "$C/search_kernels.hip"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib/libfac_$NAME.so" \
  "$C/build/unicode.o" "$C/build/builder.o" "$C/build/api.o" "$C/build/stream.o" "$C/build/var/sk_$NAME.o" \
  "$C/build/rank_kernels.o" "$C/build/stage_kernels.o"
echo "built libfac_$NAME.so"
