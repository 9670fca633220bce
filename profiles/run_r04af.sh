#!/bin/bash
# r04af: dedup-free pass compiled for 3 waves/SIMD (149 VGPRs, no spills; libfac_lw3.so) vs 4 (128 VGPRs,
# 16 spilled), C3 and fresh C3, same box
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04af
mkdir -p "$OUT"
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag "$@" > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));g=d['diagnostics'];print('$tag', round(d['ms_per_step'],2), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
}
run head $L/libfac.so
run lw3 $L/libfac_lw3.so
run head_b $L/libfac.so
run lw3_b $L/libfac_lw3.so
run fresh_head $L/libfac.so --vocab 0 --steps 2
run fresh_lw3 $L/libfac_lw3.so --vocab 0 --steps 2
