#!/bin/bash
# r04ab: C2 regression bisect over round-4 commits (libraries built from each commit, same box), the
# entry cap; C3 with the 168-VGPR small build variant (libfac_small3.so)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04ab
mkdir -p "$OUT"
run() {  # tag lib config env...
  local tag=$1 lib=$2 cfg=$3; shift 3
  env "$@" FAC_DIAGNOSTICS=1 FAC_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-fresh-diag > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));g=d['diagnostics'];print('$tag', round(d['ms_per_step'],2), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
}
run c2_r04a $L/libfac_r04a.so c2 X=0
for c in 683c90c 5872f0b ad595f5 1219ea5; do run c2_$c $L/libfac_b$c.so c2 X=0; done
run c2_head $L/libfac.so c2 X=0
run c2_head_e16 $L/libfac.so c2 FAC_RC_ENTRIES=16777216
run c2_head_deep $L/libfac.so c2 FAC_RC_DEEPEST=1
run c2_r04a_2 $L/libfac_r04a.so c2 X=0
run c3_small3 $L/libfac_small3.so c3 FAC_BUILD_SMALL=1
# fresh words: early spill of long resumed queues, spills to the <256,256> variant first
for kv in "X=0" "FAC_LIVE_NQMAX=100" "FAC_LIVE_NQMAX=116" "FAC_SPILL_SMALL=1"; do
  env $kv FAC_DIAGNOSTICS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag --vocab 0 --steps 2 > "$OUT/f.json" 2> "$OUT/f.err"
  python3 -c "import json;d=json.load(open('$OUT/f.json'));g=d['diagnostics'];print('fresh $kv', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
done
