#!/bin/bash
# r04aa: C2 / C4 against the round-start library (same box) and the round-4 knobs that touch them (FAC_DIAGNOSTICS=1: knobs apply);
# C3 with the small build variant at 168 VGPRs (libfac_small3.so)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04aa
mkdir -p "$OUT"
run() {  # tag lib config env...
  local tag=$1 lib=$2 cfg=$3; shift 3
  env "$@" FAC_DIAGNOSTICS=1 FAC_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-fresh-diag > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));g=d['diagnostics'];print('$tag', round(d['ms_per_step'],2), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
}
for c in c2 c4; do
  run ${c}_r04a $L/libfac_r04a.so $c X=0
  run ${c}_head $L/libfac.so $c X=0
  run ${c}_e16 $L/libfac.so $c FAC_RC_ENTRIES=16777216
  run ${c}_ct $L/libfac.so $c FAC_RC_CT_ENTRIES=1
  run ${c}_deep $L/libfac.so $c FAC_RC_DEEPEST=1
  run ${c}_r04a2 $L/libfac_r04a.so $c X=0
done
run c3_head $L/libfac.so c3 X=0
run c3_small3 $L/libfac_small3.so c3 FAC_BUILD_SMALL=1
run c3_small4 $L/libfac.so c3 FAC_BUILD_SMALL=1
