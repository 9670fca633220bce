#!/bin/bash
# r04ac: level-0/1 lookup tables back at 4 slots per entry (sampled levels 2 per kept snapshot): C2, C4,
# C3 against the round-start library, same box; the sampled levels' multiplier
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04ac
mkdir -p "$OUT"
run() {  # tag lib config env...
  local tag=$1 lib=$2 cfg=$3; shift 3
  env "$@" FAC_DIAGNOSTICS=1 FAC_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-fresh-diag > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));g=d['diagnostics'];print('$tag', round(d['ms_per_step'],2), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
}
for c in c2 c4 c3; do
  run ${c}_r04a $L/libfac_r04a.so $c X=0
  run ${c}_head $L/libfac.so $c X=0
  run ${c}_m2_4 $L/libfac.so $c FAC_RC_CT_MULT2=4
done
run c2_m_8 $L/libfac.so c2 FAC_RC_CT_MULT=8
