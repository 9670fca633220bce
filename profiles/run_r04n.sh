#!/bin/bash
# r04n: sampled-level policy under the fixed builds (vocabulary and fresh words), against the round-start library
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04n
mkdir -p "$OUT"
for v in r04a head; do
  lib=$L/libfac.so; [ $v = r04a ] && lib=$L/libfac_r04a.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/b_$v.json'));g=d['diagnostics'];print('$v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
done
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04n_v "X=0" "FAC_RC_T2=3" "FAC_RC_LEVELS=5,7" "FAC_RC_LEVELS=5,6" "FAC_RC_LEVELS=5,6,7,8"
BENCH_ARGS="--vocab 0 --no-fresh-diag" bash profiles/ab_knobs.sh r04n_f "X=0" "FAC_RC_K2=0" "FAC_RC_T2=3" "FAC_RC_LEVELS=5" "FAC_LIVE_NQMAX=160"
