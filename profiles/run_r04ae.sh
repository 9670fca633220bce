#!/bin/bash
# r04ae: count-table slots grouped by parent key (siblings adjacent in entry order, so a build wave
# resumes consecutive keys from one parent snapshot): blocks of 64 (HEAD) vs 16 vs none (libfac_blk1.so)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04ae
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane_serial or dedup_free or differential_random or golden" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
run() {  # tag lib config env...
  local tag=$1 lib=$2 cfg=$3; shift 3
  env "$@" FAC_DIAGNOSTICS=1 FAC_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-fresh-diag > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  python3 -c "import json;d=json.load(open('$OUT/$tag.json'));g=d['diagnostics'];print('$tag', round(d['ms_per_step'],2), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
}
for c in c3 c2; do
  run ${c}_blk1 $L/libfac_blk1.so $c X=0
  run ${c}_blk64 $L/libfac.so $c X=0
  run ${c}_blk16 $L/libfac_blk16.so $c X=0
  run ${c}_blk1b $L/libfac_blk1.so $c X=0
  run ${c}_blk64b $L/libfac.so $c X=0
done
bash profiles/timeline_c3.sh r04ae "X=0" | grep -E "==|rc_count|rc_build|lookup|window_kernel"
