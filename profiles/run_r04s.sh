#!/bin/bash
# r04s: count-table slots with the count in the key word (then: representative written at the second sighting): prefix-cache
# library vs HEAD, a timeline, the sampled counts' grid
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04s
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane_serial or dedup_free or differential_random or golden" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in r04a head r04a head; do
  lib=$L/libfac.so; [ $v = r04a ] && lib=$L/libfac_r04a.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/b_$v.json'));g=d['diagnostics'];print('$v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
done
bash profiles/ab_knobs.sh r04s_k "FAC_RC_STRIDE2=4" "FAC_RC_STRIDE2=4 FAC_RC_T2=2"
bash profiles/timeline_c3.sh r04s "X=0" | grep -E "==|rc_count|rc_build|lookup|window_kernel"
