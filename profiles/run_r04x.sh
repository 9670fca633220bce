#!/bin/bash
# r04x: text chars from the window registers (no per-state text loads) vs not (libfac_nort.so):
# prefix-cache parity subset, then C3 same box; fresh words
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04x
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane_serial or dedup_free or differential_random or golden or halo or shard" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in nort head nort head; do
  lib=$L/libfac.so; [ $v = nort ] && lib=$L/libfac_nort.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/b_$v.json'));g=d['diagnostics'];print('$v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
done
for v in nort head; do
  lib=$L/libfac.so; [ $v = nort ] && lib=$L/libfac_nort.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag --vocab 0 --steps 3 > "$OUT/f_$v.json" 2> "$OUT/f_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/f_$v.json'));g=d['diagnostics'];print('fresh $v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1), g['matches_per_step'])"
done
