#!/bin/bash
# r04o: snapshot prefetch: prefix-cache parity subset, then round-start library vs HEAD (vocabulary, fresh)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04o
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane_serial or dedup_free or differential_random or golden" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in r04a head r04a head; do
  lib=$L/libfac.so; [ $v = r04a ] && lib=$L/libfac_r04a.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/b_$v.json'));g=d['diagnostics'];print('$v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
done
FAC_LIB=$L/libfac.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag --vocab 0 --steps 3 > "$OUT/f_head.json" 2> "$OUT/f_head.err"
python3 -c "import json;d=json.load(open('$OUT/f_head.json'));g=d['diagnostics'];print('fresh head', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
