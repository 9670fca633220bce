#!/bin/bash
# Round 5: pair kernel variants (live table 128 / 256 entries per window) vs the one-window kernel
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05n
mkdir -p "$OUT"
export TMPDIR=/tmp FAC_DIAGNOSTICS=1
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k c3 > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in pair128 pair256 nopair; do
  lib=$L/libfac.so; extra="FAC_X=0"
  [ $v = pair256 ] && lib=$L/libfac_l256.so
  [ $v = nopair ] && extra="FAC_NO_PAIR=1"
  env $extra FAC_LIB=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_$v.json" 2> "$OUT/c3_$v.err"
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));g=d['diagnostics'];f=g.get('fresh_words') or {};print('$v', round(d['ms_per_step'],2), 'wave', round(g.get('search_kernel_ms_per_step'),2), 'matches', g.get('matches_per_step'), 'fresh', round(f.get('ms_per_step',0),2), round(f.get('search_kernel_ms_per_step'),2), f.get('matches_per_step'))" "$OUT/c3_$v.json"
done
