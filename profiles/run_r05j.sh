#!/bin/bash
# Round 5: live kernel occupancy -- the live table in global memory (LDS 10 -> 6 KB per wave) at 4 / 5 / 6
# waves per SIMD (compile-time FAC_LIVE_GLOBAL / FAC_LIVE_WAVES variants); C3 + the fresh-word diagnostic
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05j
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
for v in base lg4 lg5 lg6; do
  lib=$L/libfac_$v.so; [ $v = base ] && lib=$L/libfac.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_$v.json" 2> "$OUT/c3_$v.err"
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));f=d['diagnostics'].get('fresh_words') or {};print('$v', round(d['ms_per_step'],2), 'wave', d['diagnostics'].get('search_kernel_ms_per_step'), 'fresh', round(f.get('ms_per_step',0),2), f.get('search_kernel_ms_per_step'))" "$OUT/c3_$v.json"
done
