#!/bin/bash
# Round 5: C2 (1 GiB, one-edit engine) prefix-cache level sweep at the round-5 kernels
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05v
mkdir -p "$OUT"
export TMPDIR=/tmp FAC_DIAGNOSTICS=1
for lv in 5 5,6 5,7 6 5,6,7; do
  FAC_RC_LEVELS=$lv timeout -k 10 300 python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/c2_$lv.json" 2> "$OUT/c2_$lv.err"
  python3 -c "import json;d=json.load(open('$OUT/c2_$lv.json'));g=d['diagnostics'];print('levels $lv', round(d['ms_per_step'],2), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
done
