#!/bin/bash
# C3 bench under several FAC_* knob sets (run through gpurun from the repo root):
#   bash profiles/ab_knobs.sh TAG "ENV1=a ENV2=b" "ENV3=c" ...   (each argument one run; "X=0" = defaults)
# Outputs gpurun_out/TAG/ab<i>.json / .err; RC_DEBUG=1 adds the FAC_RC_DEBUG lines (slows the kernels:
# per-window counters); BENCH_ARGS adds bench.py flags.
set -eo pipefail
TAG=${1:?tag}
shift
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for combo in "$@"; do
  dbg=""
  [ "${RC_DEBUG:-0}" = "1" ] && dbg="FAC_RC_DEBUG=1"
  env $combo $dbg FAC_DIAGNOSTICS=1 timeout -k 10 400 python bench.py --steps 3 --warmup 1 \
    --no-cpu-baseline --no-fresh-diag ${BENCH_ARGS:-} > "$OUT/ab$i.json" 2> "$OUT/ab$i.err"
  echo "$combo: $(python3 -c "import json;d=json.load(open('$OUT/ab$i.json'));g=d['diagnostics'];print(round(d['ms_per_step'],1),'ms', g['matches_per_step'], 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))")"
  i=$((i+1))
done
