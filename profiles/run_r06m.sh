#!/bin/bash
# Round 6: lookup-table slots per kept snapshot of the sampled levels (FAC_RC_CT_MULT2 = 1 / 2 / 4) on C2 and C3.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06m
mkdir -p "$OUT"
cd "$ROOT"
for cfg in c2 c3; do
  for m in 4 2 1 4; do
    FAC_DIAGNOSTICS=1 FAC_RC_CT_MULT2=$m timeout -k 10 300 python bench.py --config $cfg --steps 5 --no-cpu-baseline --no-fresh-diag \
      > "$OUT/${cfg}_m$m.json" 2> "$OUT/${cfg}_m$m.err"
    python3 -c "import json,sys; d=json.load(open('$OUT/${cfg}_m$m.json')); g=d['diagnostics']; print('$cfg m=$m', '%.2f ms' % d['ms_per_step'], 'cache %.2f lane %.2f wave %.2f' % (g['prefix_cache_ms_per_step'], g['lane_kernel_ms_per_step'], g['search_kernel_ms_per_step']))"
  done
done
