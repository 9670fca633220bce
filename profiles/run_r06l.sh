#!/bin/bash
# Round 6: C2's prefix-cache levels and lookup outcomes (FAC_RC_DEBUG).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06l
mkdir -p "$OUT"
cd "$ROOT"
FAC_DIAGNOSTICS=1 FAC_RC_DEBUG=1 timeout -k 10 300 python bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/c2_debug.json" 2> "$OUT/c2_debug.err"
grep "FAC_RC\|FAC_LK\|FAC_LANE" "$OUT/c2_debug.err" | tail -12
