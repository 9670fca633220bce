#!/bin/bash
# r04h: lane-build deferral statistics; the small build variant A/B (vocabulary and fresh words)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04h
mkdir -p "$OUT"
FAC_DIAGNOSTICS=1 FAC_RC_DEBUG=1 FAC_LANE_BUILD=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
  --no-fresh-diag > "$OUT/dbg.json" 2> "$OUT/dbg.err"
grep -E "^FAC_(LB|RC |LK)" "$OUT/dbg.err" || true
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04h_v "X=0" "FAC_BUILD_SMALL=1" "FAC_BUILD_SMALL=1 FAC_RC_T2=3"
BENCH_ARGS="--vocab 0 --no-fresh-diag" bash profiles/ab_knobs.sh r04h_f "X=0" "FAC_BUILD_SMALL=1"
