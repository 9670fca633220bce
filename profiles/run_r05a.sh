#!/bin/bash
# Round 5, first look at fresh-word C3: RC_DEBUG counters (spills, pops by pass) and the
# FAC_LIVE_NQMAX routing knob (windows whose snapshot queue is longer go straight to the exact kernel).
set -eo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r05a
mkdir -p "$OUT"
export FAC_DIAGNOSTICS=1
timeout -k 10 300 env FAC_RC_DEBUG=1 python bench.py --vocab 0 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/dbg.json" 2> "$OUT/dbg.err"
grep -E "FAC_" "$OUT/dbg.err" | tail -30
BENCH_ARGS="--vocab 0" bash profiles/ab_knobs.sh r05a "X=0" "FAC_LIVE_NQMAX=8" "FAC_LIVE_NQMAX=16" "FAC_LIVE_NQMAX=32" "FAC_LIVE_NQMAX=64"
