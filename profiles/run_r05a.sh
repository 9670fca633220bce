#!/bin/bash
# Round 5, first GPU call: the GPU suite on the round-5 sources (variants removed, device-staged
# shards, call-scratch pool), then fresh-word C3 diagnostics: RC_DEBUG counters (spills: their live
# pops, snapshot queues) and the FAC_LIVE_NQMAX routing knob.
set -eo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r05a
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
export FAC_DIAGNOSTICS=1
timeout -k 10 300 env FAC_RC_DEBUG=1 python bench.py --vocab 0 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/dbg.json" 2> "$OUT/dbg.err"
grep -E "FAC_" "$OUT/dbg.err" | tail -30
BENCH_ARGS="--vocab 0" bash profiles/ab_knobs.sh r05a "X=0" "FAC_LIVE_NQMAX=8" "FAC_LIVE_NQMAX=16" "FAC_LIVE_NQMAX=32" "FAC_LIVE_NQMAX=64"
