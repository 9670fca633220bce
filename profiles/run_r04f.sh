#!/bin/bash
# r04f: lane-serial sampled-level builds: parity subset, then A/B against the wave build alone.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04f
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fullsize.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane_serial or dedup_free or differential_random or golden or c3" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04f_v "X=0" "FAC_NO_LANE_BUILD=1" "FAC_RC_T2=3" "FAC_LIVE_NQMAX=64"
BENCH_ARGS="--vocab 0 --no-fresh-diag" bash profiles/ab_knobs.sh r04f_f "X=0" "FAC_NO_LANE_BUILD=1" "FAC_LIVE_NQMAX=48" "FAC_LIVE_NQMAX=80"
