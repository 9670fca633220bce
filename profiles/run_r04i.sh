#!/bin/bash
# r04i: small sampled-level build variant with deferral of what it cannot hold: parity under the knob,
# then A/B (vocabulary and fresh words)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04i
mkdir -p "$OUT"
FAC_DIAGNOSTICS=1 FAC_BUILD_SMALL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fullsize.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane_serial or dedup_free or differential_random or golden or c3" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04i_v "X=0" "FAC_BUILD_SMALL=1" "FAC_BUILD_SMALL=1 FAC_RC_T2=3"
BENCH_ARGS="--vocab 0 --no-fresh-diag" bash profiles/ab_knobs.sh r04i_f "X=0" "FAC_BUILD_SMALL=1" "FAC_BUILD_SMALL=1 FAC_RC_T2=3"
