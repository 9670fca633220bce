#!/bin/bash
# r04ao: split sampled counts with the deeper count on a stream of its own (FAC_RC_SPLIT=1)
# builds, the 6/7-char levels after the level-1 build, beside the 5-char build): parity, C3, C2, fresh
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04ao
mkdir -p "$OUT"
FAC_RC_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane or dedup_free or differential_random or golden" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash profiles/ab_knobs.sh r04ao "X=0" "FAC_RC_SPLIT=1" "X=0" "FAC_RC_SPLIT=1"
BENCH_ARGS="--vocab 0" bash profiles/ab_knobs.sh r04ao_f "X=0" "FAC_RC_SPLIT=1"
bash profiles/timeline_c3.sh r04ao "FAC_RC_SPLIT=1" | grep -E "==|rc_count|rc_build|lookup|window_kernel"
