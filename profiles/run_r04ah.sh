#!/bin/bash
# r04ah: 12-state lane rings as the default: prefix-cache / lane parity subset, then C3 and C2
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04ah
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_shards_streams.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane or dedup_free or differential_random or golden or stream" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash profiles/ab_knobs.sh r04ah "X=0" "FAC_LANE_Q16=1"
BENCH_ARGS="--config c2" bash profiles/ab_knobs.sh r04ah_c2 "X=0" "FAC_LANE_Q16=1"
BENCH_ARGS="--config c4" bash profiles/ab_knobs.sh r04ah_c4 "X=0" "FAC_LANE_Q16=1"
