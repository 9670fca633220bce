#!/bin/bash
# r04ag: lane kernel with 12-state rings (10 KB of LDS: 16 waves per CU instead of 12) vs 16, C3 + fresh
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/ab_knobs.sh r04ag "X=0" "FAC_LANE_Q12=1" "X=0" "FAC_LANE_Q12=1"
BENCH_ARGS="--vocab 0" bash profiles/ab_knobs.sh r04ag_f "X=0" "FAC_LANE_Q12=1"
