#!/bin/bash
# r04t: fresh-word C3 (--vocab 0): entry caps of the prefix-cache levels; vocabulary C3 with the same caps
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
BENCH_ARGS="--vocab 0" bash profiles/ab_knobs.sh r04t_f "X=0" "FAC_RC_ENTRIES=33554432" "FAC_RC_ENTRIES=50331648"
bash profiles/ab_knobs.sh r04t_v "X=0" "FAC_RC_ENTRIES=33554432" "FAC_RC_STRIDE2=4 FAC_RC_T2=1"
