#!/bin/bash
# r04ad: cache policy sweep now that the counts are cheaper: sampled stride / threshold / levels
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/ab_knobs.sh r04ad "X=0" "FAC_RC_STRIDE2=1 FAC_RC_T2=2" "FAC_RC_STRIDE2=1 FAC_RC_T2=3" "FAC_RC_STRIDE2=1 FAC_RC_T2=4" \
  "FAC_RC_LEVELS=5,6,7,8" "FAC_RC_LEVELS=5,6,8" "FAC_RC_LEVELS=5,7"
