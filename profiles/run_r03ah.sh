#!/bin/bash
# r03ah: re-sweep of the beamed engines' sampled prefix-cache levels at the round's final kernels
# (the r03 sweeps predate the select-as-call and cache-build epilogue changes)
set -eo pipefail
bash profiles/ab_knobs.sh r03ah "X=0" "FAC_RC_LEVELS=5,6,7" "FAC_RC_T2=1" "FAC_RC_LEVELS=5,6,7 FAC_RC_T2=3" \
  "FAC_RC_LEVELS=5,7,9" "FAC_RC_LEVELS=5,6" "FAC_RC_STRIDE2=4 FAC_RC_T2=1" "FAC_LANE_POPS=48" "X=0"
