#!/bin/bash
# r03ai: sampled-level sets around "5,6,7" (best of r03ah, 147.1 vs 149.0 / 149.7 ms), repeated
set -eo pipefail
bash profiles/ab_knobs.sh r03ai "X=0" "FAC_RC_LEVELS=5,6,7" "FAC_RC_LEVELS=5,6,8" "FAC_RC_LEVELS=5,6,7,8" \
  "FAC_RC_LEVELS=5,6,7,9" "FAC_RC_LEVELS=5,6,7 FAC_LANE_POPS=48" "X=0" "FAC_RC_LEVELS=5,6,7"
