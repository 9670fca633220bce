#!/bin/bash
# r04y: knob sweep on the current sources: demand level, lane pop budget
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/ab_knobs.sh r04y "X=0" "FAC_RC_DEMAND=8" "FAC_RC_LEVELS=5,6 FAC_RC_DEMAND=7" "FAC_LANE_POPS=48" "FAC_LANE_POPS=24" "FAC_LANE_POPS=64"
