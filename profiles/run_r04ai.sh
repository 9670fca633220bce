#!/bin/bash
# r04ai: cache-build chunk (representatives per work-counter turn: a chunk of heavy keys holds its wave
# at the end of a level) and the lane pop budget with 12-state rings
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/ab_knobs.sh r04ai "X=0" "FAC_BUILD_CHUNK=16" "FAC_BUILD_CHUNK=4" "FAC_BUILD_CHUNK=1" "FAC_LANE_POPS=64" "FAC_LANE_POPS=16" "X=0"
