#!/bin/bash
# r04u: level-1 build priority and the sampled counts' grid now that the counts are cheaper
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/ab_knobs.sh r04u "X=0" "FAC_L1_HIGH=1" "FAC_RC_CGRID2=1" "FAC_RC_CGRID2=4" "X=0"
