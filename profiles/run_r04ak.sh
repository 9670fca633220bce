#!/bin/bash
# r04ak: the sampled counts' grid (workgroups per CU) on the final sources
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/ab_knobs.sh r04ak "X=0" "FAC_RC_CGRID2=3" "FAC_RC_CGRID2=1" "X=0" "FAC_RC_CGRID2=3"
