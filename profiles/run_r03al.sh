#!/bin/bash
# r03al: level-1 build priority and the sampled counts' grid, with the one-pass counts
set -eo pipefail
bash profiles/ab_knobs.sh r03al "X=0" "FAC_L1_HIGH=1" "FAC_RC_CGRID2=1" "FAC_RC_CGRID2=4" "FAC_RC_ONE_STREAM=1" "X=0" "FAC_L1_HIGH=1"
