#!/bin/bash
# r03y: fresh-container baseline at HEAD -- default C3 bench with the prefix-cache debug lines, then the
# phase profile and pops-per-window histogram builds (profiles/diag_c3.sh)
set -eo pipefail
OUT=gpurun_out/r03y; mkdir -p $OUT
RC_DEBUG=1 bash profiles/ab_knobs.sh r03y "X=0"
grep -E "FAC_" $OUT/ab0.err | head -40
bash profiles/diag_c3.sh r03y
