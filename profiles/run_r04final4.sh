#!/bin/bash
# Round-4 evidence, C2 / C4: PMC traffic, then the lines with their CPU baseline and the traffic
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_evidence.sh r04final4 pmc2 c2t pmc4 c4t
