#!/bin/bash
# Round-4 evidence, C5: the line, PMC traffic, the line again carrying the traffic
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_evidence.sh r04final3 c5 pmc5 c5t
