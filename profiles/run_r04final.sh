#!/bin/bash
# Round-4 evidence on the final sources: GPU suite, smoke, C3 (CPU baseline + fresh-word diagnostic),
# C2, C4, C5, C3 kernel trace, C3 PMC traffic
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_evidence.sh r04final tests smoke c3 c2 c4 c5 kt pmc
