#!/bin/bash
# Round-4 evidence on the final sources (12-state lane rings): GPU suite, smoke, C3 / C2 / C4 lines, C3
# kernel trace and PMC traffic, then the C3 line again carrying the traffic
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_evidence.sh r04final2 tests smoke c3 c2 c4 kt pmc c3t
