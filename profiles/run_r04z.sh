#!/bin/bash
# r04z: round-4 evidence, part 1: GPU suite, smoke, the C3 line (CPU baseline + fresh-word diagnostic), C2, C4
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_evidence.sh r04z tests smoke c3 c2 c4
