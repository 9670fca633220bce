#!/bin/bash
# r04aj: the whole GPU suite on the final sources (incl. the count-threshold cases of the round-4 path test)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_evidence.sh r04aj tests smoke
