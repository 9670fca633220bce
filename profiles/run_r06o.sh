#!/bin/bash
# Round 6: SQ counters of one C3 step at the current sources (builds, live, lane, lookup).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out/r06o
bash profiles/pmc_c3.sh r06o > gpurun_out/r06o/summary.txt 2>&1 || { tail -20 gpurun_out/r06o/summary.txt; exit 1; }
head -130 gpurun_out/r06o/summary.txt
