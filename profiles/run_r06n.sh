#!/bin/bash
# Round 6: SQ counters of one C2 step (rc_lookup and the lane kernel: issue / wait breakdown).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
BENCH_ARGS="--config c2" bash profiles/pmc_c3.sh r06n > gpurun_out/r06n_summary.txt 2>&1 || { tail -20 gpurun_out/r06n_summary.txt; exit 1; }
mkdir -p gpurun_out/r06n && mv gpurun_out/r06n_summary.txt gpurun_out/r06n/summary.txt
head -80 gpurun_out/r06n/summary.txt
