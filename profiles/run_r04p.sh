#!/bin/bash
# r04p: HEAD evidence: kernel trace timeline + HBM traffic (FETCH/WRITE_SIZE), then SQ issue/wait per kernel
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_evidence.sh r04p kt pmc
bash profiles/pmc_c3.sh r04p > gpurun_out/r04p/sq_summary.txt
head -80 gpurun_out/r04p/sq_summary.txt
