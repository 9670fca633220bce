#!/bin/bash
# r04j: defaults after r04i, plus A/B of the small variant for level 1 and for the spilled windows
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04j_plain.json 2> gpurun_out/r04j_plain.err; python3 -c "import json;d=json.load(open('gpurun_out/r04j_plain.json'));print('plain', round(d['ms_per_step'],1), d['diagnostics']['fresh_words']['ms_per_step'])"
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04j_v "X=0" "FAC_BUILD_SMALL_L1=1" "FAC_SPILL_SMALL=1"
BENCH_ARGS="--vocab 0 --no-fresh-diag" bash profiles/ab_knobs.sh r04j_f "X=0" "FAC_BUILD_SMALL_L1=1" "FAC_SPILL_SMALL=1" "FAC_RC_K2=0"
