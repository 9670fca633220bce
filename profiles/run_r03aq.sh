#!/bin/bash
# r03aq: the fresh-word C3 workload (--vocab 0) under the sampled-level knobs: does its best cache policy
# differ from the vocabulary workload's defaults?
set -eo pipefail
BENCH_ARGS="--vocab 0" bash profiles/ab_knobs.sh r03aq "X=0" "FAC_RC_LEVELS=5,6" "FAC_RC_T2=1" "FAC_RC_STRIDE2=1" "FAC_RC_LEVELS=5,6,8"
