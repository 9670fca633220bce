#!/bin/bash
# A/B of the beam's two reference-order restatements on C3 (run through gpurun from the repo root):
#   bash profiles/ab_beam.sh TAG
# default (hashbrown edge order + select_nth_unstable_by), FAC_BEAM_CANONICAL (rounds 1-2's tie rule),
# FAC_EDGE_INSERTION (insertion edge order), both; FAC_RC_DEBUG lines go to the .err files.
set -eo pipefail
TAG=${1:?tag}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for combo in "X=0" "FAC_BEAM_CANONICAL=1" "FAC_EDGE_INSERTION=1" "FAC_BEAM_CANONICAL=1 FAC_EDGE_INSERTION=1"; do
  env $combo FAC_DIAGNOSTICS=1 FAC_RC_DEBUG=1 timeout -k 10 400 python bench.py --steps 2 --warmup 0 --no-cpu-baseline \
    --prestaged ${EXTRA:-} > "$OUT/ab$i.json" 2> "$OUT/ab$i.err"
  echo "$combo: $(python3 -c "import json;d=json.load(open('$OUT/ab$i.json'));print(round(d['ms_per_step'],1),'ms', d['diagnostics']['matches_per_step'])")"
  i=$((i+1))
done
