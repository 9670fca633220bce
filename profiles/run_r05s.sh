#!/bin/bash
# Round 5: C5 with the prefix cache on (default) / off for the re-searched windows (FAC_RC_MIN)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05s
mkdir -p "$OUT"
export TMPDIR=/tmp FAC_DIAGNOSTICS=1
for v in default rcoff; do
  extra="FAC_X=0"; [ $v = rcoff ] && extra="FAC_RC_MIN=100000000"
  env $extra timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c5_$v.json" 2> "$OUT/c5_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/c5_$v.json'));g=d['diagnostics'];print('$v', round(d['value'],1), round(d['ms_per_step'],2), g['matches_per_step'])"
done
