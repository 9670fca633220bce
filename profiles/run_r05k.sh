#!/bin/bash
# Round 5: prefix-cache level / sampling sweep at the round-5 kernels (C3 + fresh-word diagnostic)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05k
mkdir -p "$OUT"
export TMPDIR=/tmp FAC_DIAGNOSTICS=1
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_$tag.json" 2> "$OUT/c3_$tag.err"
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));f=d['diagnostics'].get('fresh_words') or {};print('$tag', round(d['ms_per_step'],2), 'fresh', round(f.get('ms_per_step',0),2))" "$OUT/c3_$tag.json"
}
run default FAC_X=0
run l57 FAC_RC_LEVELS=5,7
run l56 FAC_RC_LEVELS=5,6
run l5 FAC_RC_LEVELS=5
run l567s4 FAC_RC_STRIDE2=4
run lanepops64 FAC_LANE_POPS=64
run lanepops16 FAC_LANE_POPS=16
