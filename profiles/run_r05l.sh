#!/bin/bash
# Round 5: paired live kernel (two windows per wave): GPU suite, then C3 + fresh-word with the pair
# kernel (default) and the one-window kernel (FAC_NO_PAIR=1)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05l
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
export FAC_DIAGNOSTICS=1
for v in pair nopair; do
  extra="FAC_X=0"; [ $v = nopair ] && extra="FAC_NO_PAIR=1"
  env $extra timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_$v.json" 2> "$OUT/c3_$v.err"
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));g=d['diagnostics'];f=g.get('fresh_words') or {};print('$v', round(d['ms_per_step'],2), 'wave', g.get('search_kernel_ms_per_step'), 'matches', g.get('matches_per_step'), 'fresh', round(f.get('ms_per_step',0),2), f.get('search_kernel_ms_per_step'), f.get('matches_per_step'))" "$OUT/c3_$v.json"
done
