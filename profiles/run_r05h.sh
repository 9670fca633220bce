#!/bin/bash
# Round 5: family-build stop reasons (FAC_RC_DEBUG) and C3 step time per FAC_FAMILY mask
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05h
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
export FAC_DIAGNOSTICS=1
FAC_FAMILY=2 FAC_RC_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/dbg_2.json" 2> "$OUT/dbg_2.err"
grep -E "^FAC_RC windows|^FAC_FAM" "$OUT/dbg_2.err" | tail -3 | cut -c1-400
for fm in 2 0; do
  FAC_FAMILY=$fm timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_f$fm.json" 2> "$OUT/c3_f$fm.err"
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));f=d['diagnostics'].get('fresh_words') or {};print('FAC_FAMILY=$fm', d['ms_per_step'], d['value'], 'fresh', f.get('ms_per_step'))" "$OUT/c3_f$fm.json"
done
