#!/bin/bash
# Round 5: host ranking of small windows through pinned staging buffers: pre-filter / stream GPU tests and
# the C5 line with FAC_TIMING phases (owned = the host ranking phase per window)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05af
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "prefilter or qgram or bitap or stream or c5 or bytes or prefiltered or owned or rank" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
FAC_DIAGNOSTICS=1 FAC_TIMING=1 timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err"
python3 -c "import json;d=json.load(open('$OUT/c5.json'));g=d['diagnostics'];print('c5', round(d['value'],1), round(d['ms_per_step'],2), 'prefilter', round(g['prefilter_ms_per_step'],2), g['matches_per_step'])"
grep "FAC_TIMING window" "$OUT/c5.err" | tail -4
