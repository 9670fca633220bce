#!/bin/bash
# Round 5: q-gram verify with word loads: pre-filter tests, C5 line and kernel stats
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05p
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "prefilter or qgram or bitap or stream or c5 or bytes or distributed or prefiltered" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 400 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err"
python3 -c "import json;d=json.load(open('$OUT/c5.json'));g=d['diagnostics'];print(d['value'], d['ms_per_step'], {k:g[k] for k in g if 'ms' in k})"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o c5 \
  -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/kt.log" 2>&1)
f=$(find "$OUT/kt" -name '*kernel_stats.csv' | head -1); head -5 "$f" | cut -d, -f1-4
