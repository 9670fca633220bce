#!/bin/bash
# Round 5: family builds with forks (run_window FAM resumes past the parent's queue). GPU suite, then
# C3 (+ fresh-word diagnostic) per FAC_FAMILY level mask, and one kernel timeline for 2 (default) and 0
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05g
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for fm in 2 0 3 6; do
  FAC_FAMILY=$fm timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_f$fm.json" 2> "$OUT/c3_f$fm.err"
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));f=d['diagnostics'].get('fresh_words') or {};print('FAC_FAMILY=$fm', d['ms_per_step'], d['value'], 'fresh', f.get('ms_per_step'))" "$OUT/c3_f$fm.json"
done
export FAC_DIAGNOSTICS=1
for fm in 2 0; do
  (cd /tmp && FAC_FAMILY=$fm timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$fm" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt_$fm.log" 2>&1)
  find "$OUT/kt_$fm" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/c3_timeline_$fm.txt"
  FAC_FAMILY=$fm FAC_RC_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/dbg_$fm.json" 2> "$OUT/dbg_$fm.err"
  echo "== $fm"; grep -E "^FAC_RC windows|^FAC_LK" "$OUT/dbg_$fm.err" | tail -2 | cut -c1-400
  grep -E "rc_build|rc_family|bfs_window|lane_window|rc_lookup|radix|rc_parent" "$OUT/c3_timeline_$fm.txt" | head -30
done
