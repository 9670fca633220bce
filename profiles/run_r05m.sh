#!/bin/bash
# Round 5: pair vs one-window live kernel: C3 kernel timeline and FAC_RC_DEBUG counters each
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05m
mkdir -p "$OUT"
export TMPDIR=/tmp FAC_DIAGNOSTICS=1
for v in pair nopair; do
  extra="FAC_X=0"; [ $v = nopair ] && extra="FAC_NO_PAIR=1"
  (cd /tmp && env $extra timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$v" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt_$v.log" 2>&1)
  find "$OUT/kt_$v" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/c3_timeline_$v.txt"
  env $extra FAC_RC_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/dbg_$v.json" 2> "$OUT/dbg_$v.err"
  echo "== $v"; grep -E "^FAC_LIVE|^FAC_RC launch" "$OUT/dbg_$v.err" | cut -c1-400
  grep -E "bfs_window|lane_window" "$OUT/c3_timeline_$v.txt" | head
done
