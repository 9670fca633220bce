#!/bin/bash
# Round 5: family builds on vs off (FAC_NO_FAMILY=1) on C3: one step's kernel timeline each, and the
# FAC_RC_DEBUG counters (keys, cached snapshots, lookup levels)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05f
mkdir -p "$OUT"
export TMPDIR=/tmp FAC_DIAGNOSTICS=1
for mode in fam nofam; do
  extra=""; [ $mode = nofam ] && extra="FAC_NO_FAMILY=1"
  (cd /tmp && env $extra timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$mode" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt_$mode.log" 2>&1)
  find "$OUT/kt_$mode" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/c3_timeline_$mode.txt"
  env $extra FAC_RC_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/dbg_$mode.json" 2> "$OUT/dbg_$mode.err"
  echo "== $mode"; grep -E "^FAC_RC windows|^FAC_LK" "$OUT/dbg_$mode.err" | tail -2 | cut -c1-400
  grep -E "rc_build|rc_family|bfs_window|lane_window|rc_lookup|radix|rc_parent" "$OUT/c3_timeline_$mode.txt" | head -30
done
