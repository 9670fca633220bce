#!/bin/bash
# Round 5: C2 (1 GiB) and C4 step timelines
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05t
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in c2 c4; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$cfg" -o $cfg \
    -- python3 "$ROOT/bench.py" --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt_$cfg.log" 2>&1)
  find "$OUT/kt_$cfg" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/${cfg}_timeline.txt"
  echo "== $cfg"; grep -v "fillBuffer\|slot_init\|word_kernel" "$OUT/${cfg}_timeline.txt" | awk '$NF > 0.3'
  tail -1 "$OUT/kt_$cfg.log" | cut -c1-200
done
