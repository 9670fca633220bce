#!/bin/bash
# Round 6: kernel trace of the C3 1/8 shard's step (strong-scaling fixed costs).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06g
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o shard \
  -- python3 "$ROOT/profiles/shard_trace.py" 8 3 3 > "$OUT/kt.log" 2>&1)
cat "$OUT/kt.log" | grep shard
find "$OUT/kt" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/shard_step_timeline.txt"
cat "$OUT/shard_step_timeline.txt"
