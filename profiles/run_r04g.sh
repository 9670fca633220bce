#!/bin/bash
# r04g: kernel timeline of one C3 step with the lane-serial sampled builds (vocabulary workload)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r04g
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o c3 \
  -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt.log" 2>&1)
find "$OUT/kt" -name '*kernel_trace.csv' -exec python3 "$ROOT/profiles/step_timeline.py" {} \; > "$OUT/c3_step_timeline.txt"
cat "$OUT/c3_step_timeline.txt"
rm -rf "$OUT/kt"
