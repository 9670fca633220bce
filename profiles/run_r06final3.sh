#!/bin/bash
# Round 6 final evidence, part 3: C3 kernel stats and step timeline, C5 kernel stats, C2 kernel stats
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash profiles/gpu_evidence.sh r06final3 kt
OUT=$ROOT/gpurun_out/r06final3
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt5" -o c5 \
  -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/kt5.log" 2>&1)
find "$OUT/kt5" -name '*kernel_stats.csv' -exec cp {} "$OUT/c5_kernel_stats.csv" \;
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt2" -o c2 \
  -- python3 "$ROOT/bench.py" --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt2.log" 2>&1)
find "$OUT/kt2" -name '*kernel_stats.csv' -exec cp {} "$OUT/c2_kernel_stats.csv" \;
find "$OUT/kt2" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/c2_step_timeline.txt"
head -6 "$OUT/c5_kernel_stats.csv" | cut -c1-160
head -8 "$OUT/c2_kernel_stats.csv" | cut -c1-160
