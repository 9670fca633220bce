#!/bin/bash
# Round 5 final evidence, part 9 (after the 16-wave scan blocks): C3 kernel stats and step timeline, and C5 kernel stats, at the final sources
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash profiles/gpu_evidence.sh r05final9 kt
OUT=$ROOT/gpurun_out/r05final9
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt5" -o c5 \
  -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/kt5.log" 2>&1)
find "$OUT/kt5" -name '*kernel_stats.csv' -exec cp {} "$OUT/c5_kernel_stats.csv" \;
head -6 "$OUT/c5_kernel_stats.csv" | cut -c1-160
