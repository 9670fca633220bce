#!/bin/bash
# Round 6: C5 kernel trace (one 12.5 GiB step at 256 KiB windows) -- where the pre-filter's time goes.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06y
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o c5 \
  -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/kt.log" 2>&1)
f=$(find "$OUT/kt" -name 'c5_kernel_stats.csv' | head -1)
cp "$f" "$OUT/c5_kernel_stats.csv"
python3 - "$OUT/c5_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(r["Name"][:70], r["Calls"], "%.3f ms total" % (float(r["TotalDurationNs"]) / 1e6), "%.3f avg" % (float(r["AverageNs"]) / 1e6))
PY
