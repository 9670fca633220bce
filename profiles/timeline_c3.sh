#!/bin/bash
# One C3 step's kernel timeline under diagnostics env settings: bash profiles/timeline_c3.sh TAG "ENV=.." ...
set -eo pipefail
TAG=${1:?tag}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp FAC_DIAGNOSTICS=1
i=0
for setting in "$@"; do
  i=$((i + 1))
  (cd /tmp && env $setting timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/t$i" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --no-fresh-diag $BENCH_ARGS > "$OUT/t$i.log" 2>&1)
  echo "== $setting"
  find "$OUT/t$i" -name '*kernel_trace.csv' -exec python3 "$ROOT/profiles/step_timeline.py" {} \; | tee "$OUT/timeline$i.txt"
done
