#!/bin/bash
# r04c: current C3 picture at HEAD: prefix-cache debug lines and one-step kernel timelines, on the
# vocabulary workload and on fresh words (--vocab 0).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r04c
mkdir -p "$OUT"
cd "$ROOT"
for v in 50000 0; do
  FAC_DIAGNOSTICS=1 FAC_RC_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    --no-fresh-diag --vocab $v > "$OUT/dbg_v$v.json" 2> "$OUT/dbg_v$v.err"
  grep -E "^FAC_" "$OUT/dbg_v$v.err" || true
done
export TMPDIR=/tmp
for v in 50000 0; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_v$v" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag --vocab $v > "$OUT/kt_v$v.log" 2>&1)
  find "$OUT/kt_v$v" -name '*kernel_stats.csv' -exec cp {} "$OUT/c3_v${v}_kernel_stats.csv" \;
  find "$OUT/kt_v$v" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/c3_v${v}_step_timeline.txt"
  cat "$OUT/c3_v${v}_step_timeline.txt"
done
rm -rf "$OUT"/kt_v*/
