#!/bin/bash
# Round 5 final evidence, part 1: GPU suite, smoke, the C3 / C2 / C4 / C5 lines, C3 kernel stats and
# step timeline, the FAC_RC_DEEPEST A/B (fixed sentinel)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash profiles/gpu_evidence.sh r05final tests smoke c3 kt c2 c4 c5
OUT=$ROOT/gpurun_out/r05final
export TMPDIR=/tmp FAC_DIAGNOSTICS=1
for v in default deepest; do
  extra="FAC_X=0"; [ $v = deepest ] && extra="FAC_RC_DEEPEST=1"
  (cd /tmp && env $extra timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$v" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/deepest_$v.json" 2> "$OUT/deepest_$v.err")
  find "$OUT/kt_$v" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/c3_timeline_$v.txt"
  echo "== $v $(python3 -c "import json;d=json.load(open('$OUT/deepest_$v.json'));print(round(d['ms_per_step'],2))")"; grep rc_lookup "$OUT/c3_timeline_$v.txt"
done
