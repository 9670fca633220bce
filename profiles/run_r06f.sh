#!/bin/bash
# Round 6: strong-scaling policy sweep on the C3 shards of 8 (prefix-cache knobs), and the 1/8 shard's
# kernel trace.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06f
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 500 python profiles/shard_sweep.py 8 default FAC_RC_LEVELS=5,6 FAC_RC_LEVELS=5,7 FAC_RC_LEVELS=5 \
  FAC_RC_STRIDE2=1 FAC_RC_LEVELS=6 FAC_RC_STRIDE1=4 > "$OUT/sweep8.jsonl" 2> "$OUT/sweep8.err"
cat "$OUT/sweep8.jsonl"
