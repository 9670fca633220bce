#!/bin/bash
# Round 5: C5 host phases per stream window (FAC_TIMING)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05r
mkdir -p "$OUT"
export TMPDIR=/tmp FAC_DIAGNOSTICS=1 FAC_TIMING=1
timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err"
grep FAC_TIMING "$OUT/c5.err" | tail -12
