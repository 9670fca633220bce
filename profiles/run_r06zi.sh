#!/bin/bash
# Round 6: repeated search_stream calls in one process.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06zi
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python profiles/stream_probe.py 2 4 > "$OUT/probe.log" 2> "$OUT/probe.err"
cat "$OUT/probe.log"
FAC_DIAGNOSTICS=1 FAC_TIMING=1 timeout -k 10 400 python profiles/stream_probe.py 0.5 2 > "$OUT/probe_t.log" 2> "$OUT/probe_t.err"
cat "$OUT/probe_t.log"
