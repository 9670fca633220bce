#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r05e
mkdir -p "$OUT"
timeout -k 10 120 python profiles/fam_debug.py > "$OUT/fam.log" 2>&1; echo rc=$?
timeout -k 10 120 python profiles/fam_debug.py nofam > "$OUT/nofam.log" 2>&1; echo rc=$?
grep -E "^case|^gpu|^orc" "$OUT/fam.log" "$OUT/nofam.log" | cut -c1-300
