#!/bin/bash
# r04v: phase profile (libfac_prof.so, FAC_PHASE_PROF cycle counters) of one C3 step: where the cache
# builds and the main pass spend their wave cycles
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04v
mkdir -p "$OUT"
FAC_LIB=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib/libfac_prof.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 \
  --no-cpu-baseline --no-fresh-diag > "$OUT/prof.json" 2> "$OUT/prof.err"
grep FAC_PROF "$OUT/prof.err"
