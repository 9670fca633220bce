#!/bin/bash
# r04d: fresh-word C3 (--vocab 0) with fewer / no sampled levels; then the phase profile (make prof)
# of both workloads.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
BENCH_ARGS="--vocab 0 --no-fresh-diag" bash profiles/ab_knobs.sh r04d "X=0" "FAC_RC_K2=0" "FAC_RC_LEVELS=6" "FAC_RC_T2=4"
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04d_v "X=0" "FAC_RC_DEEPEST=1" "FAC_RC_K2=0" "FAC_RC_LEVELS=6,7" "FAC_RC_T2=3" "FAC_RC_T2=4" "FAC_RC_T2=3 FAC_RC_STRIDE2=1"
OUT=$ROOT/gpurun_out/r04d
L=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
for v in 50000 0; do
  FAC_DIAGNOSTICS=1 FAC_LIB=$L/libfac_prof.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    --no-fresh-diag --vocab $v > "$OUT/prof_v$v.json" 2> "$OUT/prof_v$v.err"
  grep -E "^FAC_PROF" "$OUT/prof_v$v.err" || true
done
