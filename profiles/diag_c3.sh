#!/bin/bash
# Diagnostic builds on C3 (one step each): phase profile (libfac_prof.so) and pops-per-window
# histogram (libfac_hist.so), with the prefix-cache debug lines. Outputs under gpurun_out/TAG/.
set -eo pipefail
TAG=${1:?tag}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$OUT"
L=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
export FAC_DIAGNOSTICS=1 FAC_RC_DEBUG=1
FAC_LIB=$L/libfac_prof.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/prof.json" 2> "$OUT/prof.err"
grep -E "FAC_" "$OUT/prof.err"
FAC_LIB=$L/libfac_hist.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/hist.json" 2> "$OUT/hist.err"
grep -E "FAC_HIST" "$OUT/hist.err"
