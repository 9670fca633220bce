#!/bin/bash
# r04e: phase profiles (make prof) of both workloads + T2=3 on fresh words, with a plain bench first
# to calibrate the box.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04e
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag > "$OUT/plain.json" 2> "$OUT/plain.err"
python3 -c "import json;d=json.load(open('$OUT/plain.json'));print('plain', round(d['ms_per_step'],1))"
BENCH_ARGS="--vocab 0 --no-fresh-diag" bash profiles/ab_knobs.sh r04e_f "FAC_RC_T2=3" "FAC_RC_T2=6"
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04e_v "X=0" "FAC_RC_T2=3 FAC_RC_LEVELS=5,6" "FAC_RC_T2=3 FAC_RC_LEVELS=5,6,7,8"
L=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
for v in 50000 0; do
  FAC_DIAGNOSTICS=1 FAC_LIB=$L/libfac_prof.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    --no-fresh-diag --vocab $v > "$OUT/prof_v$v.json" 2> "$OUT/prof_v$v.err"
  grep -E "^FAC_PROF" "$OUT/prof_v$v.err" || true
done
