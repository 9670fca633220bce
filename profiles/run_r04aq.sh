#!/bin/bash
# r04aq: split sampled counts, the host waiting on the level-1 event before the deeper count and the first level's build (libfac_splith.so; FAC_RC_SPLIT=1) against HEAD
# the r04ao patch; FAC_RC_SPLIT=1) against HEAD: parity subset on the variant, C3, fresh C3, a timeline
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
OUT=$ROOT/gpurun_out/r04aq
mkdir -p "$OUT"
FAC_LIB=$L/libfac_splith.so FAC_RC_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or differential_random" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash profiles/ab_knobs.sh r04aq "X=0" "FAC_LIB=$L/libfac_splith.so FAC_RC_SPLIT=1" "X=0" "FAC_LIB=$L/libfac_splith.so FAC_RC_SPLIT=1"
BENCH_ARGS="--vocab 0" bash profiles/ab_knobs.sh r04aq_f "X=0" "FAC_LIB=$L/libfac_splith.so FAC_RC_SPLIT=1"
bash profiles/timeline_c3.sh r04aq "FAC_LIB=$L/libfac_splith.so FAC_RC_SPLIT=1" | grep -E "==|rc_count|rc_build|rc_parent|lookup|window_kernel"
