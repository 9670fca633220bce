#!/bin/bash
# r03ao: presence filters in front of the prefix-cache lookup tables (misses skip the HBM probe);
# parity files, then A/B against HEAD's kernels (libfac_base.so) and a kernel timeline
set -eo pipefail
OUT=gpurun_out/r03ao; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q -k "fullsize or prefix_cache or benched or lane or dedup_free" --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
L=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
bash profiles/ab_knobs.sh r03ao "FAC_LIB=$L/libfac_base.so" "X=0" "FAC_RC_CT_MULT=2" "FAC_LIB=$L/libfac_base.so" "X=0" "FAC_RC_CT_MULT=2"
bash profiles/timeline_c3.sh r03ao "X=0" | tail -30
