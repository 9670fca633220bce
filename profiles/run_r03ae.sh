#!/bin/bash
# r03ae: breadth-first node ids (child = edge index + 1: pushes without edge loads) and GT_SWAP
# entries (a swap in one lookup); parity, then A/B: previous kernels / both / no swap table
set -eo pipefail
OUT=gpurun_out/r03ae; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
L=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
bash profiles/ab_knobs.sh r03ae "FAC_LIB=$L/libfac_base.so" "X=0" "FAC_NO_SWAP_TABLE=1" "FAC_LIB=$L/libfac_base.so" "X=0" "FAC_NO_SWAP_TABLE=1"
