#!/bin/bash
# r03ab: build epilogue without the key chars (publish reads them from the representative's text),
# one table read; build code compiled into the build kernels only -- parity, then A/B vs HEAD's library
set -eo pipefail
OUT=gpurun_out/r03ab; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
L=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
bash profiles/ab_knobs.sh r03ab "FAC_LIB=$L/libfac_base.so" "X=0" "FAC_LIB=$L/libfac_base.so" "X=0"
