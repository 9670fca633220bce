#!/bin/bash
# r03x: cache-build lists sorted by parent key -- parity (incl. the full-size sampled check) and A/B
set -eo pipefail
OUT=gpurun_out/r03x; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 900 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash profiles/ab_knobs.sh r03x "X=0" "FAC_RC_NO_SORT=1" "X=1"
