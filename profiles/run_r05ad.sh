#!/bin/bash
# Round 5: q-gram candidate-region overflow test (regions full, overflow list regrown) plus the pre-filter
# GPU tests, with the FAC_TIMING candidate counts of the overflow case
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ad
mkdir -p "$OUT"
export TMPDIR=/tmp
FAC_TIMING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -s -k "regions_overflow" > "$OUT/overflow.log" 2>&1 || { tail -30 "$OUT/overflow.log"; exit 1; }
grep -E "FAC_QGRAM|PASS|FAIL" "$OUT/overflow.log" | head -12
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "prefilter or qgram or bitap or stream or c5 or bytes or prefiltered" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
