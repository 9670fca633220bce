#!/bin/bash
# bisect the k4 differential failure: family builds off / main-pass chunk pinned
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r05d
mkdir -p "$OUT"
T="tests/test_gpu_parity.py::test_differential_random"
for env in "X=0" "FAC_DIAGNOSTICS=1 FAC_NO_FAMILY=1" "FAC_DIAGNOSTICS=1 FAC_RC_CHUNK=256"; do
  echo "== $env"
  env $env timeout -k 10 200 python -u -m pytest "$T" -m gpu -x -q --timeout 120 --timeout-method thread -k "k4 and vocab0 and False" 2>&1 | tail -3
  rc=$?
  [ $rc -ge 124 ] && exit $rc
done
exit 0
