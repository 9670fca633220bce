#!/bin/bash
# Round 6: key parts with the dense window lists (C2 slice), and the shard / stream tests around it.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06zg
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards_streams.py -x -q --timeout 500 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
