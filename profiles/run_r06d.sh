#!/bin/bash
# Round 6: batched stream windows (C5 at the crate's 256 KiB windows; fac_stream_* batches) -- stream tests,
# C5 at 256 KiB against 1 GiB windows, the search_stream line.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06d
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards_streams.py tests/test_gpu_parity.py -k "stream or replace or window" -x -v --timeout 500 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py --config c5 --steps 2 --no-cpu-baseline > "$OUT/c5_256k.json" 2> "$OUT/c5_256k.err"
cat "$OUT/c5_256k.json"
timeout -k 10 300 python bench.py --config c5 --steps 2 --window-kib 0 --no-cpu-baseline > "$OUT/c5_1g.json" 2> "$OUT/c5_1g.err"
cat "$OUT/c5_1g.json"
timeout -k 10 300 python bench.py --config stream --steps 1 --gib 4 > "$OUT/stream.json" 2> "$OUT/stream.err"
cat "$OUT/stream.json"
