#!/bin/bash
# Round 6 final evidence, part 4: the product's search_stream (fac_stream_*) line, 4 GiB in-memory reader
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06final4
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python bench.py --config stream --gib 4 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_stream.json" 2> "$OUT/bench_stream.err"
cat "$OUT/bench_stream.json"
