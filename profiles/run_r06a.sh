#!/bin/bash
# Round 6, first GPU call: the new GPU tests (empty Unicode shard), the default bench line with its new
# diagnostics legs (strong-scaling emulation, C2, C5), and the phase profile of C3 (cut reasons).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06a
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_shards_streams.py -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest_shards.log" 2>&1 || { tail -30 "$OUT/pytest_shards.log"; exit 1; }
tail -3 "$OUT/pytest_shards.log"
timeout -k 10 500 python bench.py --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
cat "$OUT/bench_c3.json"
FAC_LIB=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib/libfac_prof.so timeout -k 10 200 \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err"
grep FAC_PROF "$OUT/prof_c3.err" | tail -20
