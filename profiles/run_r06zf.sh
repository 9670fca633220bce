#!/bin/bash
# Round 6: sampled-level count table size (FAC_RC_SLOTS2 = log2 slots per level) on C3 and fresh-word C3.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06zf
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_shards_streams.py -x -q --timeout 300 --timeout-method thread \
  -k "dense_window_list" > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
export FAC_DIAGNOSTICS=1
for sl in 27 26 25 24 27; do
  FAC_RC_SLOTS2=$sl timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --no-fresh-diag > "$OUT/c3_s$sl.json" 2> "$OUT/c3_s$sl.err"
  python3 -c "import json; d=json.load(open('$OUT/c3_s$sl.json')); g=d['diagnostics']; print('c3 slots2=$sl', '%.2f ms' % d['ms_per_step'], 'cache %.2f lane %.2f wave %.2f cached %.3g' % (g['prefix_cache_ms_per_step'], g['lane_kernel_ms_per_step'], g['search_kernel_ms_per_step'], g['states_from_prefix_cache_per_step']))"
done
for sl in 27 25; do
  FAC_RC_SLOTS2=$sl timeout -k 10 300 python bench.py --vocab 0 --steps 2 --no-cpu-baseline --no-fresh-diag > "$OUT/fresh_s$sl.json" 2> "$OUT/fresh_s$sl.err"
  python3 -c "import json; d=json.load(open('$OUT/fresh_s$sl.json')); g=d['diagnostics']; print('fresh slots2=$sl', '%.2f ms' % d['ms_per_step'], 'cache %.2f lane %.2f wave %.2f' % (g['prefix_cache_ms_per_step'], g['lane_kernel_ms_per_step'], g['search_kernel_ms_per_step']))"
done
