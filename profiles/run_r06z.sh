#!/bin/bash
# Round 6: staging kernels (transposed LDS tile + LDS property bytes; register decode + LDS fold in
# write_tile) -- the whole GPU suite, then C3 and a key part's trace.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06z
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --no-fresh-diag > "$OUT/c3.json" 2> "$OUT/c3.err"
python3 -c "import json; d=json.load(open('$OUT/c3.json')); g=d['diagnostics']; print('c3', '%.2f ms' % d['ms_per_step'], 'staging %.2f' % g['staging_ms_per_step'], 'cache %.2f lane %.2f wave %.2f' % (g['prefix_cache_ms_per_step'], g['lane_kernel_ms_per_step'], g['search_kernel_ms_per_step']))"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o keys \
  -- python3 "$ROOT/profiles/shard_trace.py" 8 3 3 keys > "$OUT/kt.log" 2>&1)
grep "key part" "$OUT/kt.log"
f=$(find "$OUT/kt" -name 'keys_kernel_trace.csv' | head -1)
python3 profiles/step_timeline.py "$f" > "$OUT/keypart_timeline.txt"
head -8 "$OUT/keypart_timeline.txt"
