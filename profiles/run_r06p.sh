#!/bin/bash
# Round 6: lookups with the shallower probes deferred into full waves -- parity (prefix cache, full size), C2 / C3
# lines, and C2 / C3 kernel stats.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06p
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shards_streams.py -x -q --timeout 700 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for cfg in c2 c3; do
  timeout -k 10 300 python bench.py --config $cfg --steps 5 --no-cpu-baseline --no-fresh-diag > "$OUT/$cfg.json" 2> "$OUT/$cfg.err"
  python3 -c "import json,sys; d=json.load(open('$OUT/$cfg.json')); g=d['diagnostics']; print('$cfg', '%.2f ms' % d['ms_per_step'], 'cache %.2f lane %.2f wave %.2f' % (g['prefix_cache_ms_per_step'], g['lane_kernel_ms_per_step'], g['search_kernel_ms_per_step']), 'matches', g['matches_per_step'])"
done
export TMPDIR=/tmp
for cfg in c2 c3; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$cfg" -o $cfg \
    -- python3 "$ROOT/bench.py" --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt_$cfg.log" 2>&1)
  f=$(find "$OUT/kt_$cfg" -name '*kernel_stats.csv')
  grep -i "lookup\|Name" "$f" | cut -d, -f1-5
done
