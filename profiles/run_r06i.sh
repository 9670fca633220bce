#!/bin/bash
# Round 6: key partition without the window-loop check (cache-off parts walk a window list) -- tests, C3
# line, and the kernel trace of key part 3 of 8.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06i
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards_streams.py -x -q -k "key_partition or shard" --timeout 500 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-fresh-diag > "$OUT/c3_$i.json" 2> "$OUT/c3_$i.err"
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/c3_*.json")):
    d = json.load(open(f)); g = d["diagnostics"]
    print(f.split("/")[-1], "ms %.2f" % d["ms_per_step"], "cache %.2f" % g["prefix_cache_ms_per_step"], "wave %.2f" % g["search_kernel_ms_per_step"])
PY
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o keys \
  -- python3 "$ROOT/profiles/shard_trace.py" 8 3 3 keys > "$OUT/kt.log" 2>&1)
grep "key part" "$OUT/kt.log"
