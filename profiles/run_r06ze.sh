#!/bin/bash
# Round 6: key-part lists through tiled masks, coalesced write_tile -- GPU suite, the default line
# (strong-scaling estimate, C2 / C5 legs), a key part's trace.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06ze
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 600 python bench.py --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
python3 - "$OUT" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/bench_c3.json"))
g = d["diagnostics"]
print("c3 %.3f Gchars/s %.2f ms staging %.2f cache %.2f lane %.2f wave %.2f" % (d["value"], d["ms_per_step"], g["staging_ms_per_step"], g["prefix_cache_ms_per_step"], g["lane_kernel_ms_per_step"], g["search_kernel_ms_per_step"]))
for k in ("shards", "keys"):
    print(k, {n: (round(v["max_rank_ms"], 2), round(v["predicted_speedup"], 2), v["rank_ms"]) for n, v in g["strong_emulated"][k].items()})
print("fresh", round(g["fresh_words"]["ms_per_step"], 1), "c2", round(g["c2"]["value"], 2), round(g["c2"]["ms_per_step"], 2), "c5", round(g["c5"]["value"], 1))
PY
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o keys \
  -- python3 "$ROOT/profiles/shard_trace.py" 8 3 3 keys > "$OUT/kt.log" 2>&1)
grep "key part" "$OUT/kt.log"
f=$(find "$OUT/kt" -name 'keys_kernel_trace.csv' | head -1)
python3 profiles/step_timeline.py "$f" > "$OUT/keypart_timeline.txt"
head -10 "$OUT/keypart_timeline.txt"
