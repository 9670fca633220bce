#!/bin/bash
# Round 6 checkpoint: the whole GPU suite, smoke, and the default bench line (C3 + every diagnostics leg).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06k
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
cat "$OUT/smoke.log"
timeout -k 10 600 python bench.py --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
python3 - "$OUT" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/bench_c3.json"))
g = d["diagnostics"]
print("c3 %.3f Gchars/s %.2f ms cache %.2f lane %.2f wave %.2f" % (d["value"], d["ms_per_step"], g["prefix_cache_ms_per_step"], g["lane_kernel_ms_per_step"], g["search_kernel_ms_per_step"]))
for k in ("shards", "keys"):
    print(k, {n: (round(v["max_rank_ms"], 2), round(v["predicted_speedup"], 2)) for n, v in g["strong_emulated"][k].items()})
print("fresh", round(g["fresh_words"]["ms_per_step"], 1), "c2", round(g["c2"]["value"], 2), round(g["c2"]["ms_per_step"], 2), "c5", round(g["c5"]["value"], 1))
PY
