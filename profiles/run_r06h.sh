#!/bin/bash
# Round 6: key-split strong scaling (fac_haystack_set_key_partition) -- its GPU test, then the default bench
# line (strong_emulated for shards and keys, C2 / C5 / fresh-word legs).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06h
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards_streams.py -x -q --timeout 500 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 600 python bench.py --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
python3 - "$OUT" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/bench_c3.json"))
g = d["diagnostics"]
print("c3 %.3f Gchars/s %.2f ms" % (d["value"], d["ms_per_step"]))
for k in ("shards", "keys"):
    print(k, {n: (round(v["max_rank_ms"], 2), round(v["predicted_speedup"], 2)) for n, v in g["strong_emulated"][k].items()})
print("fresh", round(g["fresh_words"]["ms_per_step"], 1), "c2", round(g["c2"]["value"], 2), "c5", round(g["c5"]["value"], 1))
PY
