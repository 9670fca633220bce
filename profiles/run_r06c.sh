#!/bin/bash
# Round 6: tail by value into the beam selects (no scratch-resident tail), vcount in an SGPR, the build
# epilogue reading its table from LDS per pass -- prefix-cache / beam parity subset, then C3 and fresh-word C3.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06c
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 500 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-fresh-diag > "$OUT/c3_$i.json" 2> "$OUT/c3_$i.err"
done
timeout -k 10 200 python bench.py --steps 3 --vocab 0 --no-cpu-baseline --no-fresh-diag > "$OUT/c3fresh.json" 2> "$OUT/c3fresh.err"
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/c3*.json")):
    d = json.load(open(f))
    g = d["diagnostics"]
    print(f.split("/")[-1], "ms %.2f" % d["ms_per_step"], "cache %.2f" % g["prefix_cache_ms_per_step"], "lane %.2f" % g["lane_kernel_ms_per_step"], "wave %.2f" % g["search_kernel_ms_per_step"], "matches", g["matches_per_step"])
PY
