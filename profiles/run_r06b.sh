#!/bin/bash
# Round 6: in-batch duplicates resolved in the window body (no batch cut) -- GPU suite, C3 A/B against
# the round-5 cut rule (FAC_DUP_CUT=1), and the phase profile with the epilogue split.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06b
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-fresh-diag > "$OUT/c3_new_$i.json" 2> "$OUT/c3_new_$i.err"
  FAC_DIAGNOSTICS=1 FAC_DUP_CUT=1 timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-fresh-diag > "$OUT/c3_cut_$i.json" 2> "$OUT/c3_cut_$i.err"
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/c3_*.json")):
    d = json.load(open(f))
    g = d["diagnostics"]
    print(f.split("/")[-1], "ms %.2f" % d["ms_per_step"], "cache %.2f" % g["prefix_cache_ms_per_step"], "wave %.2f" % g["search_kernel_ms_per_step"], "matches", g["matches_per_step"], "popped", g["states_popped_per_step"])
PY
FAC_LIB=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib/libfac_prof.so timeout -k 10 200 \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err"
grep FAC_PROF "$OUT/prof_c3.err" | tail -4
