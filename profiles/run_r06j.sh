#!/bin/bash
# Round 6: same-box A/B of the C3 line, current sources against the r06c library (commit 8ae49ce).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06j
mkdir -p "$OUT"
cd "$ROOT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-fresh-diag > "$OUT/new_$i.json" 2> "$OUT/new_$i.err"
  FAC_LIB=$L/libfac_r06c.so timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-fresh-diag > "$OUT/old_$i.json" 2> "$OUT/old_$i.err"
done
python3 - "$OUT" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f)); g = d["diagnostics"]
    print(f.split("/")[-1], "ms %.2f" % d["ms_per_step"], "cache %.2f" % g["prefix_cache_ms_per_step"], "lane %.2f" % g["lane_kernel_ms_per_step"], "wave %.2f" % g["search_kernel_ms_per_step"], "stage %.2f" % g["staging_ms_per_step"])
PY
