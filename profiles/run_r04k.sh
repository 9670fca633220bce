#!/bin/bash
# r04k: the round-start library (commit 39cd544, libfac_r04a.so) against HEAD on the same box, with
# one-step kernel timelines of each
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04k
mkdir -p "$OUT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
for v in old new old new; do
  lib=$L/libfac.so; [ $v = old ] && lib=$L/libfac_r04a.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/b_$v.json'));g=d['diagnostics'];print('$v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
done
export TMPDIR=/tmp
for v in old new; do
  lib=$L/libfac.so; [ $v = old ] && lib=$L/libfac_r04a.so
  (cd /tmp && FAC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$v" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt_$v.log" 2>&1)
  find "$OUT/kt_$v" -name '*kernel_trace.csv' -exec python3 "$ROOT/profiles/step_timeline.py" {} \; > "$OUT/timeline_$v.txt"
  rm -rf "$OUT/kt_$v"
  echo "== $v"; grep -E "rc_build|rc_count_kernel|lookup|lane_window|bfs_window" "$OUT/timeline_$v.txt"
done
