#!/bin/bash
# r04m: after reverting the interleaved count slots: round-start library vs HEAD on the same box, then
# HEAD's round-4 knobs one at a time, and HEAD's kernel timeline
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04m
mkdir -p "$OUT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
for v in r04a head r04a head; do
  lib=$L/libfac.so; [ $v = r04a ] && lib=$L/libfac_r04a.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/b_$v.json'));g=d['diagnostics'];print('$v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
done
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04m_v "X=0" "FAC_NO_BUILD_SMALL=1" "FAC_RC_CT_ENTRIES=1" "FAC_NO_BUILD_SMALL=1 FAC_RC_CT_ENTRIES=1" "FAC_RC_DEEPEST=1"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o c3 \
  -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt.log" 2>&1)
find "$OUT/kt" -name '*kernel_trace.csv' -exec python3 "$ROOT/profiles/step_timeline.py" {} \; > "$OUT/timeline_head.txt"
rm -rf "$OUT/kt"
grep -E "rc_build|rc_count_kernel|rc_parent|lookup|lane_window|bfs_window" "$OUT/timeline_head.txt"
