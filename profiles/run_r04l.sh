#!/bin/bash
# r04l: same-box comparison of library builds: round start (r04a), HEAD, HEAD + rare kernel arguments
# loaded on use (cold), each with its kernel timeline; parity subset on HEAD first
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r04l
mkdir -p "$OUT"
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fullsize.py -x -q \
  --timeout 500 --timeout-method thread -k "prefix_cache or lane_serial or dedup_free or differential_random or golden or c3" \
  > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in r04a head cold coldlw3 r04a head cold coldlw3; do
  lib=$L/libfac.so; [ $v = r04a ] && lib=$L/libfac_r04a.so; [ $v = cold ] && lib=$L/libfac_cold.so; [ $v = coldlw3 ] && lib=$L/libfac_cold_lw3.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag > "$OUT/b_$v.json" 2> "$OUT/b_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/b_$v.json'));g=d['diagnostics'];print('$v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
done
for v in head cold; do
  lib=$L/libfac.so; [ $v = cold ] && lib=$L/libfac_cold.so
  FAC_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-fresh-diag --vocab 0 --steps 3 > "$OUT/f_$v.json" 2> "$OUT/f_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/f_$v.json'));g=d['diagnostics'];print('fresh $v', round(d['ms_per_step'],1), 'cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
done
export TMPDIR=/tmp
for v in head cold; do
  lib=$L/libfac.so; [ $v = cold ] && lib=$L/libfac_cold.so
  (cd /tmp && FAC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$v" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt_$v.log" 2>&1)
  find "$OUT/kt_$v" -name '*kernel_trace.csv' -exec python3 "$ROOT/profiles/step_timeline.py" {} \; > "$OUT/timeline_$v.txt"
  rm -rf "$OUT/kt_$v"
  echo "== $v"; grep -E "rc_build|rc_count_kernel|rc_parent|lookup|lane_window|bfs_window" "$OUT/timeline_$v.txt"
done
cd "$ROOT"
BENCH_ARGS="--no-fresh-diag" bash profiles/ab_knobs.sh r04l_v "X=0" "FAC_BUILD_SMALL_L1=1" "FAC_LANE_POPS=64" "FAC_LANE_Q32=1 FAC_LANE_POPS=64" "FAC_RC_DEMAND=8"
