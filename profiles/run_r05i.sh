#!/bin/bash
# Round 5: fresh-word C3 (--vocab 0): one step's kernel timeline, the phase profile (libfac_prof.so)
# and the FAC_RC_DEBUG counters
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05i
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o fresh \
  -- python3 "$ROOT/bench.py" --vocab 0 --steps 2 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt.log" 2>&1)
find "$OUT/kt" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/fresh_timeline.txt"
grep -E "rc_build|bfs_window|lane_window|rc_lookup|rc_count" "$OUT/fresh_timeline.txt" | head -30
FAC_LIB=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib/libfac_prof.so timeout -k 10 300 python bench.py --vocab 0 --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/prof.json" 2> "$OUT/prof.err"
grep FAC_PROF "$OUT/prof.err" | cut -c1-900
FAC_DIAGNOSTICS=1 FAC_RC_DEBUG=1 timeout -k 10 300 python bench.py --vocab 0 --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/dbg.json" 2> "$OUT/dbg.err"
grep -E "^FAC_" "$OUT/dbg.err" | cut -c1-500
