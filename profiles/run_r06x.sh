#!/bin/bash
# Round 6: dense bitmaps + the lookups' window list -- prefix-cache parity, then C2 / C3 with and without them.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06x
mkdir -p "$OUT"
cd "$ROOT"
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 500 --timeout-method thread \
  -k "dense or prefix_cache or differential or lane_serial or sampled or beamed" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 "$OUT/pytest_gpu.log"
export FAC_DIAGNOSTICS=1  # the env knobs (FAC_RC_NO_DENSE, FAC_RC_DEBUG) are read only with it
for v in on no4 off; do  # on: bitmaps + list; no4: without level 1's bitmap; off: neither
  for cfg in c2 c3; do
    unset FAC_RC_NO_DENSE FAC_RC_NO_DENSE_LIST FAC_RC_NO_DENSE4
    if [ $v = off ]; then export FAC_RC_NO_DENSE=1; fi
    if [ $v = no4 ]; then export FAC_RC_NO_DENSE4=1; fi
    timeout -k 10 300 python bench.py --config $cfg --steps 5 --no-cpu-baseline --no-fresh-diag > "$OUT/${cfg}_$v.json" 2> "$OUT/${cfg}_$v.err"
    python3 -c "import json; d=json.load(open('$OUT/${cfg}_$v.json')); g=d['diagnostics']; print('$cfg $v', '%.2f ms' % d['ms_per_step'], 'cache %.2f lane %.2f wave %.2f matches %d' % (g['prefix_cache_ms_per_step'], g['lane_kernel_ms_per_step'], g['search_kernel_ms_per_step'], g['matches_per_step']))"
  done
done
unset FAC_RC_NO_DENSE FAC_RC_NO_DENSE_LIST FAC_RC_NO_DENSE4
for cfg in c2 c3; do
  FAC_RC_DEBUG=1 timeout -k 10 300 python bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/${cfg}_debug.json" 2> "$OUT/${cfg}_debug.err"
  grep -E "FAC_LK|FAC_LANE" "$OUT/${cfg}_debug.err" > "$OUT/${cfg}_debug_lines.txt" || true
  head -2 "$OUT/${cfg}_debug_lines.txt"
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o c2 \
  -- python3 "$ROOT/bench.py" --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-fresh-diag > "$OUT/kt.log" 2>&1)
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/c2_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r["Name"][:60], r["Calls"], "%.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
