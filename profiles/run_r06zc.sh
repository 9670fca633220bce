#!/bin/bash
# Round 6: the 5-gram screen where it applies (every piece >= 5 symbols), and C5 after its gate.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06zc
mkdir -p "$OUT"
cd "$ROOT"
export FAC_DIAGNOSTICS=1 TMPDIR=/tmp
for v in on off; do
  if [ $v = off ]; then export FAC_QG_NO5=1; else unset FAC_QG_NO5; fi
  (cd /tmp && FAC_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$v" -o p \
    -- python3 "$ROOT/profiles/qg5_probe.py" > "$OUT/probe_$v.log" 2> "$OUT/probe_$v.err")
  cat "$OUT/probe_$v.log"
  grep "FAC_QGRAM text" "$OUT/probe_$v.err" | tail -1
  f=$(find "$OUT/kt_$v" -name 'p_kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:4]:
    print("  ", r["Name"][:60], r["Calls"], "%.3f ms avg" % (float(r["AverageNs"]) / 1e6))
PY
done
unset FAC_QG_NO5
timeout -k 10 400 python bench.py --config c5 --steps 2 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err"
python3 -c "import json; d=json.load(open('$OUT/c5.json')); g=d['diagnostics']; print('c5', '%.1f Gchars/s %.2f ms' % (d['value'], d['ms_per_step']), 'prefilter %.2f' % g['prefilter_ms_per_step'])"
