#!/bin/bash
# Round 6: search_stream line (4 GiB) with the dense bitmaps on / list off / off -- where did 1.4 s go?
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06zh
mkdir -p "$OUT"
cd "$ROOT"
export FAC_DIAGNOSTICS=1
for v in on nolist off nocache; do
  unset FAC_RC_NO_DENSE FAC_RC_NO_DENSE_LIST FAC_NO_RC
  [ $v = nolist ] && export FAC_RC_NO_DENSE_LIST=1
  [ $v = off ] && export FAC_RC_NO_DENSE=1
  [ $v = nocache ] && export FAC_NO_RC=1
  timeout -k 10 300 python bench.py --config stream --gib 4 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/stream_$v.json" 2> "$OUT/stream_$v.err"
  python3 -c "import json; d=json.load(open('$OUT/stream_$v.json')); print('$v', '%.3f Gchars/s %.1f ms' % (d['value'], d['ms_per_step']))"
done
unset FAC_RC_NO_DENSE FAC_RC_NO_DENSE_LIST FAC_NO_RC
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o s \
  -- python3 "$ROOT/bench.py" --config stream --gib 1 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/kt.log" 2>&1)
f=$(find "$OUT/kt" -name 's_kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print("  ", r["Name"][:60], r["Calls"], "%.2f ms total" % (float(r["TotalDurationNs"]) / 1e6))
PY
