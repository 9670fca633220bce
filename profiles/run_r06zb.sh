#!/bin/bash
# Round 6: 5-gram screening of the q-gram pre-filter -- pre-filter / stream parity, C5 with and without it.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06zb
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards_streams.py tests/test_distributed.py -x -q \
  --timeout 600 --timeout-method thread -m gpu -k "qgram or prefilter or stream or bitap or c5" > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
export FAC_DIAGNOSTICS=1
for v in on off; do
  if [ $v = off ]; then export FAC_QG_NO5=1; else unset FAC_QG_NO5; fi
  timeout -k 10 400 python bench.py --config c5 --steps 2 --no-cpu-baseline > "$OUT/c5_$v.json" 2> "$OUT/c5_$v.err"
  python3 -c "import json; d=json.load(open('$OUT/c5_$v.json')); g=d['diagnostics']; print('c5 $v', '%.1f Gchars/s %.2f ms' % (d['value'], d['ms_per_step']), 'prefilter %.2f research %.2f matches %d' % (g['prefilter_ms_per_step'], g['research_kernel_ms_per_step'], g['matches_per_step']))"
done
unset FAC_QG_NO5
FAC_TIMING=1 timeout -k 10 300 python bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/c5_timing.json" 2> "$OUT/c5_timing.err"
grep "FAC_QGRAM text" "$OUT/c5_timing.err" | head -3
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o c5 \
  -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/kt.log" 2>&1)
f=$(find "$OUT/kt" -name 'c5_kernel_stats.csv' | head -1)
cp "$f" "$OUT/c5_kernel_stats.csv"
python3 - "$OUT/c5_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:6]:
    print(r["Name"][:70], r["Calls"], "%.3f ms total" % (float(r["TotalDurationNs"]) / 1e6))
PY
