#!/bin/bash
# Knob sweep on C3 (diagnostics env knobs, FAC_DIAGNOSTICS=1): one bench line per setting.
# usage: bash profiles/sweep_c3.sh TAG "ENV1=a ENV2=b" "ENV3=c" ...   (each arg = one run; "" = defaults)
set -o pipefail
TAG=${1:?tag}
shift
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for setting in "$@"; do
  i=$((i + 1))
  env FAC_DIAGNOSTICS=1 $setting timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS \
    > "$OUT/run$i.json" 2> "$OUT/run$i.err" || { echo "run $i ($setting) failed"; tail -5 "$OUT/run$i.err"; exit 1; }
  python3 -c "
import json,sys
d=json.load(open('$OUT/run$i.json')); g=d['diagnostics']
print('%-40s %7.1f ms  cache %6.1f lane %5.1f wave %5.1f' % ('$setting' or 'defaults', d['ms_per_step'], g['prefix_cache_ms_per_step'], g['lane_kernel_ms_per_step'], g['search_kernel_ms_per_step']))"
done
