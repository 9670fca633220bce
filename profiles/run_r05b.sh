#!/bin/bash
# Round 5: the q-gram pre-filter rewrite (pass masks + host bitmap, batched verify loads): its GPU
# tests, the C5 line, kernel stats of one C5 step and the SQ split of the pre-filter kernels.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05b
mkdir -p "$OUT"
export TMPDIR=/tmp
#timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
#  -k "prefilter or bitap or qgram" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
#tail -2
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
python3 -c "import json;d=json.load(open('$OUT/bench_c5.json'));print(d['value'],d['ms_per_step'],d['diagnostics'])"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ks" -o c5 -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/ks.log" 2>&1)
find "$OUT/ks" -name '*kernel_stats.csv' -exec cp {} "$OUT/c5_kernel_stats.csv" \;
head -12 "$OUT/c5_kernel_stats.csv" | cut -c1-160
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES \
  --output-format csv -d "$OUT/p1" -o c5 -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/p1.log" 2>&1)
find "$OUT/p1" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc1.csv" \;
python3 profiles/pmc_summary.py "$OUT"/pmc1.csv 2>&1 | grep -A12 -E "qgram|bitap|runs_kernel" | head -60
