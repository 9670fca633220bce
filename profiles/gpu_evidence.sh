#!/bin/bash
# Round evidence on one MI355X (run through gpurun from the repo root):
#   bash profiles/gpu_evidence.sh TAG [what...]
# what: tests smoke c3 c3e2e c2 c4 c5 c5t kt pmc pmc5 pmc2 pmc4 c2t c4t c3t  (default: tests smoke c3 c2 c5 kt pmc). Outputs under gpurun_out/TAG/.
# Every GPU step has its own time limit; the script stops at the first failing step.
set -eo pipefail
TAG=${1:?tag}
shift
WHAT=${*:-tests smoke c3 c2 c5 kt pmc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
has() { [[ " $WHAT " == *" $1 "* ]]; }

if has tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
if has smoke; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  cat "$OUT/smoke.log"
fi
if has c3; then
  timeout -k 10 400 python bench.py > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
  cat "$OUT/bench_c3.json"
fi
if has c3e2e; then
  timeout -k 10 400 python bench.py --end-to-end --no-cpu-baseline > "$OUT/bench_c3_e2e.json" 2> "$OUT/bench_c3_e2e.err"
  cat "$OUT/bench_c3_e2e.json"
fi
if has c2; then
  timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
  cat "$OUT/bench_c2.json"
fi
if has c4; then
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
  cat "$OUT/bench_c4.json"
fi
if has c5; then  # one GPU's full 12.5 GiB share of the 100 GiB stream, CPU baseline included
  timeout -k 10 600 python bench.py --config c5 --steps 2 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
  cat "$OUT/bench_c5.json"
fi
export TMPDIR=/tmp
if has kt; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-fresh-diag $BENCH_ARGS > "$OUT/kt.log" 2>&1)
  find "$OUT/kt" -name '*kernel_stats.csv' -exec cp {} "$OUT/c3_kernel_stats.csv" \;
  find "$OUT/kt" -name '*kernel_trace.csv' -exec python3 profiles/step_timeline.py {} \; > "$OUT/c3_step_timeline.txt"
  head -20 "$OUT/c3_kernel_stats.csv"
  cat "$OUT/c3_step_timeline.txt"
fi
if has pmc; then
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o c3 \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --no-fresh-diag $BENCH_ARGS > "$OUT/pmc_$c.log" 2>&1)
    find "$OUT/pmc_$c" -name '*counter_collection.csv' -exec cp {} "$OUT/c3_pmc_$c.csv" \;
  done
  python3 profiles/make_traffic.py c3 256 2 "$OUT/c3_pmc_FETCH_SIZE.csv" "$OUT/c3_pmc_WRITE_SIZE.csv" "$(python3 -c "import bench; print(bench.sources_sha())")" > "$OUT/traffic.log"
  cp profiles/traffic_c3.json "$OUT/traffic_c3.json"
  head -c 1500 "$OUT/traffic.log"
fi
if has pmc5; then  # C5: one GPU's 12.5 GiB share of the 100 GiB stream
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc5_$c" -o c5 \
      -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc5_$c.log" 2>&1)
    find "$OUT/pmc5_$c" -name '*counter_collection.csv' -exec cp {} "$OUT/c5_pmc_$c.csv" \;
  done
  python3 profiles/make_traffic.py c5 102400 1 "$OUT/c5_pmc_FETCH_SIZE.csv" "$OUT/c5_pmc_WRITE_SIZE.csv" "$(python3 -c "import bench; print(bench.sources_sha())")" > "$OUT/traffic5.log"
  cp profiles/traffic_c5.json "$OUT/traffic_c5.json"
  head -c 1500 "$OUT/traffic5.log"
fi
for cfg in c2 c4; do  # pmc2 / pmc4: PMC traffic of the C2 (1 GiB) / C4 (128 MiB) line; c2t / c4t: the line after it
  mib=1024; [ $cfg = c4 ] && mib=128
  if has pmc${cfg#c}; then
    for c in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc${cfg}_$c" -o $cfg \
        -- python3 "$ROOT/bench.py" --config $cfg --steps 2 --warmup 0 --no-cpu-baseline --no-fresh-diag > "$OUT/pmc${cfg}_$c.log" 2>&1)
      find "$OUT/pmc${cfg}_$c" -name '*counter_collection.csv' -exec cp {} "$OUT/${cfg}_pmc_$c.csv" \;
    done
    python3 profiles/make_traffic.py $cfg $mib 2 "$OUT/${cfg}_pmc_FETCH_SIZE.csv" "$OUT/${cfg}_pmc_WRITE_SIZE.csv" "$(python3 -c "import bench; print(bench.sources_sha())")" > "$OUT/traffic_$cfg.log"
    cp profiles/traffic_$cfg.json "$OUT/traffic_$cfg.json"
    head -c 600 "$OUT/traffic_$cfg.log"
  fi
  if has ${cfg}t; then  # with the CPU baseline and the traffic just measured
    timeout -k 10 400 python bench.py --config $cfg > "$OUT/bench_${cfg}_traffic.json" 2> "$OUT/bench_${cfg}_traffic.err"
    cat "$OUT/bench_${cfg}_traffic.json"
  fi
done
if has c5t; then  # after traffic_c5.json exists
  timeout -k 10 600 python bench.py --config c5 --steps 2 > "$OUT/bench_c5_traffic.json" 2> "$OUT/bench_c5_traffic.err"
  cat "$OUT/bench_c5_traffic.json"
fi
if has c3t; then  # bench after traffic.json exists: the line carries roofline.traffic
  timeout -k 10 400 python bench.py > "$OUT/bench_c3_traffic.json" 2> "$OUT/bench_c3_traffic.err"
  cat "$OUT/bench_c3_traffic.json"
fi
echo "evidence $TAG done"
