#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over one C3 step: SQ issue/wait breakdown and
# L2 hit/miss per kernel. Outputs under gpurun_out/TAG/.
set -eo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_FLAT"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o c3 \
    -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-fresh-diag $BENCH_ARGS > "$OUT/p$i.log" 2>&1)
  find "$OUT/p$i" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc$i.csv" \;
done
python3 profiles/pmc_summary.py "$OUT"/pmc*.csv
