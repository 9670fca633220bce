#!/bin/bash
# Round 5: SQ counters of the final q-gram scan and verify (one C5 step, two passes)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ag
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES \
  --output-format csv -d "$OUT/p1" -o c5 -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/p1.log" 2>&1)
find "$OUT/p1" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc1.csv" \;
(cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/p2" -o c5 -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/p2.log" 2>&1)
find "$OUT/p2" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc2.csv" \;
python3 profiles/pmc_summary.py "$OUT"/pmc1.csv "$OUT"/pmc2.csv > "$OUT/summary.txt"
grep -A20 -E "^qgram" "$OUT/summary.txt" | head -50
