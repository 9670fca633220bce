#!/bin/bash
# r03af: C2 / C4 / C5 (full 12.5 GiB share, PMC traffic) lines and the fresh-word C3 / C2 lines at the
# round's final sources (same csrc as r03ac)
set -eo pipefail
OUT=gpurun_out/r03af; mkdir -p $OUT
bash profiles/gpu_evidence.sh r03af c2 c4 c5 pmc5 c5t
timeout -k 10 400 python bench.py --vocab 0 --no-cpu-baseline > $OUT/bench_c3_vocab0.json 2> $OUT/bench_c3_vocab0.err
cat $OUT/bench_c3_vocab0.json
timeout -k 10 400 python bench.py --config c2 --vocab 0 --no-cpu-baseline > $OUT/bench_c2_vocab0.json 2> $OUT/bench_c2_vocab0.err
cat $OUT/bench_c2_vocab0.json
