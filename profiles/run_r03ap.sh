#!/bin/bash
# r03ap: the remaining lines at the HEAD sources: C3 end to end from host bytes, fresh-word C3 / C2
set -eo pipefail
OUT=gpurun_out/r03ap; mkdir -p $OUT
bash profiles/gpu_evidence.sh r03ap c3e2e
timeout -k 10 600 python bench.py --vocab 0 --no-cpu-baseline > $OUT/bench_c3_vocab0.json 2> $OUT/bench_c3_vocab0.err
cat $OUT/bench_c3_vocab0.json
timeout -k 10 600 python bench.py --config c2 --vocab 0 --no-cpu-baseline > $OUT/bench_c2_vocab0.json 2> $OUT/bench_c2_vocab0.err
cat $OUT/bench_c2_vocab0.json
