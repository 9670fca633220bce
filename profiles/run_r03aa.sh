#!/bin/bash
# r03aa: clean phase profile (no FAC_RC_DEBUG counters) with prologue / flush / build-epilogue /
# group-setup / wave-lifetime slots
set -eo pipefail
OUT=gpurun_out/r03aa; mkdir -p $OUT
L=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
FAC_DIAGNOSTICS=1 FAC_LIB=$L/libfac_prof.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof.json 2> $OUT/prof.err
grep -E "FAC_PROF" $OUT/prof.err | tail -4
python3 -c "import json;d=json.load(open('$OUT/prof.json'));g=d['diagnostics'];print(round(d['ms_per_step'],1),'ms cache', round(g['prefix_cache_ms_per_step'],1), 'lane', round(g['lane_kernel_ms_per_step'],1), 'wave', round(g['search_kernel_ms_per_step'],1))"
