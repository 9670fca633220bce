#!/bin/bash
# r03u: LDS-DMA probe, GPU parity subset with the snapshot prefetch, then A/B (prefetch vs none, lane knobs, canonical rule)
set -eo pipefail
OUT=gpurun_out/r03u; mkdir -p $OUT
timeout -k 5 60 ./profiles/probe/dma_test
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash profiles/ab_knobs.sh r03u "X=0" "FAC_LIB=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib/libfac_pfnb.so" "FAC_LIB=fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib/libfac_nopf.so" "FAC_LANE_Q32=1 FAC_LANE_POPS=128" "FAC_BEAM_CANONICAL=1" "FAC_RC_LEVELS=5,6,7" "FAC_NO_RC_L0=1"
