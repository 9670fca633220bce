#!/bin/bash
# Round 5: q-gram scan blocks of 16 waves sharing one bitmap (libfac_x_w16.so: 56 KB, 2 blocks = 32 waves
# per CU) against 8-wave blocks (default: 44 KB, 3 blocks = 24 waves per CU): pre-filter GPU tests,
# C5 line, candidates (FAC_TIMING) and the pre-filter kernel times from one traced step each
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ah
mkdir -p "$OUT"
export TMPDIR=/tmp
L=$ROOT/fuzzy-aho-corasick-rs_amd/fuzzy_aho_corasick/_lib
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "prefilter or qgram or bitap or stream or c5 or bytes or distributed or prefiltered" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in b17 w16; do
  lib=$L/libfac_x_$v.so; [ $v = b17 ] && lib=$L/libfac.so
  FAC_LIB=$lib FAC_DIAGNOSTICS=1 FAC_TIMING=1 timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c5_$v.json" 2> "$OUT/c5_$v.err"
  python3 -c "import json;d=json.load(open('$OUT/c5_$v.json'));g=d['diagnostics'];print('$v', round(d['value'],1), round(d['ms_per_step'],2), 'prefilter', round(g['prefilter_ms_per_step'],2), g['matches_per_step'])"
  grep -m1 FAC_QGRAM "$OUT/c5_$v.err" || true
  (cd /tmp && FAC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_$v" -o c5 \
    -- python3 "$ROOT/bench.py" --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/kt_$v.log" 2>&1)
  f=$(find "$OUT/kt_$v" -name '*kernel_stats.csv' | head -1); python3 - "$f" <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:2]:
    print('   ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3))
PY
done
