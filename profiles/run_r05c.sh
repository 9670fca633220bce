#!/bin/bash
# Round 5: family builds (rc_family_kernel), smaller main-pass chunks for few windows, the 16-position
# q-gram scan and 32-bit verify: the GPU suite, then the C3 (with the fresh-word diagnostic), C5 and C2 lines.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05c
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prefix_cache or differential or lane" > "$OUT/pytest_pc.log" 2>&1 || { tail -40 "$OUT/pytest_pc.log"; exit 1; }
tail -2 "$OUT/pytest_pc.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for c in c3 c5 c2; do
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  python3 -c "import json;d=json.load(open('$OUT/bench_$c.json'));g=d['diagnostics'];print('$c', round(d['value'],3), round(d['ms_per_step'],1), {k:(round(v,2) if isinstance(v,float) else v) for k,v in g.items() if k.endswith('ms_per_step') or k=='fresh_words'})"
done
