#!/bin/bash
# Round 6: stream batches with arithmetic window bounds and one runs round trip; stream buffer compaction
# once per feed -- stream tests, C5 256 KiB and 1 GiB, search_stream line, C3 kernel trace + step timeline.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06e
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards_streams.py tests/test_distributed.py -m gpu -x -q --timeout 500 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py --config c5 --steps 3 --no-cpu-baseline > "$OUT/c5_256k.json" 2> "$OUT/c5_256k.err"
timeout -k 10 300 python bench.py --config c5 --steps 3 --window-kib 0 --no-cpu-baseline > "$OUT/c5_1g.json" 2> "$OUT/c5_1g.err"
timeout -k 10 300 python bench.py --config stream --steps 1 --gib 4 > "$OUT/stream.json" 2> "$OUT/stream.err"
python3 - "$OUT" <<'PY'
import json, sys
for f in ("c5_256k", "c5_1g", "stream"):
    d = json.load(open(f"{sys.argv[1]}/{f}.json"))
    print(f, "%.1f Gchars/s" % d["value"], "%.2f ms/step" % d["ms_per_step"], d.get("diagnostics"))
PY
bash profiles/gpu_evidence.sh r06e/kt kt > "$OUT/kt_stdout.txt" 2>&1 || { tail -20 "$OUT/kt_stdout.txt"; exit 1; }
cat gpurun_out/r06e/kt/c3_step_timeline.txt | tail -45
