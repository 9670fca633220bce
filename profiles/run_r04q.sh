#!/bin/bash
# r04q: level-1 build alone vs beside the sampled counts (timelines); fresh-word runs: FAC_RC_DEBUG
# counters, then the live pass's early spill knob
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/timeline_c3.sh r04q "FAC_RC_ONE_STREAM=1" "FAC_RC_CGRID2=1" | grep -E "==|rc_count|rc_build|lookup|window_kernel"
BENCH_ARGS="--vocab 0" RC_DEBUG=1 bash profiles/ab_knobs.sh r04q_fd "X=0"
grep -E "FAC_RC|FAC_LK|FAC_LANE|FAC_LIVE" gpurun_out/r04q_fd/ab0.err | cut -c1-400
BENCH_ARGS="--vocab 0" bash profiles/ab_knobs.sh r04q_f "X=0" "FAC_LIVE_NQMAX=64" "FAC_LIVE_NQMAX=128"
