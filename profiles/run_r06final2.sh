#!/bin/bash
# Round 6 final evidence, part 2: the C3 (default, with the CPU baseline, the strong-scaling estimate and
# the C2 / C5 legs), C2, C4 and C5 lines carrying the traffic of part 1
set -eo pipefail
bash profiles/gpu_evidence.sh r06final2 c3t c2t c4t c5t
