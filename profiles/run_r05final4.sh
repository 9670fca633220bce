#!/bin/bash
# Round 5 final evidence, part 4: PMC traffic of the C3 / C2 / C4 / C5 steps stamped to the final
# sources, then the lines carrying it
set -eo pipefail
bash profiles/gpu_evidence.sh r05final4 pmc pmc2 pmc4 pmc5 c3t c2t c4t c5t
