#!/bin/bash
# Round 5 final evidence, part 8 (after the 16-wave scan blocks): GPU suite, smoke, the C5 line with its CPU
# baseline, then PMC traffic of the C3 / C2 / C4 / C5 steps stamped to the final sources and the lines
# carrying it
set -eo pipefail
bash profiles/gpu_evidence.sh r05final8 tests smoke c5 pmc pmc2 pmc4 pmc5 c3t c2t c4t c5t
