#!/bin/bash
# Round 6 final evidence, part 1 (final sources): GPU suite, smoke, PMC traffic of the C3 / C2 / C4 / C5
# steps stamped to these sources (profiles/traffic_*.json)
set -eo pipefail
bash profiles/gpu_evidence.sh r06final1 tests smoke pmc pmc2 pmc4 pmc5
