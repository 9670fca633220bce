#!/bin/bash
# Round 5 final check: GPU suite and smoke on the library rebuilt from the final sources
set -eo pipefail
bash profiles/gpu_evidence.sh r05final7 tests smoke
