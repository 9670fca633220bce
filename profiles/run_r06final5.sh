#!/bin/bash
# Round 6 final evidence, part 5: the whole GPU suite with the round's last tests, and smoke
set -eo pipefail
bash profiles/gpu_evidence.sh r06final5 tests smoke
