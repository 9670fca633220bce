#!/bin/bash
# Round 5 final evidence, part 3 (after the q-gram scan / verify rewrite): GPU suite, smoke, the C5 line
# with its CPU baseline
set -eo pipefail
bash profiles/gpu_evidence.sh r05final3 tests smoke c5
