#!/bin/bash
# box check: can torch see the GPU after the repo's HIP library has run?
set -o pipefail
timeout -k 5 120 python -c "
import sys; sys.path.insert(0, 'fuzzy-aho-corasick-rs_amd')
from fuzzy_aho_corasick import FuzzyAhoCorasickBuilder as B
e = B().build(['hello'])
print('fac ok', len(e.search('hello world')))
import torch; print('torch after fac: available', torch.cuda.is_available(), torch.cuda.device_count())
" 2>&1 | grep -v amdgpu.ids
