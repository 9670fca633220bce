"""One shard of the C3 haystack (bench.py --shard's step: device staging of the shard + search +
records), `steps` steps after a warm-up -- for a kernel trace of the strong-scaling step.

    python profiles/shard_trace.py N R [steps] [keys]   (keys: the key part, fac_haystack_set_key_partition)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fuzzy-aho-corasick-rs_amd")]

import bench  # noqa: E402
import torch  # noqa: E402
from fuzzy_aho_corasick import workloads as W  # noqa: E402

n, r = int(sys.argv[1]), int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
keys = len(sys.argv) > 4 and sys.argv[4] == "keys"
wl = W.config("c3", 256 << 20, seed=3, hay_seed=1003)
eng = W.builder_for(wl).device(0).build(wl.patterns)
stream = torch.cuda.current_stream().cuda_stream
dt, w, k, b = bench._time_shard(eng, wl.haystack, n, r, 0, stream, steps, wl.threshold, keys=keys)
print(f"{'key part' if keys else 'shard'} {r} of {n}: {dt / steps * 1e3:.2f} ms per step, {w} windows, {k} records, {b} bytes")
