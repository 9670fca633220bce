"""search_stream called repeatedly in one process (round 6): per-call wall time, to see whether a
second stream of the same size runs slower than the first."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from fuzzy_aho_corasick import workloads as W  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
wl = W.config("c5", 1 << 30, seed=5)
engine = W.builder_for(wl).device(0).build(wl.patterns)
total = int(gib * (1 << 30))
for c in range(calls):
    hits = [0]
    t = time.perf_counter()
    n = engine.search_stream(bench._RepeatReader(wl.haystack, total), wl.threshold, lambda m: hits.__setitem__(0, hits[0] + 1))
    print("call %d: %.1f ms, %d bytes, %d matches" % (c, (time.perf_counter() - t) * 1e3, n, hits[0]), flush=True)
