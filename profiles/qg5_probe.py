"""5-gram screening probe (round 6): a C5-shaped block searched with a pre-filter whose pieces are all
>= 5 symbols (edits <= 1 without swaps: k <= 1, pieces of m / 2 >= 5), FAC_QG_NO5 unset / set.
Prints the candidate counts (FAC_TIMING line on stderr) and the pre-filter call's wall time."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fuzzy-aho-corasick-rs_amd"))
from fuzzy_aho_corasick import workloads  # noqa: E402
from fuzzy_aho_corasick.engine import FuzzyAhoCorasickBuilder, prefilter_windows  # noqa: E402
from fuzzy_aho_corasick.structs import FuzzyLimits  # noqa: E402

w = workloads.config("c5", 256 << 20, 5)
eng = FuzzyAhoCorasickBuilder().fuzzy(FuzzyLimits().edits(1).swaps(0)).build(w.patterns)
hay = w.haystack.decode("utf-8")
prefilter_windows(eng, hay[: 1 << 20], w.threshold)  # warm-up
for _ in range(2):
    t = time.perf_counter()
    n = len(prefilter_windows(eng, hay, w.threshold))
    print("windows", n, "call ms %.1f" % ((time.perf_counter() - t) * 1e3), "NO5" if os.environ.get("FAC_QG_NO5") else "5-gram", flush=True)
