"""Recall of C3's canonical beam (SURVEY §7 hard part 1, Appendix A Q9).

The reference's beam (search.rs:577-589: select_nth_unstable_by + truncate) keeps the bw smallest
penalties, with ties at the cut and the survivors' order decided by Rust's selection algorithm and
hashbrown's edge order — not reproducible here. Oracle and GPU share one canonical rule instead
(DESIGN.md §2). This script measures what the beam costs in results at all: C3's beamed engine
(edits 2, beam 64, 10K patterns, case-insensitive Unicode) against the same engine without a beam,
on a slice of the C3 haystack, on the GPU. Reported: matches found only unbeamed (missing), only
beamed (extra), both; and over the common (start, end, pattern) keys the worst similarity loss.

usage: python profiles/beam_recall.py [MiB] > out.json
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fuzzy-aho-corasick-rs_amd"))

from fuzzy_aho_corasick import workloads as W  # noqa: E402
from fuzzy_aho_corasick.engine import StagedHaystack  # noqa: E402


def main():
    mib = float(sys.argv[1]) if len(sys.argv) > 1 else 16.0
    wl = W.config("c3", int(mib * (1 << 20)))
    res = {}
    for name, beam in (("beam64", 64), ("unbeamed", 0)):
        w = W.Workload(wl.name, wl.patterns, wl.haystack, wl.edits, beam, wl.case_insensitive, wl.threshold)
        eng = W.builder_for(w).device(0).build(w.patterns)
        st = StagedHaystack(eng, w.haystack)
        t = time.perf_counter()
        recs, stats = st.search_windows_records(w.threshold)
        dt = time.perf_counter() - t
        res[name] = ({(int(r["start"]), int(r["end"]), int(r["pattern_index"])): float(r["similarity"]) for r in recs},
                     dt, stats.states_popped + stats.states_cached)
    b, u = res["beam64"][0], res["unbeamed"][0]
    common = b.keys() & u.keys()
    worst = max((u[k] - b[k] for k in common), default=0.0)
    lower = sum(1 for k in common if b[k] < u[k])
    out = {
        "workload": f"c3 slice: first {len(wl.haystack)} bytes, {len(wl.patterns)} patterns, edits 2, threshold {wl.threshold}",
        "beamed_matches": len(b), "unbeamed_matches": len(u), "common": len(common),
        "missing_with_beam": len(u.keys() - b.keys()), "extra_with_beam": len(b.keys() - u.keys()),
        "recall": len(common) / max(1, len(u)),
        "common_with_lower_similarity": lower, "worst_similarity_loss": worst,
        "seconds": {"beam64": res["beam64"][1], "unbeamed": res["unbeamed"][1]},
        "states": {"beam64": res["beam64"][2], "unbeamed": res["unbeamed"][2]},
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
