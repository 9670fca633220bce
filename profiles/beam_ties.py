"""How much C3's beamed results depend on the tie rules the reference leaves to its toolchain
(VERDICT r02 next #2a).

The reference's beam is `queue[q_idx..].select_nth_unstable_by(bw - 1, total_cmp)` + `truncate`
(search.rs:584-587) over a queue whose push order follows `Node.transitions` iteration order
(builder.rs:336-342). The oracle (CPU restatement, oracle/oracle.cpp) runs the C3 engine on a
prefix of the C3 haystack under each restatement mode:
  insertion+canonical  insertion edge order, keep the bw smallest by (penalty, queue position)
                       in queue order (the rule rounds 1-2 used on oracle and GPU)
  insertion+latest     the same, ties at the cut broken towards the latest queue position
  hashbrown+canonical  FxHasher + hashbrown iteration order, canonical beam
  hashbrown+select     FxHasher + hashbrown order, core's select_nth_unstable_by (the default now)
  hashbrown+select_r03 the same with round 3's defective early exit (index == mid after the
                       equal-to-ancestor split stopped the select; VERDICT r03 missing #1)
  unbeamed             no beam (recall reference)
and reports, against hashbrown+select, the (start, end, pattern) keys only one side has, keys
whose similarity differs, and keys whose edit-count fields differ.

usage: python profiles/beam_ties.py [MiB] [threads] > out.json   (CPU only)
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fuzzy-aho-corasick-rs_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from fuzzy_aho_corasick import workloads as W  # noqa: E402
import oracle_harness as OH  # noqa: E402


def run(wl, edge, beam_rule, beam, threads):
    OH.set_modes(edge, beam_rule)
    w = W.Workload(wl.name, wl.patterns, wl.haystack, wl.edits, beam, wl.case_insensitive, wl.threshold)
    eng = OH.OracleEngine(W.builder_for(w), w.patterns)
    pt = OH.PreparedText(eng, w.haystack)
    t = time.perf_counter()
    rows = pt.search(w.threshold, threads=threads, full=True)
    return {(r[0], r[1], r[2]): r[3:] for r in rows}, time.perf_counter() - t, pt.n


def diff(a, b):
    ka, kb = a.keys(), b.keys()
    common = ka & kb
    return {"only_here": len(ka - kb), "only_in_default": len(kb - ka),
            "similarity_differs": sum(1 for k in common if a[k][0] != b[k][0]),
            "edit_counts_differ": sum(1 for k in common if a[k][0] == b[k][0] and a[k][1:] != b[k][1:])}


def main():
    mib = float(sys.argv[1]) if len(sys.argv) > 1 else 16.0
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    wl = W.config("c3", int(mib * (1 << 20)))
    modes = {"hashbrown+select": (1, 2, 64), "hashbrown+select_r03": (1, 3, 64), "hashbrown+canonical": (1, 0, 64), "insertion+canonical": (0, 0, 64),
             "insertion+latest": (0, 1, 64), "unbeamed": (1, 2, 0)}
    res, secs = {}, {}
    for name, (e, r, bw) in modes.items():
        res[name], secs[name], n = run(wl, e, r, bw, threads)
        print(f"{name}: {len(res[name])} matches, {secs[name]:.1f} s", file=sys.stderr)
    OH.set_modes(1, 2)
    d = res["hashbrown+select"]
    out = {"workload": f"c3 prefix: {len(wl.haystack)} bytes, {n} graphemes, {len(wl.patterns)} patterns, edits 2, "
                       f"beam 64, threshold {wl.threshold}; oracle on {threads} threads",
           "matches": {k: len(v) for k, v in res.items()},
           "vs_hashbrown_select": {k: diff(v, d) for k, v in res.items() if k != "hashbrown+select"},
           "insertion+latest_vs_insertion+canonical": diff(res["insertion+latest"], res["insertion+canonical"]),
           "seconds": secs}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
