#!/usr/bin/env python3
"""Generate tests/golden/*.json: small seeded instances of BASELINE.json configs C1-C5 with the
expected raw matches computed by the CPU oracle (oracle/, itself pinned by the reference's own
assertions in tests/test_reference_behaviour.py and tests/test_host_and_oracle.py).

The reference (Rust) cannot run here, so these vectors are oracle outputs: they pin the GPU engine
and guard the oracle against regressions. The oracle's default restatement modes apply (edge order
= the transitions map's FxHasher + hashbrown order, beam = core's select_nth_unstable_by). Run from the repo root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "fuzzy-aho-corasick-rs_amd"), os.path.join(REPO, "tests")]

from fuzzy_aho_corasick import workloads as W  # noqa: E402
from oracle_harness import OracleEngine  # noqa: E402

SIZES = {"c1": 16384, "c2": 16384, "c3": 32768, "c4": 16384, "c5": 65536}
PATTERN_CAP = {}  # every config with its full pattern set (C3: all 10K patterns, beam 64)


def main():
    for name, nbytes in SIZES.items():
        w = W.config(name, nbytes)
        if name in PATTERN_CAP:
            w.patterns = w.patterns[: PATTERN_CAP[name]]
        # plant a few exact pattern copies so every fixture has matches
        extra = " ".join(w.patterns[:: max(1, len(w.patterns) // 8)][:8])
        hay = (w.haystack.decode("utf-8") + " " + extra).encode("utf-8")
        eng = OracleEngine(W.builder_for(w), w.patterns)
        rows = eng.raw_rows(hay, w.threshold, prefilter=w.prefilter)
        doc = {
            "config": name, "patterns": w.patterns, "haystack": hay.decode("utf-8"), "edits": w.edits,
            "beam": w.beam, "case_insensitive": w.case_insensitive, "threshold": w.threshold,
            "prefilter": w.prefilter,
            "expected": [[s, e, p, __import__("struct").unpack("<I", __import__("struct").pack("<f", sim))[0],
                          i, d, su, sw, ed] for (s, e, p, sim, i, d, su, sw, ed) in rows],
            "generator": "tests/golden/make_golden.py (oracle/ CPU restatement)",
        }
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(doc, f, ensure_ascii=False)
        print(name, len(w.patterns), len(hay), "bytes", len(rows), "matches")


if __name__ == "__main__":
    main()
