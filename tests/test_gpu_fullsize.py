"""The exact benched configurations, at their benched sizes, against the oracle.

bench.py searches C3 (256 MiB), C2 (1 GiB) and C4 (128 MiB per GPU) with the library's default policy
(prefix cache with sampled / derived levels, dedup-free builds, the lane-serial and live kernels,
spills) — paths the small differential tests only reach with knobs. Here the whole haystack is
searched exactly as bench.py does, with no FAC_* knob set, and ~32 random 32 KiB ranges of start
windows are re-searched by the oracle on halo slices: windows are independent (search.rs:533-575),
so search_raw's records for the windows starting in [a, b) are those of the slice [a, b + halo)
searched with windows (0, owned) — the halo (max_match_graphemes() + 2 graphemes, stream.rs:213-258
plus the text[j + 1] lookahead) keeps every state of those windows inside the slice. Every field
is compared, similarity bits and edit counts included.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from fuzzy_aho_corasick import workloads as W
from fuzzy_aho_corasick.engine import StagedHaystack
from oracle_harness import OracleEngine, PreparedText, graphemes

pytestmark = pytest.mark.gpu

SLICE = 32 << 10
N_SLICES = 32


def _workload(name, mib, vocab=50_000):
    nbytes = mib << 20
    if name == "c4":  # bench.py: the C2 engine on the seed-40 haystack
        return W.config("c4", nbytes, hay_seed=40, vocab=vocab)
    seed = {"c2": 2, "c3": 3}[name]
    return W.config(name, nbytes, seed=seed, hay_seed=seed + 1000, vocab=vocab)


def _after_space(data: bytes, p: int) -> int:
    """The byte after the next ' ' at or after p: a grapheme boundary whose segmentation needs no
    left context (the haystacks are words separated by ASCII spaces)."""
    q = data.find(b" ", p)
    return len(data) if q < 0 else q + 1


def _key(rows):
    return sorted((int(r[0]), int(r[1]), int(r[2]), int(np.float32(r[3]).view(np.uint32)), int(r[4]), int(r[5]),
                   int(r[6]), int(r[7]), int(r[8])) for r in rows)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,mib,vocab", [("c3", 256, 50_000), ("c4", 128, 50_000), ("c2", 1024, 50_000),
                                            ("c3", 256, None), ("c2", 1024, None)],
                         ids=["c3", "c4", "c2", "c3-fresh", "c2-fresh"])
def test_benched_config_sampled_windows_match_oracle(name, mib, vocab):
    """vocab None: every filler word fresh, SURVEY.md §8(d)'s generator literally (bench.py --vocab 0)."""
    wl = _workload(name, mib, vocab)
    data = wl.haystack
    eng = W.builder_for(wl).device(0).build(wl.patterns)
    staged = StagedHaystack(eng, data)
    recs, _ = staged.search_windows_records(wl.threshold)
    assert len(recs) > 0
    starts = recs["start"]
    order = np.argsort(starts, kind="stable")
    recs, starts = recs[order], starts[order]
    halo = (eng.max_match_graphemes() + 2) * 4 + 64  # bytes: at most 4 per grapheme here
    orc = OracleEngine(W.builder_for(wl), wl.patterns)
    rng = np.random.default_rng({"c2": 21, "c3": 31, "c4": 41}[name] + (0 if vocab else 100))
    picks = sorted(int(x) for x in rng.integers(0, len(data) - 2 * SLICE, size=N_SLICES))
    cases = []
    for p in picks:
        a = _after_space(data, p)
        b = _after_space(data, a + SLICE)
        e = min(len(data), _after_space(data, b + halo))
        cases.append((a, b, e))

    def oracle_slice(c):
        a, b, e = c
        pt = PreparedText(orc, data[a:e])
        owned = (b - a) if pt.ascii else len(graphemes(data[a:b].decode("utf-8")))
        rows = pt._run(wl.threshold, False, 0, owned, full=True)
        return [(s + a, en + a) + tuple(r) for (s, en, *r) in rows]

    with ThreadPoolExecutor(max_workers=min(16, len(os.sched_getaffinity(0)))) as ex:
        want = list(ex.map(oracle_slice, cases))
    total = 0
    for (a, b, e), w in zip(cases, want):
        lo, hi = np.searchsorted(starts, a, "left"), np.searchsorted(starts, b, "left")
        got = [(r["start"], r["end"], r["pattern_index"], r["similarity"], r["insertions"], r["deletions"],
                r["substitutions"], r["swaps"], r["edits"]) for r in recs[lo:hi]]
        gk, wk = _key(got), _key(w)
        assert gk == wk, f"{name}: windows starting in bytes [{a}, {b}): gpu {len(gk)} vs oracle {len(wk)} records; " \
                         f"first difference {next(((x, y) for x, y in zip(gk, wk) if x != y), None)}"
        total += len(wk)
    assert total > 0
