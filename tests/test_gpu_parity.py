"""GPU engine vs CPU oracle on identical seeded inputs (bit-exact spans, pattern ids, similarity
bits and edit counts). Mirrors the reference's own differential fuzz (prefilter.rs:441-546:
xorshift Rng, random vocab/filler haystacks, edits 0..=2, random case-insensitivity, thresholds
0.6-0.9) and widens it to the options the hot path has (beam, per-pattern limits, penalties,
min_symbol_similarity, custom similarity, Unicode, empty/edge inputs)."""
import pytest

from fuzzy_aho_corasick import (FuzzyAhoCorasickBuilder as B, FuzzyLimits as L, FuzzyPenalties, Pattern,
                                SearchOptions as O, Similarity)
from oracle_harness import OracleEngine

pytestmark = pytest.mark.gpu


class Rng:  # prefilter.rs:441-452
    def __init__(self, s):
        self.s = s

    def next(self):
        x = self.s
        x ^= (x << 13) & 0xFFFFFFFFFFFFFFFF
        x ^= x >> 7
        x ^= (x << 17) & 0xFFFFFFFFFFFFFFFF
        self.s = x
        return x


def rows(ms):
    return sorted((m.start, m.end, m.pattern_index, m.sim_bits(), m.insertions, m.deletions, m.substitutions,
                   m.swaps, m.edits) for m in ms)


def compare(builder, patterns, hay, thr, prefilter=False):
    gpu = builder.build(patterns)
    orc = OracleEngine(builder, patterns)
    if prefilter:
        g = gpu.with_prefilter().search(hay, O().threshold(thr))
        o = orc.with_prefilter().search(hay, O().threshold(thr))
    else:
        g = gpu.search(hay, O().threshold(thr))
        o = orc.search(hay, O().threshold(thr))
    gr, orr = rows(g), rows(o)
    assert gr == orr, f"patterns={patterns!r} hay={hay!r} thr={thr} prefilter={prefilter}\n gpu={gr}\n orc={orr}"
    return len(gr)


ASCII_VOCAB = ["hello", "world", "vestibulum", "abc", "lorem", "cell", "saddam", "hussein", "ab", "x"]
ASCII_FILLER = ["a", "b", "c", "d", "e", " ", "1", "o", "0", "l", "S", "H"]
UNI_VOCAB = ["café", "naïve", "Ωμέγα", "Москва", "señor", "école", "résumé"]
UNI_FILLER = ["a", "é", "ñ", "ω", "м", " ", "o", "0", "é", "Ω", "\r\n", "Σ"]
# code points beyond the BMP: swaps there take the two-lookup path (GT_SWAP entries are BMP-only)
ASTRAL_VOCAB = ["a😀b", "𝒜bc", "𐍈𐌹𐍈", "x😀y😀", "hello", "b𝒜a"]
ASTRAL_FILLER = ["😀", "𝒜", "a", "b", " ", "𐍈", "c", "x", "𐌹", "y"]


def random_case(rng, vocab, filler, allow_beam=True, allow_limits=True):
    npat = 1 + rng.next() % 4
    pats = [vocab[rng.next() % len(vocab)] for _ in range(npat)]
    edits = rng.next() % 4
    b = B().case_insensitive(rng.next() & 1 == 0)
    mode = rng.next() % 6
    if edits > 0 and mode != 5:
        b = b.fuzzy(L().edits(edits))
    if mode == 5 and allow_limits:  # per-type / per-pattern limits -> the 255 path
        b = b.fuzzy(L().insertions(rng.next() % 2).deletions(rng.next() % 2).substitutions(rng.next() % 2)
                    .swaps(rng.next() % 2))
        pats = [Pattern(p).fuzzy(L().edits(rng.next() % 3)) if rng.next() % 2 else p for p in pats]
    if rng.next() % 5 == 0:
        b = b.penalties(FuzzyPenalties.default().with_swap(0.6).with_insertion(0.5).with_deletion(0.8))
    if allow_beam and rng.next() % 4 == 0:
        b = b.beam_width(1 + rng.next() % 12)
    if rng.next() % 7 == 0:
        b = b.min_symbol_similarity(0.3)
    hay = ""
    for _ in range(rng.next() % 60):
        if rng.next() % 7 == 0:
            w = pats[rng.next() % len(pats)]
            hay += (w if isinstance(w, str) else w.pattern) + " "
        else:
            hay += filler[rng.next() % len(filler)]
    thr = 0.6 + (rng.next() % 4) * 0.1 if rng.next() % 5 else 0.0
    return b, pats, hay, thr


@pytest.mark.parametrize("root_cache", ["off", "k4", "k2+k4", "k3+k8"])
@pytest.mark.parametrize("per_edge_only", [False, True])
@pytest.mark.parametrize("seed,vocab,filler", [
    (0x1234_5678_9abc_def1, ASCII_VOCAB, ASCII_FILLER),
    (0xdead_beef_0bad_f00d, UNI_VOCAB, UNI_FILLER),
    (0x0a57_2a1c_0de5_51de, ASTRAL_VOCAB, ASTRAL_FILLER),
])
def test_differential_random(seed, vocab, filler, per_edge_only, root_cache, monkeypatch):
    """per_edge_only: FAC_NO_FAST disables the O(1) goto-table expansion, so the per-edge unit
    path is checked on every state as well. root_cache: the root-pop cache off, or forced on for
    every search with 4-char keys (it is normally used from 4096 windows on, with the longest key
    that still gives 8 windows per snapshot)."""
    if per_edge_only:
        monkeypatch.setenv("FAC_NO_FAST", "1")
    if root_cache == "off":
        monkeypatch.setenv("FAC_NO_RC", "1")
    else:  # "kA" one level of A-char keys; "kA+kB": level 2 with B-char keys for every sampled key
        levels = root_cache.split("+")
        monkeypatch.setenv("FAC_RC_MIN", "1")
        monkeypatch.setenv("FAC_RC_K", levels[0][1:])
        if len(levels) == 2:
            for k, v in (("FAC_RC_K2", levels[1][1:]), ("FAC_RC_MIN2", "1"), ("FAC_RC_STRIDE2", "1"),
                         ("FAC_RC_T2", "1")):
                monkeypatch.setenv(k, v)
        else:
            monkeypatch.setenv("FAC_RC_K2", "0")
    rng = Rng(seed)
    total = 0
    for _ in range(150):
        b, pats, hay, thr = random_case(rng, vocab, filler)
        total += compare(b, pats, hay, thr)
    assert total > 0


@pytest.mark.parametrize("sel_limit", ["16", "1", "0"])
def test_beam_select_restatement(sel_limit, monkeypatch):
    """The beam cut is core's select_nth_unstable_by restated (search.rs:584-587; oracle.cpp rsel,
    search_kernels.hip beam_select): dense ties (many equal penalties), widths 1 (min_index), up to 8
    (insertion sort of <= 16 pending) and beyond (pivots, partitions, the equal-to-ancestor split),
    with every window searched from the root and with the prefix cache forced on. sel_limit lowers
    select.rs's 16 partition rounds on both sides so median_of_medians runs too."""
    import oracle_harness as OH
    monkeypatch.setenv("FAC_SEL_LIMIT", sel_limit)
    OH.set_modes(sel_limit=int(sel_limit))
    try:
        rng = Rng(0x5EED0BEA)
        words = ["abcab", "bacab", "cabba", "abcba", "aabbc", "ccab", "bbca", "acbcab", "cbacbab", "abab"]
        for t in range(24):
            pats = [words[rng.next() % len(words)] + "abc"[rng.next() % 3] for _ in range(6 + rng.next() % 20)]
            hay = "".join("abc "[rng.next() % 4] for _ in range(150 + rng.next() % 250))
            bw = [1, 2, 3, 5, 8, 9, 13, 21, 40][t % 9]
            if t % 2:
                monkeypatch.setenv("FAC_RC_MIN", "1")
            else:
                monkeypatch.setenv("FAC_NO_RC", "1")
            compare(B().fuzzy(L().edits(2 + t % 2)).beam_width(bw), pats, hay, 0.3 + 0.1 * (t % 4))
            monkeypatch.delenv("FAC_RC_MIN", raising=False)
            monkeypatch.delenv("FAC_NO_RC", raising=False)
    finally:
        OH.set_modes(sel_limit=16)


@pytest.mark.parametrize("seed,vocab,filler", [
    (0x1234_5678_9abc_def1, ASCII_VOCAB, ASCII_FILLER),
    (0xdead_beef_0bad_f00d, UNI_VOCAB, UNI_FILLER),
])
def test_prefilter_differential(seed, vocab, filler):
    """Prefiltered::search == engine.search (prefilter.rs:467-546), GPU vs oracle, both paths."""
    rng = Rng(seed ^ 0x55)
    for _ in range(120):
        b, pats, hay, thr = random_case(rng, vocab, filler, allow_beam=False)
        n = compare(b, pats, hay, thr, prefilter=True)
        gpu = b.build(pats)
        full = rows(gpu.search(hay, O().threshold(thr)))
        pf = rows(gpu.with_prefilter().search(hay, O().threshold(thr)))
        assert [r[:4] for r in full] == [r[:4] for r in pf]
        assert len(pf) == n


@pytest.mark.parametrize("seed,vocab,filler", [
    (0x1234_5678_9abc_def1, ASCII_VOCAB, ASCII_FILLER),
    (0xdead_beef_0bad_f00d, UNI_VOCAB, UNI_FILLER),
])
def test_bitap_windows_match_reference_merge(seed, vocab, filler):
    """GPU bitap + run extraction == bitap_windows + sort + merge (prefilter.rs:319-342), and is
    deterministic across repeated calls."""
    from fuzzy_aho_corasick.engine import prefilter_windows
    rng = Rng(seed ^ 0x77)
    for _ in range(120):
        b, pats, hay, thr = random_case(rng, vocab, filler, allow_beam=False)
        gpu = b.build(pats)
        orc = OracleEngine(b, pats)
        want = orc.prefilter_windows(hay, thr)
        for _rep in range(3):
            got = prefilter_windows(gpu, hay, thr)
            assert got == want, f"patterns={pats!r} hay={hay!r} thr={thr}\n gpu={got}\n orc={want}"


@pytest.mark.parametrize("qgram", [True, False])
@pytest.mark.parametrize("long_patterns", [False, True])
def test_bitap_packed_words_match_reference(long_patterns, qgram, monkeypatch):
    """Many patterns packed several to an automaton word (first-fit by edit budget): windows equal
    the oracle's per-pattern bitap_windows + merge (prefilter.rs:319-342, 410-435). Lengths 1..20
    (32-bit words) or 1..60 (64-bit words), mixed weights and per-pattern edit limits (several k
    groups), planted fuzzy copies. qgram: patterns whose k + 1 pieces hold >= 3 symbols take the
    pigeonhole q-gram scan + per-candidate verification (the others the packed full scan); off: every
    pattern the full scan."""
    from fuzzy_aho_corasick.engine import prefilter_windows
    if not qgram:
        monkeypatch.setenv("FAC_NO_QGRAM", "1")
    rng = Rng(0x5EED_B17A_9ACC_0001 ^ int(long_patterns))
    alpha = "abcdefghij"
    top = 60 if long_patterns else 20
    pats = []
    for i in range(300):
        w = "".join(alpha[rng.next() % len(alpha)] for _ in range(1 + rng.next() % top))
        p = Pattern(w).with_weight(0.7 + (rng.next() % 7) * 0.1)
        if rng.next() % 3 == 0:
            p = p.fuzzy(L().edits(rng.next() % 3))
        pats.append(p)
    hay = []
    for _ in range(400):
        if rng.next() % 4 == 0:
            w = list(pats[rng.next() % len(pats)].pattern)
            if w and rng.next() % 2:
                w[rng.next() % len(w)] = alpha[rng.next() % len(alpha)]
            hay.append("".join(w))
        else:
            hay.append("".join(alpha[rng.next() % len(alpha)] for _ in range(1 + rng.next() % 12)))
    hay = " ".join(hay)
    b = B().fuzzy(L().edits(2))
    gpu = b.build(pats)
    orc = OracleEngine(b, pats)
    for thr in (0.75, 0.85, 0.95):
        want = orc.prefilter_windows(hay, thr)
        got = prefilter_windows(gpu, hay, thr)
        assert got == want, f"thr={thr}: {len(got)} vs {len(want)} windows"
    compare(b, pats, hay, 0.85, prefilter=True)


def test_qgram_prefilter_c5_slice(monkeypatch):
    """C5-shaped stream block (1K patterns of 10-16, threshold 0.85, k from k_for): merged bitap
    windows of the q-gram path == the packed full scan (4 MiB) == the oracle's bitap_windows + merge
    (first 192 KiB), and the pre-filtered search equals on the slice."""
    from fuzzy_aho_corasick import workloads
    from fuzzy_aho_corasick.engine import prefilter_windows
    w = workloads.config("c5", 4 << 20, 5)
    b = workloads.builder_for(w)
    gpu = b.build(w.patterns)
    hay = w.haystack.decode("utf-8")
    got = prefilter_windows(gpu, hay, w.threshold)
    monkeypatch.setenv("FAC_NO_QGRAM", "1")
    full = prefilter_windows(gpu, hay, w.threshold)
    assert got and got == full
    small = hay[: 192 << 10]
    assert prefilter_windows(gpu, small, w.threshold) == OracleEngine(b, w.patterns).prefilter_windows(small, w.threshold)
    monkeypatch.delenv("FAC_NO_QGRAM")
    assert prefilter_windows(gpu, small, w.threshold) == OracleEngine(b, w.patterns).prefilter_windows(small, w.threshold)


@pytest.mark.parametrize("ci", [False, True])
def test_qgram_bytes_mode_matches_ids_and_full_scan(ci, monkeypatch):
    """Every pattern on the q-gram path of an ASCII text: the scan and verify read the haystack's bytes
    (grams keyed by case-folded bytes, symbol ids looked up per candidate) instead of a transcoded id
    buffer. Windows == the id-buffer q-gram path (FAC_QGRAM_IDS) == the packed full scan == the oracle's
    bitap_windows + merge (prefilter.rs:319-342), mixed-case text, and the pre-filtered search equals the
    plain one (prefilter.rs:467-546)."""
    from fuzzy_aho_corasick.engine import prefilter_windows
    rng = Rng(0xB17E_5_0DE ^ int(ci))
    alpha = "abcdefghijklmnopqrstuvwxyz"
    pats = ["".join(alpha[rng.next() % 26] for _ in range(12 + rng.next() % 5)) for _ in range(60)]
    words = []
    for _ in range(3000):
        if rng.next() % 5 == 0:
            w = list(pats[rng.next() % len(pats)])
            w[rng.next() % len(w)] = alpha[rng.next() % 26]
        else:
            w = [alpha[rng.next() % 26] for _ in range(2 + rng.next() % 10)]
        words.append("".join(c.upper() if rng.next() % 3 == 0 else c for c in w))
    hay = " ".join(words) + "."
    b = B().case_insensitive(ci).fuzzy(L().edits(2))
    gpu = b.build(pats)
    orc = OracleEngine(b, pats)
    for thr in (0.8, 0.9):
        got = prefilter_windows(gpu, hay, thr)
        monkeypatch.setenv("FAC_QGRAM_IDS", "1")
        ids = prefilter_windows(gpu, hay, thr)
        monkeypatch.setenv("FAC_NO_QGRAM", "1")
        full = prefilter_windows(gpu, hay, thr)
        monkeypatch.delenv("FAC_QGRAM_IDS")
        monkeypatch.delenv("FAC_NO_QGRAM")
        assert got and got == ids == full == orc.prefilter_windows(hay, thr)
        for cut in (1, 5, 13):  # other text lengths: the last sixteens read byte by byte up to the end
            sub = hay[:len(hay) - cut]
            assert prefilter_windows(gpu, sub, thr) == orc.prefilter_windows(sub, thr)
    assert rows(gpu.with_prefilter().search(hay, O().threshold(0.8))) == rows(gpu.search(hay, O().threshold(0.8)))


def test_qgram_candidate_regions_overflow(monkeypatch):
    """Candidates beyond a scan block's region of the list (1/16 of its positions) go to the overflow
    list, and an overflowing overflow list is regrown and the scan re-run: runs of 'a' (3-18) between
    other letters, against patterns whose pieces start with "aaa" / "aaaa", make ~36 candidates per
    run position (~1.5 M in all, past the first 1 Mi-entry overflow list: every block's first
    reservation overflows); with "a" * 16 alone (4 entries per gram: 256 per queue drain) the regions
    fill part way before overflowing.
    Windows == the packed full scan == the oracle."""
    from fuzzy_aho_corasick.engine import prefilter_windows
    rng = Rng(0x0F10_0D)
    pats = ["a" * L for L in range(10, 17)] + ["a" * L + "b" + "a" * (13 - L) for L in range(5, 10)]
    parts, n = [], 0
    while n < 800_000:
        s = "".join("bcdefghij"[rng.next() % 9] for _ in range(10 + rng.next() % 50)) + "a" * (3 + rng.next() % 16)
        parts.append(s)
        n += len(s)
    hay = "".join(parts)
    b = B().fuzzy(L().edits(2))
    for sub in (pats, pats[6:7]):
        gpu = b.build(sub)
        orc = OracleEngine(b, sub)
        got = prefilter_windows(gpu, hay, 0.8)
        monkeypatch.setenv("FAC_NO_QGRAM", "1")
        full = prefilter_windows(gpu, hay, 0.8)
        monkeypatch.delenv("FAC_NO_QGRAM")
        assert got and got == full == orc.prefilter_windows(hay, 0.8)


def test_edge_inputs():
    b = B().fuzzy(L().edits(2))
    compare(b, ["abc"], "", 0.0)                      # empty haystack
    compare(b, [], "hello", 0.0)                      # no patterns
    compare(b, [""], "ab", 0.0)                        # empty pattern: NaN similarity kept (Q7)
    compare(b, ["a"], "a", 0.0)                        # 1-grapheme pattern, deletion-only empty spans (Q4)
    compare(B(), ["JOINT STOCK COMPANY", "STOCK"], "JOINT STOCK COMPANY GAZPROM", 0.8)  # Q1
    compare(B().fuzzy(L().edits(1)), ["ab\r\ncd"], "xx ab\r\ncd yy é", 0.5)           # Q3 unicode \r\n
    compare(B().fuzzy(L().edits(1)), ["ab\r\ncd"], "xx ab\r\ncd yy", 0.5)             # Q3 ascii \r\n
    compare(B().case_insensitive(True).fuzzy(L().edits(1)), ["ÉCOLE", "école"], "école école ÉCOLE", 0.5)
    compare(B().fuzzy(L().edits(1)), [("heavy", 2.0), ("light", 0.5)], "heavy light hevy lihgt", 0.5)
    sim = Similarity.from_map({("a", "b"): 0.9, ("b", "a"): 0.9, ("é", "e"): 0.8, ("ω", "o"): 0.5})
    compare(B().fuzzy(L().edits(1)).similarity(sim), ["bab", "cafe", "omega"], "aab café ωmega", 0.6)


def test_long_haystack_windows():
    """Many windows spanning several kernel chunks; exercises the grid-stride loop."""
    rng = Rng(77)
    words = ["needle", "haystack", "fuzzy", "automaton"]
    text = " ".join(words[rng.next() % 4][: 3 + rng.next() % 6] + "xyz"[rng.next() % 3] for _ in range(3000))
    compare(B().fuzzy(L().edits(1)), words, text, 0.7)
    compare(B().fuzzy(L().edits(2)).beam_width(8), words, text, 0.7)


def _staged_vs_oracle(builder, patterns, hay, thr):
    gpu = builder.build(patterns)
    got, st = gpu.stage(hay.encode("utf-8")).search_windows(thr)
    want = OracleEngine(builder, patterns).raw_rows(hay, thr)
    assert sorted(got) == sorted(want)
    return st, len(want)


def test_frontier_spill_unbeamed():
    """Runs of one letter against one-letter patterns: duplicate states explode, the dedup-free
    unbeamed variant overflows its ring, and those windows are re-run on the dedup variants."""
    rng = Rng(5)
    hay = "".join("aaaaaaaaaaaaaaaa" if rng.next() % 3 else "ab" for _ in range(40))
    st, n = _staged_vs_oracle(B().fuzzy(L().edits(3)), ["aaaaaaaaaa", "aaaab", "baaaaaaaa"], hay, 0.5)
    assert n > 0 and st.retries > 0


@pytest.mark.parametrize("beam_vcap", ["256", "512"])
def test_frontier_spill_beamed(monkeypatch, beam_vcap):
    """Beamed searches whose windows fill the dedup table (oracle: up to 456 keys per window):
    spilled windows are re-run on a larger variant with results identical to the oracle; and a
    C3-shaped slice with the table first sized `beam_vcap`."""
    from fuzzy_aho_corasick import workloads
    monkeypatch.setenv("FAC_BEAM_VCAP", beam_vcap)
    rng = Rng(5)
    hay = "".join("aaaaaaaaaaaaaaaa" if rng.next() % 3 else "ab" for _ in range(40))
    st, n = _staged_vs_oracle(B().fuzzy(L().edits(3)).beam_width(64), ["aaaaaaaaaa", "aaaab", "baaaaaaaa"], hay, 0.5)
    assert n > 0 and st.retries > 0
    w = workloads.config("c3", 24 << 10, 3)
    st, n = _staged_vs_oracle(workloads.builder_for(w), w.patterns, w.haystack.decode("utf-8"), w.threshold)
    assert n > 0


def test_frontier_beyond_2048_states():
    """Windows whose distinct-state count (oracle: up to 3038 keys at edits 5) exceeds the 2048-entry
    table: the spill ladder ends on the one-wave-per-CU (4096, 4096) variant, unbeamed and with a
    512 beam (whose 2x-beam trigger already needs the 2048 ring)."""
    pats = ["a" * 12, "ab" * 6, "b" * 12, "ba" * 6]
    hay = "ab" * 20 + "a" * 20 + "b" * 20
    st, n = _staged_vs_oracle(B().fuzzy(L().edits(5)), pats, hay, 0.3)
    assert n > 0 and st.retries > 0
    st, n = _staged_vs_oracle(B().fuzzy(L().edits(5)).beam_width(512), pats, hay, 0.3)
    assert n > 0 and st.retries > 0


def test_frontier_capacity_is_loud():
    """Edits 6 (oracle: 5706 distinct keys in a window) runs past the (4096, 4096) table onto the
    dedup-free 8192 ring; if even that overflows, the search fails with FAC_E_CAPACITY instead of
    returning a partial result."""
    from fuzzy_aho_corasick.structs import DeviceError
    pats = ["a" * 12, "ab" * 6, "b" * 12, "ba" * 6]
    hay = "ab" * 20 + "a" * 20 + "b" * 20
    try:
        _staged_vs_oracle(B().fuzzy(L().edits(6)), pats, hay, 0.3)
    except DeviceError as exc:
        assert exc.code == 105, exc


@pytest.mark.parametrize("variant", ["0,128", "0,256", "0,512", "256,256", "512,256", "512,512", "1024,1024",
                                     "2048,2048", "4096,4096", "0,8192"])
def test_every_frontier_variant(monkeypatch, variant):
    """Each LDS frontier variant (dedup table x queue ring) gives oracle-identical results."""
    monkeypatch.setenv("FAC_VARIANT", variant)
    rng = Rng(0xabcdef)
    words = ["needle", "haystack", "fuzzy", "automaton", "école", "Москва"]
    text = " ".join(words[rng.next() % 6][: 3 + rng.next() % 6] + "xyzé"[rng.next() % 4] for _ in range(600))
    _staged_vs_oracle(B().fuzzy(L().edits(2)), words, text, 0.6)
    _staged_vs_oracle(B().fuzzy(L().edits(2)).beam_width(8).case_insensitive(True), words, text, 0.6)


@pytest.mark.parametrize("seed,vocab,filler", [
    (0x1234_5678_9abc_def1, ASCII_VOCAB, ASCII_FILLER),
    (0xdead_beef_0bad_f00d, UNI_VOCAB, UNI_FILLER),
])
def test_staged_prefiltered_matches_oracle(seed, vocab, filler):
    """fac_search_staged_prefiltered (device-resident text) == the oracle's Prefiltered::raw rows."""
    rng = Rng(seed ^ 0x99)
    for _ in range(60):
        b, pats, hay, thr = random_case(rng, vocab, filler, allow_beam=False)
        got, _ = b.build(pats).stage(hay.encode("utf-8")).search_prefiltered(thr)
        want = OracleEngine(b, pats).raw_rows(hay, thr, prefilter=True)
        assert sorted(got) == sorted(want), f"patterns={pats!r} hay={hay!r} thr={thr}"


@pytest.mark.parametrize("budget,width", [(0, 2), (5, 4), (40, 8), (300, 3), (2 ** 64 - 1, 8)])
def test_auto_beam_matches_oracle(budget, width, monkeypatch):
    """auto_beam (search.rs:1096-1103): GPU two-pass (exact counting pass, beamed tail) == the
    oracle's sequential budget, per search_raw call, incl. the pre-filter's per-window calls
    (prefix cache forced on: pass 1 records queue.len() through cached prefixes too)."""
    monkeypatch.setenv("FAC_RC_MIN", "1")
    monkeypatch.setenv("FAC_RC_K", "4")
    rng = Rng(0xab ^ budget)
    for _ in range(40):
        b, pats, hay, thr = random_case(rng, ASCII_VOCAB + UNI_VOCAB, ASCII_FILLER + UNI_FILLER, allow_beam=False)
        b = b.auto_beam(budget, width)
        compare(b, pats, hay, thr)
        compare(b, pats, hay, thr, prefilter=True)


@pytest.mark.parametrize("k", ["2", "3", "4"])
def test_prefix_cache_key_lengths(k, monkeypatch):
    """Every key length of the prefix cache (forced on) == the oracle, beamed and unbeamed, ASCII
    and Unicode, including windows whose key runs past the end of the text."""
    monkeypatch.setenv("FAC_RC_MIN", "1")
    monkeypatch.setenv("FAC_RC_K", k)
    rng = Rng(0x5eed ^ int(k))
    for _ in range(60):
        b, pats, hay, thr = random_case(rng, ASCII_VOCAB + UNI_VOCAB, ASCII_FILLER + UNI_FILLER)
        compare(b, pats, hay, thr)


@pytest.mark.parametrize("k2", ["5", "6", "8"])
def test_prefix_cache_two_levels_c3_slice(k2, monkeypatch):
    """Level-2 snapshots (long prefixes, built by resuming level-1 snapshots) on a C3-shaped
    haystack: identical records with the cache on and off. (Whether the second level replays more
    pops depends on its key threshold and the beam order; only that both levels are used is checked.)"""
    from fuzzy_aho_corasick import workloads
    w = workloads.config("c3", 2 << 20, 3)
    eng = workloads.builder_for(w).build(w.patterns)
    staged = eng.stage(w.haystack)
    monkeypatch.setenv("FAC_RC_MIN2", "1")
    monkeypatch.setenv("FAC_RC_K2", k2)
    on, st_on = staged.search_windows_records(w.threshold)
    monkeypatch.setenv("FAC_RC_K2", "0")
    one, st_one = staged.search_windows_records(w.threshold)
    monkeypatch.setenv("FAC_NO_RC", "1")
    off, _ = staged.search_windows_records(w.threshold)
    assert st_on.states_cached > 0 and st_one.states_cached > 0
    assert len(on) > 0 and sorted(on.tolist()) == sorted(off.tolist()) == sorted(one.tolist())


@pytest.mark.parametrize("knobs", [{}, {"FAC_RC_DEEPEST": "1", "FAC_RC_CT_ENTRIES": "1"},
                                   {"FAC_RC_STRIDE2": "1", "FAC_RC_T2": "3"}, {"FAC_RC_T2": "1"}],
                         ids=["default", "deepest-first", "counts-every-window-thr3", "counts-thr1"])
def test_prefix_cache_round4_paths_c3_slice(knobs, monkeypatch):
    """Round-4 prefix-cache paths on a C3-shaped haystack with the sampled levels on: the default
    (count slots with the count in the key word, 12-state lane rings), the deepest-first probe order
    with entry-sized tables, and the count tables' saturating counts at thresholds 3 (every window
    counted) and 1 (the representative written at the first sighting): identical records to the
    cache off, and the deeper levels replaying pops."""
    from fuzzy_aho_corasick import workloads
    w = workloads.config("c3", 2 << 20, 3)
    staged = workloads.builder_for(w).build(w.patterns).stage(w.haystack)
    monkeypatch.setenv("FAC_RC_MIN2", "1")
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    on, st_on = staged.search_windows_records(w.threshold)
    monkeypatch.setenv("FAC_RC_K2", "0")
    one, st_one = staged.search_windows_records(w.threshold)
    monkeypatch.setenv("FAC_NO_RC", "1")
    off, _ = staged.search_windows_records(w.threshold)
    assert st_on.states_cached > st_one.states_cached > 0
    assert len(on) > 0 and sorted(on.tolist()) == sorted(off.tolist()) == sorted(one.tolist())


def test_prefix_cache_default_on_c3_slice(monkeypatch):
    """A C3-shaped haystack large enough for the default cache (4-char keys): identical records with
    the cache on and off; a slice with the cache forced on == the oracle."""
    from fuzzy_aho_corasick import workloads
    w = workloads.config("c3", 1 << 20, 3)
    eng = workloads.builder_for(w).build(w.patterns)
    staged = eng.stage(w.haystack)
    on, st_on = staged.search_windows_records(w.threshold)
    monkeypatch.setenv("FAC_NO_RC", "1")
    off, _ = staged.search_windows_records(w.threshold)
    assert st_on.states_cached > 0
    assert len(on) > 0 and sorted(on.tolist()) == sorted(off.tolist())
    n = 24 << 10  # oracle on a prefix (whole graphemes: the generator's text is valid UTF-8)
    hay = w.haystack[:n].decode("utf-8", "ignore")
    monkeypatch.delenv("FAC_NO_RC")
    monkeypatch.setenv("FAC_RC_MIN", "1")
    _staged_vs_oracle(workloads.builder_for(w), w.patterns, hay, w.threshold)


def test_dense_start_level_bitmaps(monkeypatch, capfd):
    """The start level's dense key bitmaps (rc_dense_*_kernel: "final without records" and "cached"
    bits over keys of the most frequent ASCII characters) finish most C2 windows without a lookup-table
    probe -- left out of the lookups' window list (dl_*_kernel), or, with the list off, inside the
    lookup: records == both == the bitmaps off (FAC_RC_NO_DENSE) == the cache off, on C2- and C3-shaped
    slices with the sampled level on, and the C2 slice finishes windows through them (FAC_RC_DEBUG)."""
    import re
    from fuzzy_aho_corasick import workloads
    monkeypatch.setenv("FAC_RC_MIN2", "1")
    for cfg, mib in (("c2", 4), ("c3", 2)):
        w = workloads.config(cfg, mib << 20, 3)
        staged = workloads.builder_for(w).build(w.patterns).stage(w.haystack)
        monkeypatch.setenv("FAC_RC_DEBUG", "1")
        capfd.readouterr()
        dense, st = staged.search_windows_records(w.threshold)
        err = capfd.readouterr().err
        monkeypatch.delenv("FAC_RC_DEBUG")
        m = re.findall(r"dense-final (\d+) unlisted (\d+)", err)
        assert m, err[-2000:]
        if cfg == "c2":
            assert int(m[-1][1]) > 0, err[-2000:]
        monkeypatch.setenv("FAC_RC_NO_DENSE_LIST", "1")
        monkeypatch.setenv("FAC_RC_DEBUG", "1")
        capfd.readouterr()
        inloop, _ = staged.search_windows_records(w.threshold)
        err = capfd.readouterr().err
        monkeypatch.delenv("FAC_RC_DEBUG")
        monkeypatch.delenv("FAC_RC_NO_DENSE_LIST")
        m = re.findall(r"dense-final (\d+) unlisted (\d+)", err)
        if cfg == "c2":
            assert m and int(m[-1][0]) > 0 and int(m[-1][1]) == 0, err[-2000:]
        assert sorted(inloop.tolist()) == sorted(dense.tolist()), cfg
        monkeypatch.setenv("FAC_RC_NO_DENSE", "1")
        plain, _ = staged.search_windows_records(w.threshold)
        monkeypatch.delenv("FAC_RC_NO_DENSE")
        monkeypatch.setenv("FAC_NO_RC", "1")
        off, _ = staged.search_windows_records(w.threshold)
        monkeypatch.delenv("FAC_NO_RC")
        assert st.states_cached > 0, cfg
        assert len(dense) > 0 and sorted(dense.tolist()) == sorted(plain.tolist()) == sorted(off.tolist()), cfg


@pytest.mark.parametrize("stride", ["4", "16"])
def test_prefix_cache_sampled_level1(stride, monkeypatch):
    """Level-1 keys counted on every stride-th window (the default from 64 M windows): windows whose
    key the sample missed resume from level 0 or the root; records == every window counted == the
    cache off, on C3- and C2-shaped slices (forced on here with FAC_RC_STRIDE1). The C2 slice also
    samples its single 5-char level sparsely and keeps every sampled key (FAC_RC_STRIDE2, T2 = 1: the
    one-level default from 128 M windows)."""
    from fuzzy_aho_corasick import workloads
    for cfg, mib in (("c3", 2), ("c2", 4)):
        w = workloads.config(cfg, mib << 20, 3)
        staged = workloads.builder_for(w).build(w.patterns).stage(w.haystack)
        monkeypatch.setenv("FAC_RC_STRIDE1", stride)
        if cfg == "c2":
            monkeypatch.setenv("FAC_RC_STRIDE2", stride)
            monkeypatch.setenv("FAC_RC_T2", "1")
        sampled, st = staged.search_windows_records(w.threshold)
        for k in ("FAC_RC_STRIDE2", "FAC_RC_T2"):
            monkeypatch.delenv(k, raising=False)
        monkeypatch.setenv("FAC_RC_STRIDE1", "1")
        full, _ = staged.search_windows_records(w.threshold)
        monkeypatch.setenv("FAC_NO_RC", "1")
        off, _ = staged.search_windows_records(w.threshold)
        monkeypatch.delenv("FAC_NO_RC")
        assert st.states_cached > 0, cfg
        assert len(sampled) > 0 and sorted(sampled.tolist()) == sorted(full.tolist()) == sorted(off.tolist()), cfg


@pytest.mark.parametrize("pops", ["1", "4", "32"])
def test_lane_serial_windows(pops, monkeypatch):
    """lane_window_kernel (small unfinished windows resumed from their snapshots, one lane each, no
    dedup table; windows over the pop budget, the ring, the best list or 2*beam go back to the wave
    kernel) == the wave kernel alone on C3- and C2-shaped slices, and == the oracle on the random
    differential cases with the prefix cache forced on."""
    from fuzzy_aho_corasick import workloads
    monkeypatch.setenv("FAC_LANE_POPS", pops)
    for cfg, mib in (("c3", 2), ("c2", 4)):
        w = workloads.config(cfg, mib << 20, 3)
        staged = workloads.builder_for(w).build(w.patterns).stage(w.haystack)
        on, st_on = staged.search_windows_records(w.threshold)
        monkeypatch.setenv("FAC_NO_LANE", "1")
        off, st_off = staged.search_windows_records(w.threshold)
        monkeypatch.delenv("FAC_NO_LANE")
        assert (st_on.lane_windows > 0 or pops == "1") and st_off.lane_windows == 0, cfg
        assert len(on) > 0 and sorted(on.tolist()) == sorted(off.tolist()), cfg
    monkeypatch.setenv("FAC_RC_MIN", "1")
    for k in ("2", "4"):
        monkeypatch.setenv("FAC_RC_K", k)
        rng = Rng(0x1a2e ^ int(pops) ^ (int(k) << 8))
        for _ in range(60):
            b, pats, hay, thr = random_case(rng, ASCII_VOCAB + UNI_VOCAB, ASCII_FILLER + UNI_FILLER)
            compare(b, pats, hay, thr)


@pytest.mark.parametrize("levels", ["5,6", "6"])
def test_beamed_dedup_free_first_pass(levels, monkeypatch):
    """Beamed main passes run dedup-free (bfs_window_kernel_live, lane_window_kernel) and spill the
    windows that would beam; the snapshots' dedup entries popped before a beam still skip their
    duplicates (jcheck). Records == the exact dedup variant alone, on a C3-shaped slice with sampled
    levels, and == the oracle on random beamed cases with the cache forced on."""
    from fuzzy_aho_corasick import workloads
    w = workloads.config("c3", 4 << 20, 3)
    staged = workloads.builder_for(w).build(w.patterns).stage(w.haystack)
    monkeypatch.setenv("FAC_RC_MIN2", "1")
    monkeypatch.setenv("FAC_RC_LEVELS", levels)
    fast, _ = staged.search_windows_records(w.threshold)
    monkeypatch.setenv("FAC_NO_BEAM_BAIL", "1")
    monkeypatch.setenv("FAC_NO_LANE", "1")
    exact, _ = staged.search_windows_records(w.threshold)
    assert len(fast) > 0 and sorted(fast.tolist()) == sorted(exact.tolist())
    monkeypatch.delenv("FAC_NO_BEAM_BAIL")
    monkeypatch.delenv("FAC_NO_LANE")
    for k, v in (("FAC_RC_MIN", "1"), ("FAC_RC_K", "2"), ("FAC_RC_K2", "4"), ("FAC_RC_STRIDE2", "1"),
                 ("FAC_RC_T2", "1")):
        monkeypatch.setenv(k, v)
    rng = Rng(0xbea3 ^ len(levels))
    n = 0
    while n < 60:
        b, pats, hay, thr = random_case(rng, ASCII_VOCAB + UNI_VOCAB, ASCII_FILLER + UNI_FILLER)
        if b._beam_width:
            compare(b, pats, hay, thr)
            n += 1


def FuzzyMatch_sim_bits(sim):
    import struct
    return struct.unpack("<I", struct.pack("<f", sim))[0]


def _keyrows(ms):
    return [(m.start, m.end, m.pattern_index, m.sim_bits()) for m in ms]


def test_device_apply_matches_host_apply():
    """fac_matches_apply (ranking + overlap resolution on the device, matches.rs:7-149) == the
    oracle's independent C++ restatement (orc_apply) and the host FuzzyMatches.apply, for every
    order x overlap, on random cases and a dense C2 slice. After an overlap resolution the kept
    matches are sorted by start alone (sort_unstable_by_key, ties only between empty spans), so
    those are compared as sets."""
    from fuzzy_aho_corasick import Order, Overlap
    from fuzzy_aho_corasick import workloads
    rng = Rng(0x5151)
    cases = []
    for _ in range(40):
        b, pats, hay, thr = random_case(rng, ASCII_VOCAB + UNI_VOCAB, ASCII_FILLER + UNI_FILLER)
        pats = [Pattern.from_(p) if isinstance(p, str) else p for p in pats]
        if rng.next() % 2:  # custom unique ids shared between patterns (matches.rs:118-122)
            pats = [p.custom_unique_id(rng.next() % 2) if rng.next() % 2 else p for p in pats]
        cases.append((b, pats, hay, thr))
    w = workloads.config("c2", 48 << 10, 7)  # dense: thousands of overlapping candidates
    cases.append((workloads.builder_for(w), w.patterns, w.haystack.decode(), 0.6))
    for b, pats, hay, thr in cases:
        eng = b.build(pats)
        orc = OracleEngine(b, pats)
        for order in Order:
            for overlap in Overlap:
                raw = eng.search_raw(hay, thr)  # one raw list in, every side sees the same order
                rows_in = [(m.start, m.end, m.pattern_index, m.similarity, m.insertions, m.deletions, m.substitutions,
                            m.swaps, m.edits) for m in raw.inner]
                ref = [(r[0], r[1], r[2], FuzzyMatch_sim_bits(r[3])) for r in orc.apply_rows(rows_in, order, overlap)]
                dev = eng.apply_on_device(raw, order, overlap)
                norm = (lambda x: sorted(x)) if overlap != Overlap.Keep else (lambda x: x)  # noqa: E731
                assert norm(_keyrows(dev)) == norm(ref), (order, overlap, hay[:80])
                host = raw.apply(order, overlap)
                assert _keyrows(dev) == _keyrows(host), (order, overlap, hay[:80])
                if order != Order.Unsorted:  # the search path ranks on the device too
                    assert _keyrows(eng._search_ranked(hay, thr, order, overlap)) == _keyrows(host)


def test_device_segmentation_matches_regex():
    """Device UAX #29 staging (stage_kernels.hip) == the regex module's \\X on text with combining
    marks, ZWJ emoji, flags, Hangul, Indic conjuncts, CRLF — incl. runs longer than the 1 KiB
    resync lookback (the sequential path) and chunk boundaries inside multi-byte code points."""
    import ctypes
    import regex
    from fuzzy_aho_corasick import _native
    pieces = ["a", "é", "é", "क्ष", "क्‍ष", "👩‍💻", "🇫🇷", "🇫",
              "\r\n", "\n", "\r", "가", "각", " ", "Ω", "̈", "‍", "ẍ́",
              "ü", "Σ", "؀", "ः", "😀́", "👍🏽", "­", "0", "\t"]
    rng = Rng(0x5e9)
    texts = []
    for _ in range(200):
        texts.append("".join(pieces[rng.next() % len(pieces)] for _ in range(rng.next() % 1500)))
    texts += ["a" + "́" * 3000 + "b" * 700, "🇫" * 2001 + "x", "👩‍" * 900 + "💻",
              "क्" * 1200 + "ष ok", "é" * 5000]
    eng = B().case_insensitive(True).build(["x"])
    for t in texts:
        data = t.encode("utf-8")
        want = []
        pos = 0
        for g in regex.findall(r"\X", t):
            want.append(pos)
            pos += len(g.encode("utf-8"))
        staged = eng.stage(data)
        buf = (ctypes.c_uint64 * (len(data) + 1))()
        n = _native.lib.fac_haystack_grapheme_starts(staged._h, buf, len(data) + 1)
        got = list(buf[:n]) if not data.isascii() else list(range(len(data)))
        assert got == want, t[:60]


def test_stage_device_restaging_matches_regex_and_oracle():
    """fac_haystack_stage_device (search_raw's staging of bytes already in HBM, bench.py's timed
    step): one haystack object restaged over texts of growing and shrinking size -- multi-tile
    Unicode, combining / emoji / RI runs across 16 KiB tile edges, ASCII, empty -- has the regex
    module's \\X grapheme starts and searches like the oracle; invalid UTF-8 is refused."""
    import ctypes
    import numpy as np
    import regex
    import torch
    from fuzzy_aho_corasick import DeviceError, _native
    from fuzzy_aho_corasick.engine import StagedHaystack
    pieces = ["a", "é", "é", "क्ष", "👩‍💻", "🇫🇷", "\r\n", "가", " ", "Ω", "̈", "ẍ́", "Σ", "؀", "😀́",
              "word ", "naïve ", "Москва ", "hello "]
    rng = Rng(0xdec0de)
    texts = []
    for size in (70_000, 300, 40_000, 0, 120_000, 5):
        t = "".join(pieces[rng.next() % len(pieces)] for _ in range(size // 3))
        texts.append(t)
    texts.insert(2, "x" * 16383 + "́" * 40 + "y" * 20000)  # a combining run across a tile edge
    texts.insert(4, "a" + "́" * 20000 + "b" * 100)         # the sequential (hard) path across tiles
    texts.insert(5, "plain ascii hello wolrd " * 2000)
    b = B().fuzzy(L().edits(1)).case_insensitive(True)
    pats = ["hello", "naïve", "москва", "word"]
    eng = b.build(pats)
    orc = OracleEngine(b, pats)
    st = None
    for t in texts:
        data = t.encode("utf-8")
        dev = torch.from_numpy(np.frombuffer(data + b"\0", dtype=np.uint8).copy()).to("cuda")
        st = StagedHaystack.from_device(eng, dev.data_ptr(), len(data), reuse=st)
        want, pos = [], 0
        for g in regex.findall(r"\X", t):
            want.append(pos)
            pos += len(g.encode("utf-8"))
        if data.isascii():
            assert st.graphemes == len(data)
        else:
            buf = (ctypes.c_uint64 * (len(data) + 1))()
            n = _native.lib.fac_haystack_grapheme_starts(st._h, buf, len(data) + 1)
            assert list(buf[:n]) == want, t[:40]
        got = sorted((r[0], r[1], r[2], r[3], r[8]) for r in st.search_windows(0.7)[0])
        exp = sorted((r[0], r[1], r[2], r[3], r[8]) for r in orc.raw_rows(t, 0.7))
        assert got == exp, t[:40]
        del dev
    bad = torch.tensor(list(b"ok \xc3\x28 bad"), dtype=torch.uint8, device="cuda")
    with pytest.raises(DeviceError):
        StagedHaystack.from_device(eng, bad.data_ptr(), bad.numel(), reuse=st)


def _srows(ms):
    import struct
    return [(m.start, m.end, m.pattern_index, struct.unpack("<I", struct.pack("<f", m.similarity))[0], m.text)
            for m in ms]


def test_streaming_apis_match_whole_input():  # tests.rs:1058-1141
    import io
    eng = B().fuzzy(L().edits(1)).case_insensitive(True).build(["needle"])
    filler = "the quick brown fox " * 50
    text = ""
    while len(text) < 600_000:
        text += filler + "needle "
    truth = sorted((m.start, m.end, m.pattern_index)
                   for m in eng.search(text, O().threshold(0.8).sorted().non_overlapping()))
    assert len(truth) > 300
    cb = []
    n = eng.search_stream(io.BytesIO(text.encode()), 0.8, lambda m: cb.append(m))
    assert n == len(text.encode())
    assert sorted((m.start, m.end, m.pattern_index) for m in cb) == truth
    it = list(eng.stream_matches(io.BytesIO(text.encode()), 0.8))
    assert sorted((m.start, m.end, m.pattern_index) for m in it) == truth
    assert all(text.encode()[m.start:m.end].decode() == m.text for m in cb)
    hits = []
    assert B().build(["x"]).search_stream(io.BytesIO(b""), 0.8, hits.append) == 0 and not hits  # :1144-1150


@pytest.mark.parametrize("window", [300, 1024, 4096])
def test_stream_windows_match_oracle_emulation(window):
    """fac_stream (small windows: many cuts, growth, multi-byte boundaries) == the crate's
    WindowReader + per-window search replayed on the CPU oracle."""
    import io
    from stream_emulation import stream_rows
    rng = Rng(0x57 ^ window)
    for _ in range(6):
        b, pats, hay, thr = random_case(rng, ASCII_VOCAB + UNI_VOCAB, ASCII_FILLER + UNI_FILLER, allow_beam=False)
        hay = (hay + " ") * (1 + rng.next() % 40)
        eng = b.build(pats)
        got = _srows(eng.stream_matches(io.BytesIO(hay.encode()), thr, window=window))
        orc = OracleEngine(b, pats)
        want = stream_rows(orc, hay.encode(), thr, eng.max_match_graphemes() + 1, window=window)
        assert got == want, (window, pats, hay[:80])


MAP_RULES = [("æ", "ae"), ("ks", "x"), ("ß", "ss"), ("œ", "oe"), ("ph", "f"), ("c", "k"), ("é", "é"),
             ("ω", "o"), ("ll", "l"), ("AE", "Æ")]
MAP_VOCAB_ASCII = ["encyclopaedia", "alexandr", "strasse", "phone", "cell", "oeuvre", "kafe", "ab"]
MAP_FILLER_ASCII = ["a", "e", "x", "ks", "s", "ph", "f", " ", "k", "c", "l", "oe", "A", "E"]
MAP_VOCAB_UNI = ["encyclopædia", "straße", "cœur", "café", "Ωμέγα", "alexandr", "phone"]
MAP_FILLER_UNI = ["æ", "ae", "ß", "ss", "œ", "é", "é", "ω", "o", " ", "x", "ks", "Æ", "\r\n"]


@pytest.mark.parametrize("seed,vocab,filler", [
    (0x5EED_0001, MAP_VOCAB_ASCII, MAP_FILLER_ASCII),
    (0x5EED_0002, MAP_VOCAB_UNI, MAP_FILLER_UNI),
    (0x5EED_0003, MAP_VOCAB_UNI + MAP_VOCAB_ASCII, MAP_FILLER_UNI + MAP_FILLER_ASCII),
])
def test_mappings_differential(seed, vocab, filler):
    """Multi-character mappings (builder.rs:383-442, search.rs:776-780, 883-922, 945-961): random
    rule sets (scores 1.0 / 0.8 / 0.5), ASCII and Unicode text, every option the hot path has; the
    pre-filter must fall back to the full search (prefilter.rs:162-165)."""
    rng = Rng(seed)
    total = 0
    for i in range(120):
        b, pats, hay, thr = random_case(rng, vocab, filler)
        for _ in range(1 + rng.next() % 3):
            a, c = MAP_RULES[rng.next() % len(MAP_RULES)]
            score = [1.0, 0.8, 0.5][rng.next() % 3]
            b = b.mapping(a, c) if score == 1.0 else b.mapping_scored(a, c, score)
        total += compare(b, pats, hay, thr, prefilter=(i % 5 == 0))
    assert total > 0


def test_mappings_widen_stream_overlap():
    """max_match_graphemes (stream.rs:213-253): longest pattern + max edits x longest mapping side."""
    e = B().fuzzy(L().edits(2)).mapping("x", "kss").build(["alexandr", "ab"])
    assert e.max_match_graphemes() == 8 + 2 * 3
    # a rule that applies nowhere leaves the engine without mappings (self.mappings is empty)
    e2 = B().fuzzy(L().edits(2)).mapping("q", "zzzz").build(["alexandr"])
    assert e2.max_match_graphemes() == 8 + 2
    assert e2.with_prefilter().is_active()


@pytest.mark.parametrize("lds,nmax", [(1, 256), (0, 1024)])
@pytest.mark.parametrize("limit", [16, 1, 0])
def test_device_beam_select_matches_oracle(lds, nmax, limit):
    """The device beam cut alone (beam_select_lds for rings <= 256, beam_select with its global
    scratch for larger ones) on 20 000 beam events each: the bw survivors AND their queue order are
    the oracle's select_nth_unstable_by (oracle.cpp rsel; search.rs:584-587), which
    test_rust_select.py pins to core's post-condition on >= 100 000 arrays."""
    import ctypes
    import numpy as np
    import oracle_harness as OH
    from fuzzy_aho_corasick import _native
    from test_rust_select import _beam_batch, _orc_select_batch

    keys, offs, index = _beam_batch(7000 + 10 * limit + lds, 20000, nmax)
    OH.set_modes(sel_limit=limit)
    try:
        want, bad = _orc_select_batch(keys, offs, index)
    finally:
        OH.set_modes(sel_limit=16)
    assert bad == 0
    for bw in (2, 8, 64):
        sel = np.nonzero(index == bw - 1)[0]
        sub_n = np.diff(offs)[sel]
        sub_offs = np.zeros(len(sel) + 1, np.uint64)
        sub_offs[1:] = np.cumsum(sub_n)
        sub_keys = np.concatenate([keys[int(offs[a]):int(offs[a + 1])] for a in sel])
        perm = np.zeros(len(sel) * bw, np.uint32)
        rc = _native.lib.fac_diag_beam_select(sub_keys.ctypes.data, sub_offs.ctypes.data, len(sel), bw, lds, limit,
                                              perm.ctypes.data)
        assert rc == 0, _native.last_error()
        exp = np.concatenate([want[int(offs[a]):int(offs[a]) + bw] for a in sel])
        diff = np.nonzero(perm != exp)[0]
        assert len(diff) == 0, f"bw={bw}: {len(set(diff // bw))} of {len(sel)} arrays differ (first {diff[0] // bw})"
