"""The reference crate's behaviour pins (src/tests.rs, doctests), translated.

Each test runs twice: on the CPU oracle (`oracle`, checks the restatement against the reference's
own assertions) and on the GPU engine (`gpu`, marked `gpu`). Test names and line numbers follow
/root/reference/src/tests.rs (streaming equivalence lives in test_gpu_parity.py).
"""
import pytest

from fuzzy_aho_corasick import (FuzzyAhoCorasickBuilder as B, FuzzyLimits as L, FuzzyPenalties,
                                Pattern, SearchOptions as O)


def engine_saddam(make_engine):  # tests.rs:8-12
    return make_engine(B().fuzzy(L().edits(2)), ["saddam", "hussein"])


def has(result, pattern=None, text=None):
    return any((pattern is None or m.pattern.as_str() == pattern) and (text is None or m.text == text)
               for m in result)


def test_non_overlapping_regression_0(make_engine):  # tests.rs:15-35
    fac = make_engine(B().fuzzy(L().edits(2)).case_insensitive(True), ["NA", "MENA"])
    r = fac.search("NA MENA", O().threshold(0.6).sorted().non_overlapping())
    assert has(r, "MENA", "MENA")


def test_non_overlapping_regression_2(make_engine):  # tests.rs:37-58
    fac = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["KO", "KO", "LWIN"])
    r = fac.search("KWO KO LWIN", O().threshold(0.6).sorted().non_overlapping())
    assert has(r, "KO", "KWO")


def test_non_overlapping_regression_3(make_engine):  # tests.rs:59-85
    fac = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True),
                      ["AL", "WASEL", "AND", "BABEL", "GENERAL", "TRADING", "LLC"])
    r = fac.search("AL WASL ANT BBEL GNERAL TRATING LC", O().threshold(0.6).sorted().non_overlapping_unique())
    assert has(r, "WASEL", "WASL")
    assert has(r, "BABEL", "BBEL")


def test_case_insensitive_ascii(make_engine):  # tests.rs:87-96
    e = make_engine(B().case_insensitive(True), ["world"])
    r = e.search("HeLlO WoRlD", O().threshold(0.9).sorted())
    assert any(m.text.lower() == "world" for m in r)


def test_unicode_cyrillic(make_engine):  # tests.rs:98-118
    e = make_engine(B().case_insensitive(True), ["юрий"])
    r = e.search("ЮРИЙ ГАГАРИН", O().threshold(0.9).sorted())
    assert any(m.text.lower() == "юрий" for m in r)
    assert e.segment_text("ЮРИЙГАГАРИН", O().threshold(0.9)) == "ЮРИЙ ГАГАРИН"


def test_exact_match(make_engine):  # tests.rs:120-139
    r = engine_saddam(make_engine).search("saddamhussein", O().threshold(0.5).sorted())
    assert has(r, "saddam", "saddam") and has(r, "hussein", "hussein")


def test_extra_letter(make_engine):  # tests.rs:141-155
    r = engine_saddam(make_engine).search("saddammhussein", O().threshold(0.3).sorted())
    assert has(r, "saddam", "saddam")


def test_missing_letter(make_engine):  # tests.rs:157-169
    r = engine_saddam(make_engine).search("saddmhussin", O().threshold(0.3).sorted())
    assert has(r, "saddam", "saddm")


def test_substitution(make_engine):  # tests.rs:171-185
    r = engine_saddam(make_engine).search("saddamhuzein", O().threshold(0.2).sorted())
    assert has(r, "hussein", "huzein")


def test_swap(make_engine):  # tests.rs:187-207
    fac = make_engine(B().fuzzy(L().edits(2)).case_insensitive(True), ["ALI", "KONY"])
    r = fac.search("ALIKOYN", O().threshold(0.6).sorted().non_overlapping())
    assert has(r, "KONY", "KOYN")


LOREM = ("Lorem ipsum dolor sit amet, consectetur adipiscing elit. Vestibulum eros ipsum, tincidutn eu metus ut, "
         "commodo accumsan mi. Vestibulum porta, orci nec ullamcorper posuere, eros tortor pharetra est, at "
         "porttitor mi leo a velit. Aenean sollicitudin mauris elit, ultricies congue dui vulputate in. In hac "
         "habitasse platea dictumst. Nam iaculis sagittis justo a condimentum. Curabitur sed rhoncus dolor. Lorem "
         "ipsum dolor sit amet, consectetur adipiscing elit. Vivamus egestas congue lorem, in convallis magna "
         "viverra quis. Maecenas fringilla mollis arcu quis maximus. Maecenas tincidunt semper vestibulum. Donec "
         "aliquet leo at molestie elementum. Nulla venenatis iaculis gravida. Phasellus at pulvinar odio. Etiam "
         "bibendum tempor purus at dignissim. Nam a turpis ante. Etiam imperdiet justo sit amet quam tristique "
         "porttitor. Cras ultrices tellus et dolor lobortis tempor. Suspendisse eu mi nec nisi sollicitudin "
         "pharetra. Proin imperdiet elementum ullamcorper. Nam imperdiet quis mi at vulputate. Vivamus pulvinar, "
         "quam et tempus sollicitudin, justo dolor venenatis lacus, sit amet dignissim ex quam ut est. Suspendisse "
         "feugiat libero a augue malesuada sagittis. Curabitur vel magna neque. Praesent eu nulla faucibus, egestas "
         "eros sit amet, elementum quam. Fusce porttitor et lacus vitae maximus. Ut viverra eu sem sed lobortis. "
         "Fusce feugiat vestibulum posuere. Integer erat mauris, tempor eu magna vitae, varius rutrum elit. Proin "
         "mattis, nunc at porta commodo, erat urna viverra ante, vitae feugiat velit dolor ac quam. Nulla semper "
         "elit in neque mollis molestie. Aenean a augue scelerisque, tincidunt odio ut, finibus erat. Integer "
         "feugiat eros ac dolor tempus, sed varius lectus ullamcorper. Orci varius natoque penatibus et magnis dis "
         "parturient montes, nascetur ridiculus mus.")


def test_big(make_engine):  # tests.rs:209-228
    fac = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["tincidunt", "porta"])
    r = fac.search(LOREM, O().threshold(0.8).sorted().non_overlapping())
    assert has(r, text="tincidutn") and has(r, text="tincidunt") and has(r, text="porta")


def test_overlap_vs_nonoverlap(make_engine):  # tests.rs:230-293
    e = make_engine(B(), [("saddam", 1.0, 2), ("ddamhu", 1.0, 2)])
    m = e.search("saddamddamhu", O().threshold(0.5).sorted())
    assert has(m, "saddam", "saddam") and has(m, "ddamhu", "ddamhu")
    assert len(e.search("saddamhussein", O().threshold(0.7).sorted().non_overlapping())) == 1
    two = e.search("sadam ddamhu", O().threshold(0.4).sorted().non_overlapping())
    assert len(two) == 2 and has(two, "saddam", "sadam") and has(two, "ddamhu", "ddamhu")


def test_adjustable_penalties(make_engine):  # tests.rs:295-323
    strict = make_engine(B(), [("hussein", 1.0, 2)]).search("huzein", O().threshold(0.3).sorted())
    assert has(strict, "hussein", "huzein")
    pen = FuzzyPenalties.default().with_substitution(0.8).with_insertion(0.95).with_deletion(0.95)
    loose = make_engine(B().penalties(pen), [("hussein", 1.0, 3)]).search("huzein", O().threshold(0.2).sorted())
    assert has(loose, "hussein", "huzein")


def test_regression_1(make_engine):  # tests.rs:325-336
    e = make_engine(B().case_insensitive(True), ["CO"])
    assert len(e.search("CA", O().threshold(0.8).sorted())) == 0


def test_regression_2(make_engine):  # tests.rs:338-354
    e = make_engine(B(), [Pattern("TOLA").fuzzy(L().edits(2))])
    r = e.search("TOL", O().threshold(0.5).sorted().non_overlapping())
    assert has(r, text="TOL")


def test_segment_text(make_engine):  # tests.rs:356-373
    e = make_engine(B().fuzzy(L().edits(3)), ["saddam", "hussein"])
    assert e.segment_text("sadamhusein", O().threshold(0.8)) == "sadam husein"
    assert e.segment_text("sadamhuseinaltikriti", O().threshold(0.8)) == "sadam husein altikriti"


def test_segment_readme(make_engine):  # tests.rs:375-391
    e = make_engine(B().fuzzy(L().edits(1)), ["input", "more"])
    m = e.search("someinptandm0re", O().threshold(0.75).sorted().non_overlapping())
    assert m.segment_text() == "some inpt and m0re"


def test_segment_name(make_engine):  # tests.rs:393-407
    e = make_engine(B().fuzzy(L().edits(3)), ["SHANE", "DOMINIC", "CRAWFORD"])
    assert e.segment_text("SHANEDOM INICCRAWFORD", O().threshold(0.8)) == "SHANE DOM INIC CRAWFORD"


def test_segment_text2(make_engine):  # tests.rs:409-423
    e = make_engine(B().case_insensitive(True), ["HASAN", "JAMAL", "HUSSEIN", "ZEINIYE"])
    assert e.segment_text("ZEINIYEHussEINHASaNJAMAL", O().threshold(0.8)) == "ZEINIYE HussEIN HASaN JAMAL"


def test_fail(make_engine):  # tests.rs:425-434
    e = make_engine(B(), ["saddam", "hussein"])
    assert e.segment_text("sadam husein", O().threshold(0.8)) == "sadam husein"


def test_fuzzy_replace(make_replacer):  # tests.rs:436-450
    r = make_replacer(B().case_insensitive(True), [("PUBLIC JOINT STOCK COMPANY", "PJSC"), ("PUBLIC JOINT STOCK", "PJSC"),
                                                    ("LIMITED LIABILITY COMPANY", "LLC"), ("LIMITED LIABILITY", "LLC")])
    assert r.replace("PUBLIC JOINT STOCK COMPANY GAZPROM", O().threshold(0.8)) == "PJSC GAZPROM"


def test_fuzzy_replace_fn(make_engine):  # tests.rs:452-472
    e = make_engine(B().case_insensitive(True), ["hair", "bear", "wuzzy"])
    out = e.replace("Fuzzy Wuzzy was a hair. Fuzzy Wuzzy had no bear.", O().threshold(0.8),
                    lambda m: {"bear": "hair", "hair": "bear"}.get(m.text))
    assert out == "Fuzzy Wuzzy was a bear. Fuzzy Wuzzy had no hair."


def test_longer_match_preference(make_engine):  # tests.rs:474-492 (output-merge quirk)
    e = make_engine(B(), ["JOINT STOCK COMPANY", "STOCK"])
    r = e.search("JOINT STOCK COMPANY GAZPROM", O().threshold(0.8).sorted().non_overlapping())
    assert has(r, "JOINT STOCK COMPANY")
    assert not has(r, "STOCK")


def test_regression_0(make_engine):  # tests.rs:494-511
    e = make_engine(B().fuzzy(L().edits(2).substitutions(1)).case_insensitive(True), ["zavod"])
    assert e.search("NARODNY", O().threshold(0.8).sorted().non_overlapping()).is_empty()


def test_readme(make_replacer):  # tests.rs:513-524
    r = make_replacer(B().fuzzy(L().substitutions(1)).case_insensitive(True), [("foo", "bar"), ("baz", "qux")])
    assert r.replace("fo0 and BAZ!", O().threshold(0.7)) == "bar and qux!"


def test_country(make_replacer):  # tests.rs:526-537
    r = make_replacer(B().fuzzy(L().edits(5)).case_insensitive(True), [("CZECHOSLOVAKIA", "SERBIA")])
    assert r.replace("CHEKHOSLOVAKIA", O().threshold(0.7)) == "SERBIA"


def test_strip_prefix(make_engine):  # tests.rs:539-550
    e = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["LOREM", "IPSUM"])
    assert e.strip_prefix("LrEM ISuM Lorm ZZZ", O().threshold(0.8)) == "ZZZ"


def test_strip_postfix(make_engine):  # tests.rs:552-563
    e = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["LOREM", "IPSUM"])
    assert e.strip_suffix("ZZZ LrEM ISuM Lorm", O().threshold(0.8)) == "ZZZ"


def test_split(make_engine):  # tests.rs:564-576
    e = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["LOREM", "IPSUM"])
    assert list(e.split("ZZZLrEMISuMAAA", O().threshold(0.8))) == ["ZZZ", "AAA"]


def test_beam_search(make_engine):  # tests.rs:578-626 (beam ties: canonical rule)
    nb = make_engine(B().fuzzy(L().edits(2)).case_insensitive(True), ["saddam", "hussein"])
    wb = make_engine(B().fuzzy(L().edits(2)).case_insensitive(True).beam_width(100), ["saddam", "hussein"])
    o = O().threshold(0.7).sorted().non_overlapping()
    r0, r1 = nb.search("saddamhusein", o), wb.search("saddamhusein", o)
    assert not r0.is_empty() and not r1.is_empty()
    assert has(r1, "saddam")


def test_truncated_walijan(make_engine):  # tests.rs:628-646
    e = make_engine(B().case_insensitive(True), [Pattern("WALIJAN").fuzzy(L().edits(3))])
    assert has(e.search("alijan", O().threshold(0.7).sorted()), "WALIJAN")


def test_truncated_short(make_engine):  # tests.rs:648-665
    e = make_engine(B().case_insensitive(True), [Pattern("TOLA").fuzzy(L().edits(2))])
    assert has(e.search("OLA", O().threshold(0.5).sorted()), text="OLA")


def test_truncated_with_global_limits(make_engine):  # tests.rs:667-684
    e = make_engine(B().case_insensitive(True).fuzzy(L().edits(2)), ["TOLA"])
    assert has(e.search("OLA", O().threshold(0.5).sorted()), text="OLA")


def test_truncated_walijan_with_global_limits(make_engine):  # tests.rs:686-703
    e = make_engine(B().case_insensitive(True).fuzzy(L().edits(3)), ["WALIJAN"])
    assert has(e.search("alijan", O().threshold(0.7).sorted()), "WALIJAN")


def test_phonetic_td_substitution(make_engine):  # tests.rs:705-732
    e = make_engine(B().case_insensitive(True), [Pattern("DJAMEL").fuzzy(L().edits(3))])
    assert has(e.search("Tjamel", O().threshold(0.5).sorted()), "DJAMEL")


def test_missing_middle_char(make_engine):  # tests.rs:734-757
    e = make_engine(B().case_insensitive(True), [Pattern("MOMIR").fuzzy(L().edits(3))])
    assert has(e.search("Mmir", O().threshold(0.5).sorted()), "MOMIR")


def test_aminullah_aminulah(make_engine):  # tests.rs:798-809
    e = make_engine(B().case_insensitive(True), [Pattern("AMINULLAH").fuzzy(L().edits(3))])
    assert not e.search("Aminulah", O().threshold(0.7).sorted()).is_empty()


def test_long_token_no_blowup_regression(make_engine):  # tests.rs:811-864
    lim = L().edits(3).substitutions(1).deletions(2).insertions(2).swaps(0)
    pats = [Pattern(p).fuzzy(lim.clone()) for p in
            ["SA", "LES", "CO", "JSC", "LTD", "BANK", "GROUP", "COMPANY", "CORPORATION", "JOINT STOCK COMPANY",
             "FEDERAL STATE BUDGETARY INSTITUTION OF SCIENCE"]]
    e = make_engine(B().case_insensitive(True), pats)
    import time
    t = time.time()
    r = e.search("RUSSISCHE NATIONALE RUCKVERSICHERUNGSGESELLSCHAFT JSC", O().threshold(0.8).greedy())
    assert time.time() - t < 2.0
    assert has(r, "JSC")


def test_min_symbol_similarity_floor(make_engine):  # tests.rs:1275-1343
    o = O().threshold(0.8).sorted().non_overlapping()
    nf = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["vestibulum"])
    assert len(nf.search("vxstibulum", o)) == 1
    fl = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True).min_symbol_similarity(0.3), ["vestibulum"])
    assert fl.search("vxstibulum", o).is_empty()
    assert len(fl.search("vestibulom", o)) == 1
    assert len(fl.search("vestibulum", o)) == 1


def test_deterministic_search(make_engine):  # tests.rs:1345-1453 (run-to-run equality)
    e = make_engine(B().fuzzy(L().edits(2)).case_insensitive(True), ["hello", "world", "help", "held", "shell", "yellow"])
    for hay in ["hello world", "helo world", "helllo world", "hlelo world", "hwllo world",
                "She sells sea shells by the sea shore", "Why did the yellow bird help the shell?",
                "A quick brown fox jumps over the lazy dog"]:
        for thr in (0.5, 0.7, 0.9):
            for o in (O().threshold(thr), O().threshold(thr).sorted(), O().threshold(thr).greedy(),
                      O().threshold(thr).sorted().non_overlapping()):
                first = [(m.key(), m.sim_bits(), m.edits) for m in e.search(hay, o)]
                if o.order_.name == "Unsorted":
                    first.sort()
                for _ in range(2):
                    nxt = [(m.key(), m.sim_bits(), m.edits) for m in e.search(hay, o)]
                    if o.order_.name == "Unsorted":
                        nxt.sort()
                    assert nxt == first


def test_deterministic_search_unicode(make_engine):  # tests.rs:1500-1583
    e = make_engine(B().fuzzy(L().edits(2)).case_insensitive(True), ["café", "résumé", "naïve", "piñata", "jalapeño"])
    for hay in ["J'aime le café", "Elle a un joli résumé", "Très naïve attitude", "La piñata est colorée",
                "Jalapeño poppers", "Café au lait avec du sucre", "Un café noir et un résumé clair",
                "No matches here at all", "Cafe without accent", "resume without accent"]:
        for thr in (0.5, 0.7, 0.9):
            a = sorted((m.key(), m.sim_bits()) for m in e.search(hay, O().threshold(thr)))
            b = sorted((m.key(), m.sim_bits()) for m in e.search(hay, O().threshold(thr)))
            assert a == b


# ---- doctest value pins
def test_doc_matched_spans(make_engine):  # matches.rs:474-483, 502-510; README.md:55-62
    e = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["HELLO", "WORLD"])
    m = e.search("helllo wolrd", O().threshold(0.8).sorted().non_overlapping())
    assert m.matched_spans() == [(0, 6), (7, 12)]
    assert m.matched_strings() == ["helllo", "wolrd"]
    # known answer: one insertion / one swap on a 5-grapheme pattern = 0.896 (README "0.90")
    import numpy as np
    expect = float(np.float32(np.float32(np.float32(5.0) - np.float32(np.float32(0.4) * np.float32(1.3)))
                              / np.float32(5.0)) * np.float32(1.0))
    assert all(x.similarity == expect for x in m)
    assert abs(expect - 0.8960000277) < 1e-9


def test_doc_builder_segment(make_engine):  # builder.rs:12-21
    e = make_engine(B().case_insensitive(True), ["hello", "world"])
    assert e.segment_text("justheLLowOrLd!", O().threshold(1.0)) == "just heLLo wOrLd!"


def test_doc_greek(make_engine):  # builder.rs:170-180
    e = make_engine(B().case_insensitive(True), [("Γειά", 1.0), ("σου", 1.0)])
    assert not e.search("γειά ΣΟΥ!", O().threshold(0.8).sorted()).is_empty()


def test_doc_query_search(make_engine):  # query.rs:18-28
    e = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["hello", "world"])
    found = [m.pattern.as_str() for m in e.search("helllo wolrd", O().threshold(0.8).non_overlapping())]
    assert "hello" in found and "world" in found


def test_doc_query_replace(make_engine):  # query.rs:76-85
    e = make_engine(B(), ["FOO", "BAR", "BAZ"])
    out = e.replace("FOO BAR BAZ", O().threshold(0.8), lambda m: "###" if m.pattern.pattern == "BAR" else None)
    assert out == "FOO ### BAZ"


def test_doc_query_split(make_engine):  # query.rs:155-165
    e = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["FOO", "BAR"])
    assert list(e.split("xxFo0yyBAARzz", O().threshold(0.8))) == ["xx", "yy", "zz"]


def test_doc_filter_replace(make_engine):  # matches.rs:436-447
    e = make_engine(B().fuzzy(L().edits(1)).case_insensitive(True), ["ipsum", "lorem"])
    m = e.search("ipsum and l0rem", O().threshold(0.5).sorted().non_overlapping())
    assert m.filter(lambda x: "0" in x.text).replace(lambda x: f"**{x.text}**") == "ipsum and **l0rem**"


def test_doc_retain(make_engine):  # matches.rs:405-416
    e = make_engine(B(), ["rust", "rustacean"])
    m = e.search("rustacean and rust", O().threshold(0.8).sorted().non_overlapping())
    m.retain(lambda x: x.pattern_index == 0)
    assert all(x.pattern_index == 0 for x in m)


def test_doc_prefilter(make_engine):  # prefilter.rs:102-111
    e = make_engine(B().fuzzy(L().edits(1)), ["vestibulum", "consectetur"])
    pf = e.with_prefilter()
    o = O().threshold(0.85).sorted()
    assert len(pf.search("lorem vestibulm ipsum", o)) == len(e.search("lorem vestibulm ipsum", o))


def test_prefilter_falls_back_when_not_reducible(make_engine):  # prefilter.rs:548-561 (active half)
    e = make_engine(B().fuzzy(L().edits(1)), ["caesar"])
    assert e.with_prefilter().is_active()


def _mapped(make_engine, edits, rules, patterns):
    b = B().case_insensitive(True).fuzzy(L().edits(edits))
    for r in rules:
        b = b.mapping_scored(*r) if len(r) == 3 else b.mapping(*r)
    return make_engine(b, patterns)


def test_multi_char_mapping_bidirectional(make_engine):  # tests.rs:919-960
    ae = _mapped(make_engine, 1, [("æ", "ae")], ["encyclopaedia"])
    m = ae.search("encyclopædia", O().threshold(0.95).sorted())
    assert len(m) == 1, "æ in the haystack should match the 'ae' pattern"
    assert m[0].substitutions == 1
    assert m[0].similarity > 0.999, "score-1.0 mapping should be penalty-free"
    ea = _mapped(make_engine, 1, [("æ", "ae")], ["encyclopædia"])
    assert len(ea.search("encyclopaedia", O().threshold(0.95).sorted())) == 1


def test_multi_char_mapping_many_to_one(make_engine):  # tests.rs:962-986
    mk = lambda pats: _mapped(make_engine, 1, [("ks", "x")], pats)  # noqa: E731
    assert len(mk(["alexandr"]).search("aleksandr", O().threshold(0.95).sorted())) == 1
    assert len(mk(["aleksandr"]).search("alexandr", O().threshold(0.95).sorted())) == 1


def test_multi_char_mapping_counts_as_edit(make_engine):  # tests.rs:988-1012
    build = lambda edits: _mapped(make_engine, edits, [("ß", "ss")], ["strasse"])  # noqa: E731
    assert len(build(0).search("straße", O().threshold(0.9).sorted())) == 0
    assert len(build(1).search("straße", O().threshold(0.9).sorted())) == 1


def test_multi_char_mapping_scored_penalty(make_engine):  # tests.rs:1014-1039
    exact = _mapped(make_engine, 1, [("ks", "x")], ["alexandr"])
    scored = _mapped(make_engine, 1, [("ks", "x", 0.8)], ["alexandr"])
    se = exact.search("aleksandr", O().threshold(0.5).sorted())[0].similarity
    ss = scored.search("aleksandr", O().threshold(0.5).sorted())[0].similarity
    assert se > 0.999
    assert ss < se


def test_no_mapping_is_unaffected(make_engine):  # tests.rs:1041-1056
    e = make_engine(B().case_insensitive(True).fuzzy(L().edits(1)), ["encyclopaedia"])
    assert len(e.search("encyclopædia", O().threshold(0.9).sorted())) == 0


def _spans_patterns(ms):
    return [(m.start, m.end, m.pattern_index, m.sim_bits()) for m in ms]


def test_auto_beam_exact_below_budget_and_bounded_above(make_engine):  # tests.rs:867-917
    pats = ["saddam", "hussein", "tincidunt", "porta", "vestibulum", "accumsan"]
    text = "this is a saddamhu example with multiple saddam and tincidutn matches"
    b = lambda: B().fuzzy(L().edits(2)).case_insensitive(True)
    opts = O().threshold(0.6).sorted()
    exact = make_engine(b(), pats).search(text, opts)
    huge = make_engine(b().auto_beam(2 ** 64 - 1, 8), pats).search(text, opts)
    assert _spans_patterns(exact) == _spans_patterns(huge)  # never engages: exact
    beamed = make_engine(b().auto_beam(1, 16), pats).search(text, opts)
    assert "saddam" in [pats[m.pattern_index] for m in beamed]


def test_deterministic_search_auto_beam(make_engine):  # tests.rs:1458-1500 (beam-sort path)
    e = make_engine(B().fuzzy(L().edits(4)).auto_beam(100, 500),
                    ["hello", "world", "help", "held", "shell", "yellow", "algorithms", "automaton",
                     "abbreviations"])
    for hay in ["hello world", "helo world", "She sells sea shells by the sea shore",
                "Why did the yellow bird help the shell?", "The quick brown fox jumps over the lazy dog",
                "algorithmic automata and abbreviated forms"]:
        a = _spans_patterns(e.search(hay, O().threshold(0.5).sorted()))
        assert a == _spans_patterns(e.search(hay, O().threshold(0.5).sorted()))
